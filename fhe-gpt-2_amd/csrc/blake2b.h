// BLAKE2b compression and the BLAKE2Xb counter-mode output used by SEAL's default PRNG.
//
// Written from RFC 7693 (BLAKE2b) and the BLAKE2X note (Aumasson et al., 2016): the XOF root
// is a keyed BLAKE2b whose parameter block carries xof_length; output block i is BLAKE2b of the
// 64-byte root with parameter block {digest_length = min(64, left), fanout 0, depth 0,
// leaf_length 64, node_offset i, xof_length, inner_length 64}.  SEAL's Blake2xbPRNG
// (SEAL/randomgen.cpp:185-195, util/blake2xb.c:37-180) refills a 4096-byte buffer with
// blake2xb(out, 4096, &counter, 8, seed, 64) and increments `counter`.
//
// Shared by the host (seal/random.cpp, g++) and the device (csrc/random.hip, hipcc): every
// function is MHE_HD and uses only 64-bit integer arithmetic.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define MHE_HD __host__ __device__ __forceinline__
#else
#define MHE_HD inline
#endif

namespace b2b
{
constexpr uint32_t kPrngBuffer = 4096; // SEAL/randomgen.h:263 buffer_size_

MHE_HD uint64_t iv(int i)
{
    // first 64 bits of the fractional parts of the square roots of the first 8 primes
    switch (i)
    {
    case 0: return 0x6a09e667f3bcc908ULL;
    case 1: return 0xbb67ae8584caa73bULL;
    case 2: return 0x3c6ef372fe94f82bULL;
    case 3: return 0xa54ff53a5f1d36f1ULL;
    case 4: return 0x510e527fade682d1ULL;
    case 5: return 0x9b05688c2b3e6c1fULL;
    case 6: return 0x1f83d9abfb41bd6bULL;
    default: return 0x5be0cd19137e2179ULL;
    }
}

// message word schedule, packed 4 bits per entry (RFC 7693 §2.7); rounds 10 and 11 repeat 0 and 1
MHE_HD int sigma(int round, int k)
{
    const uint64_t rows[10] = {
        0xfedcba9876543210ULL, 0x357b20c16df984aeULL, 0x491763eadf250c8bULL, 0x8f04a562ebcd1397ULL,
        0xd386cb1efa427509ULL, 0x91ef57d438b0a6c2ULL, 0xb8293670a4def15cULL, 0xa2684f05931ce7bdULL,
        0x5a417d2c803b9ef6ULL, 0x0dc3e9bf5167482aULL,
    };
    return (int)((rows[round % 10] >> (4 * k)) & 15);
}

MHE_HD uint64_t rotr(uint64_t x, int r)
{
    return (x >> r) | (x << (64 - r));
}

MHE_HD void mix(uint64_t *v, int a, int b, int c, int d, uint64_t x, uint64_t y)
{
    v[a] = v[a] + v[b] + x;
    v[d] = rotr(v[d] ^ v[a], 32);
    v[c] = v[c] + v[d];
    v[b] = rotr(v[b] ^ v[c], 24);
    v[a] = v[a] + v[b] + y;
    v[d] = rotr(v[d] ^ v[a], 16);
    v[c] = v[c] + v[d];
    v[b] = rotr(v[b] ^ v[c], 63);
}

// F(h, m, t, last): 12 rounds over the 16-word block m (little-endian words)
MHE_HD void compress(uint64_t h[8], const uint64_t m[16], uint64_t t0, uint64_t t1, bool last)
{
    uint64_t v[16];
    for (int i = 0; i < 8; i++)
    {
        v[i] = h[i];
        v[i + 8] = iv(i);
    }
    v[12] ^= t0;
    v[13] ^= t1;
    if (last) v[14] = ~v[14];
    for (int r = 0; r < 12; r++)
    {
        mix(v, 0, 4, 8, 12, m[sigma(r, 0)], m[sigma(r, 1)]);
        mix(v, 1, 5, 9, 13, m[sigma(r, 2)], m[sigma(r, 3)]);
        mix(v, 2, 6, 10, 14, m[sigma(r, 4)], m[sigma(r, 5)]);
        mix(v, 3, 7, 11, 15, m[sigma(r, 6)], m[sigma(r, 7)]);
        mix(v, 0, 5, 10, 15, m[sigma(r, 8)], m[sigma(r, 9)]);
        mix(v, 1, 6, 11, 12, m[sigma(r, 10)], m[sigma(r, 11)]);
        mix(v, 2, 7, 8, 13, m[sigma(r, 12)], m[sigma(r, 13)]);
        mix(v, 3, 4, 9, 14, m[sigma(r, 14)], m[sigma(r, 15)]);
    }
    for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[i + 8];
}

// Parameter block words 0 and 1 (the only non-zero ones here: salt and personal stay zero).
//   word 0: digest_length | key_length << 8 | fanout << 16 | depth << 24 | leaf_length << 32
//   word 1: node_offset | xof_length << 32
//   word 2: node_depth | inner_length << 8
MHE_HD void init_param(uint64_t h[8], uint64_t w0, uint64_t w1, uint64_t w2)
{
    for (int i = 0; i < 8; i++) h[i] = iv(i);
    h[0] ^= w0;
    h[1] ^= w1;
    h[2] ^= w2;
}

// Root of BLAKE2Xb(out_len = xof) keyed with the 64-byte `seed`, message = the 8-byte counter
// (blake2xb_init_key + update(counter) + blake2b_final): the key block is compressed as a
// non-final block, the counter block as the final one (t = 128 + 8).
MHE_HD void xof_root(const uint64_t seed[8], uint64_t counter, uint32_t xof, uint64_t root[8])
{
    init_param(root, 64ULL | (64ULL << 8) | (1ULL << 16) | (1ULL << 24), (uint64_t)xof << 32, 0);
    uint64_t m[16];
    for (int i = 0; i < 16; i++) m[i] = i < 8 ? seed[i] : 0;
    compress(root, m, 128, 0, false);
    m[0] = counter;
    for (int i = 1; i < 16; i++) m[i] = 0;
    compress(root, m, 136, 0, true);
}

// Output block i (64 bytes = 8 words) of the XOF with the given root (blake2xb_final).
MHE_HD void xof_block(const uint64_t root[8], uint32_t i, uint32_t xof, uint32_t block_bytes, uint64_t out[8])
{
    init_param(out, (uint64_t)block_bytes | (64ULL << 32), (uint64_t)i | ((uint64_t)xof << 32), 64ULL << 8);
    uint64_t m[16];
    for (int k = 0; k < 16; k++) m[k] = k < 8 ? root[k] : 0;
    compress(out, m, 64, 0, true);
}
} // namespace b2b
