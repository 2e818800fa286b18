// On-device sampling of the random polynomials of key generation and encryption, bit-identical
// to SEAL's samplers (SEAL/util/rlwe.cpp) fed by SEAL's default PRNG, Blake2xbPRNG
// (SEAL/randomgen.cpp:185-195): the PRNG stream is 4096-byte buffers, buffer c =
// BLAKE2Xb(out 4096, message = u64 counter c, key = the 64-byte seed).  Every 64-byte block of
// the stream is one independent BLAKE2b compression (csrc/blake2b.h), so a sampler that knows
// where its bytes sit in the stream computes them in parallel:
//
//   sample_poly_uniform (rlwe.cpp:136-162): the whole [limbs][n] u64 array is one bulk draw;
//     a word w >= max_multiple(q_l) is redrawn, in index order, from the words after the bulk.
//     The GPU draws the bulk, reduces the accepted words of the limbs the caller keeps and lists
//     the rejected indices (~q/2^64 of them); the host orders that list and assigns the
//     replacement words from the stream tail (mhe_prng_apply_fixes writes them).
//   sample_poly_ternary (rlwe.cpp:21-38): one std::uniform_int_distribution<u64>(0, 2) draw per
//     coefficient over a 32-bit adapter; libstdc++ 11 maps a 32-bit word g to (3g) >> 32
//     (Lemire, bits/uniform_int_dist.h:246-270) and redraws only when g == 0 (probability 2^-32
//     per coefficient): then one thread redoes the poly sequentially and records how many bytes the
//     redraws used, so the samples drawn after it (the CBD errors) start at the right byte -- all
//     on the stream, no host round trip.
//   sample_poly_cbd (rlwe.cpp:101-133): 6 bytes per coefficient, x[2], x[5] masked to 5 bits,
//     noise = pop(x0)+pop(x1)+pop(x2) - pop(x3)-pop(x4)-pop(x5).
// Small samples are written as canonical residues over every requested limb (rand + (flag & q)).
#include <hip/hip_runtime.h>

#include "../../include/mhe.h"
#include "arith.h"
#include "blake2b.h"

int mhe_internal_fail(int code, const char *msg);
int mhe_internal_primes(mhe_ctx *c, const PrimeDev **dev, const uint64_t **host, int *count, int *log_n);

namespace
{
struct Seed
{
    u64 w[8];
};

// limb l of the sampled array -> output limb slot (-1: not kept), max 64 limbs
struct LimbMap
{
    signed char slot[64];
    int prime[64]; // context prime index of limb l
};

// Every 64-byte block of a 4096-byte buffer is one compression of that buffer's XOF root, and a
// root costs two compressions, so a workgroup first computes the roots of the buffers its blocks
// fall in (threads 0 .. nb-1, into LDS) and every block then costs one compression.
constexpr int kMaxRoots = 8;

// roots of buffers [c0, c0 + nb) (nb <= kMaxRoots) into `roots`; a workgroup-wide barrier follows
__device__ __forceinline__ void load_roots(const Seed &s, u64 c0, int nb, u64 (*roots)[8])
{
    if ((int)threadIdx.x < nb)
    {
        u64 r[8];
        b2b::xof_root(s.w, c0 + threadIdx.x, b2b::kPrngBuffer, r);
#pragma unroll
        for (int k = 0; k < 8; k++) roots[threadIdx.x][k] = r[k];
    }
    __syncthreads();
}

// stream block `blk` from the workgroup's roots (buffer blk >> 6 must be in [c0, c0 + nb))
__device__ __forceinline__ void block_from_roots(const u64 (*roots)[8], u64 c0, u64 blk, u64 (&out)[8])
{
    u64 r[8];
#pragma unroll
    for (int k = 0; k < 8; k++) r[k] = roots[(blk >> 6) - c0][k];
    b2b::xof_block(r, (u32)(blk & 63), b2b::kPrngBuffer, 64, out);
}

// 64-byte stream block `blk` (= byte offset / 64) of the PRNG seeded with `s` (root included)
__device__ __forceinline__ void stream_block(const Seed &s, u64 blk, u64 (&out)[8])
{
    u64 root[8];
    b2b::xof_root(s.w, blk >> 6, b2b::kPrngBuffer, root);
    b2b::xof_block(root, (u32)(blk & 63), b2b::kPrngBuffer, 64, out);
}

// Bulk of sample_poly_uniform over `limbs` limbs: one thread per 64-byte block (8 words), a
// workgroup's 256 blocks in 4 buffers.
__global__ __launch_bounds__(256) void k_prng_uniform(Seed s, LimbMap map, u64 *out, const PrimeDev *primes, int limbs,
                                                      int log_n, u64 *rej, u32 *rej_count, u32 rej_cap)
{
    __shared__ u64 roots[kMaxRoots][8];
    const u64 b0 = (u64)blockIdx.x * 256, blk = b0 + threadIdx.x;
    const u64 total = (u64)limbs << log_n;
    const u64 last = ((total / 8 < b0 + 256) ? total / 8 : b0 + 256) - 1;
    load_roots(s, b0 >> 6, (int)((last >> 6) - (b0 >> 6) + 1), roots);
    if (blk * 8 >= total) return;
    u64 w[8];
    block_from_roots(roots, b0 >> 6, blk, w);
#pragma unroll
    for (int k = 0; k < 8; k++)
    {
        const u64 g = blk * 8 + k;
        const int l = (int)(g >> log_n);
        const PrimeDev p = primes[map.prime[l]];
        // max_multiple = (2^64 - 1) - barrett_reduce_64(2^64 - 1, q) - 1 (rlwe.cpp:152)
        const u64 mm = ~0ULL - barrett64(~0ULL, p) - 1;
        if (w[k] >= mm)
        {
            const u32 at = atomicAdd(rej_count, 1u);
            if (at < rej_cap) rej[at] = g;
        }
        else if (map.slot[l] >= 0)
            out[((u64)map.slot[l] << log_n) + (g & (((u64)1 << log_n) - 1))] = barrett64(w[k], p);
    }
}

__global__ void k_prng_apply(const u64 *fix, u32 count, u64 *out)
{
    const u32 i = blockIdx.x * 256 + threadIdx.x;
    if (i < count) out[fix[2 * i]] = fix[2 * i + 1];
}

// sample_poly_ternary: coefficients [0, n) from the stream bytes at byte offset `off` (64-aligned).
// A workgroup owns 256 stream blocks (4096 coefficients): one thread per block draws its 16 values
// into LDS, then the workgroup writes them coalesced to the limbs blockIdx.y, blockIdx.y +
// gridDim.y, ... (every y redraws the same values; the limbs split keeps the grid wide).  A zero word
// would be redrawn (Lemire); those are counted in state[1] (by y == 0) and k_prng_ternary_fix redoes
// the poly sequentially.
__global__ __launch_bounds__(256) void k_prng_ternary(Seed s, u64 off, u64 *out, const PrimeDev *primes, int limbs,
                                                      int log_n, u32 *state)
{
    __shared__ u64 roots[kMaxRoots][8];
    __shared__ unsigned char val[256 * 16];
    const u64 n = (u64)1 << log_n;
    const u64 nblk = n / 16, wb0 = (u64)blockIdx.x * 256;
    const u64 wg_end = (wb0 + 256 < nblk ? wb0 + 256 : nblk);
    const u64 first = (off >> 6) + wb0, last = (off >> 6) + wg_end - 1;
    load_roots(s, first >> 6, (int)((last >> 6) - (first >> 6) + 1), roots);
    if (wb0 + threadIdx.x < wg_end)
    {
        u64 w[8];
        block_from_roots(roots, first >> 6, first + threadIdx.x, w);
#pragma unroll
        for (int k = 0; k < 16; k++)
        {
            const u32 g = (u32)(w[k >> 1] >> (32 * (k & 1)));
            if (g == 0 && blockIdx.y == 0) atomicAdd(&state[1], 1u);
            val[threadIdx.x * 16 + k] = (unsigned char)(((u64)g * 3) >> 32); // {0, 1, 2} -> {-1, 0, 1}
        }
    }
    __syncthreads();
    const u32 cnt = (u32)((wg_end - wb0) * 16);
    for (int l = blockIdx.y; l < limbs; l += gridDim.y)
    {
        const u64 q = primes[l].q;
        u64 *o = out + ((u64)l << log_n) + wb0 * 16;
        for (u32 i = threadIdx.x; i < cnt; i += 256)
        {
            const u32 r = val[i];
            o[i] = r == 0 ? q - 1 : r - 1;
        }
    }
}

// The rare redraw path of sample_poly_ternary (probability ~ n 2^-32 per poly): one thread walks
// the stream 4 bytes at a time, skipping zero words as libstdc++ 11's uniform_int_distribution
// does for a 32-bit URBG (threshold 2^32 mod 3 = 1), and records in state[0] how many bytes the
// redraws consumed, which moves the offsets of the samples drawn after it.
__global__ void k_prng_ternary_fix(Seed s, u64 off, u64 *out, const PrimeDev *primes, int limbs, int log_n,
                                   u32 *state)
{
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    if (state[1] == 0)
    {
        state[0] = 0;
        return;
    }
    const u64 n = (u64)1 << log_n;
    u64 pos = off, cached = ~0ULL, w[8];
    for (u64 i = 0; i < n; i++)
    {
        u32 g;
        do
        {
            const u64 blk = pos >> 6;
            if (blk != cached)
            {
                stream_block(s, blk, w);
                cached = blk;
            }
            g = (u32)(w[(pos & 63) >> 3] >> (32 * ((pos >> 2) & 1)));
            pos += 4;
        } while (g == 0);
        const u64 r = ((u64)g * 3) >> 32;
        for (int l = 0; l < limbs; l++)
        {
            const u64 q = primes[l].q;
            out[((u64)l << log_n) + i] = r == 0 ? q - 1 : r - 1;
        }
    }
    state[0] = (u32)(pos - off - 4 * n);
}

// sample_poly_cbd: coefficients [0, n) from the bytes at offset off + (*extra when given), a
// multiple of 4.  A workgroup owns kCbdCoeffs coefficients (6 bytes each): it computes the roots
// of the <= 3 buffers and the <= 97 stream blocks those bytes span into LDS (one compression per
// block), forms the noise values in LDS, and writes them coalesced to the limbs blockIdx.y,
// blockIdx.y + gridDim.y, ... (as k_prng_ternary).
constexpr int kCbdCoeffs = 1024;
constexpr int kCbdBlocks = (6 * kCbdCoeffs) / 64 + 1;
__global__ __launch_bounds__(256) void k_prng_cbd(Seed s, u64 off, const u32 *extra, u64 *out, const PrimeDev *primes,
                                                  int limbs, int log_n)
{
    __shared__ u64 roots[kMaxRoots][8];
    __shared__ u64 bytes[kCbdBlocks * 8];
    __shared__ signed char noise[kCbdCoeffs];
    const u64 n = (u64)1 << log_n;
    const u64 c0 = (u64)blockIdx.x * kCbdCoeffs;
    const u64 cnt = (n - c0) < (u64)kCbdCoeffs ? (n - c0) : (u64)kCbdCoeffs;
    const u64 start = off + (extra ? extra[0] : 0) + 6 * c0;
    const u64 b0 = start >> 6, b1 = (start + 6 * cnt - 1) >> 6;
    load_roots(s, b0 >> 6, (int)((b1 >> 6) - (b0 >> 6) + 1), roots);
    if (threadIdx.x <= b1 - b0)
    {
        u64 w[8];
        block_from_roots(roots, b0 >> 6, b0 + threadIdx.x, w);
#pragma unroll
        for (int k = 0; k < 8; k++) bytes[threadIdx.x * 8 + k] = w[k];
    }
    __syncthreads();
    const u32 skip = (u32)(start - 64 * b0);
    auto byte_at = [&](u32 i) -> u32 {
        i += skip;
        return (u32)(bytes[i >> 3] >> (8 * (i & 7))) & 0xff;
    };
    for (u32 k = threadIdx.x; k < cnt; k += 256)
    {
        const u32 c = 6 * k;
        noise[k] = (signed char)(__popc(byte_at(c)) + __popc(byte_at(c + 1)) + __popc(byte_at(c + 2) & 0x1f) -
                                 __popc(byte_at(c + 3)) - __popc(byte_at(c + 4)) - __popc(byte_at(c + 5) & 0x1f));
    }
    __syncthreads();
    for (int l = blockIdx.y; l < limbs; l += gridDim.y)
    {
        const u64 q = primes[l].q;
        u64 *o = out + ((u64)l << log_n) + c0;
        for (u32 k = threadIdx.x; k < cnt; k += 256)
        {
            const int v = noise[k];
            o[k] = v >= 0 ? (u64)v : q - (u64)(-v);
        }
    }
}

int launch_check(const char *what)
{
    if (hipGetLastError() != hipSuccess) return mhe_internal_fail(MHE_ERR_DEVICE, what);
    return MHE_OK;
}
} // namespace

#define MHE_EXPORT extern "C" __attribute__((visibility("default")))

MHE_EXPORT int mhe_prng_uniform_bulk(mhe_ctx *c, const uint64_t seed[8], int limbs, const int *prime_of_limb,
                                     const int *slot_of_limb, uint64_t *out, uint64_t *rej, uint32_t *rej_count,
                                     uint32_t rej_cap, void *stream)
{
    const PrimeDev *primes;
    const uint64_t *q;
    int K, log_n;
    if (mhe_internal_primes(c, &primes, &q, &K, &log_n)) return mhe_internal_fail(MHE_ERR_ARG, "context is not valid");
    if (!seed || !prime_of_limb || !slot_of_limb || !out || !rej || !rej_count || limbs < 1 || limbs > 64)
        return mhe_internal_fail(MHE_ERR_ARG, "invalid sampling arguments");
    Seed s;
    LimbMap m;
    for (int i = 0; i < 8; i++) s.w[i] = seed[i];
    for (int l = 0; l < 64; l++)
    {
        m.slot[l] = l < limbs ? (signed char)slot_of_limb[l] : -1;
        m.prime[l] = l < limbs ? prime_of_limb[l] : 0;
        if (l < limbs && (prime_of_limb[l] < 0 || prime_of_limb[l] >= K))
            return mhe_internal_fail(MHE_ERR_ARG, "invalid sampling arguments");
    }
    hipStream_t st = (hipStream_t)stream;
    const u64 blocks = ((u64)limbs << log_n) / 8;
    hipLaunchKernelGGL(k_prng_uniform, dim3((unsigned)((blocks + 255) / 256)), dim3(256), 0, st, s, m, out, primes,
                       limbs, log_n, rej, rej_count, rej_cap);
    return launch_check("uniform sampling kernel launch failed");
}

MHE_EXPORT int mhe_prng_apply_fixes(mhe_ctx *c, const uint64_t *fixes_dev, uint32_t count, uint64_t *out, void *stream)
{
    if (!c || (count && (!fixes_dev || !out))) return mhe_internal_fail(MHE_ERR_ARG, "invalid sampling arguments");
    if (!count) return MHE_OK;
    hipLaunchKernelGGL(k_prng_apply, dim3((count + 255) / 256), dim3(256), 0, (hipStream_t)stream, fixes_dev, count,
                       out);
    return launch_check("sampling fix-up launch failed");
}

MHE_EXPORT int mhe_prng_small(mhe_ctx *c, const uint64_t seed[8], uint64_t byte_offset, int kind, int limbs,
                              uint64_t *out, uint32_t *state_dev, void *stream)
{
    const PrimeDev *primes;
    const uint64_t *q;
    int K, log_n;
    if (mhe_internal_primes(c, &primes, &q, &K, &log_n)) return mhe_internal_fail(MHE_ERR_ARG, "context is not valid");
    if (!seed || !out || limbs < 1 || limbs > K || (byte_offset & 63) || log_n < 5)
        return mhe_internal_fail(MHE_ERR_ARG, "invalid sampling arguments");
    Seed s;
    for (int i = 0; i < 8; i++) s.w[i] = seed[i];
    hipStream_t st = (hipStream_t)stream;
    const u64 n = (u64)1 << log_n;
    if (kind == MHE_SAMPLE_TERNARY)
    {
        if (!state_dev) return mhe_internal_fail(MHE_ERR_ARG, "invalid sampling arguments");
        if (hipMemsetAsync(state_dev, 0, 8, st) != hipSuccess)
            return mhe_internal_fail(MHE_ERR_DEVICE, "sampling state reset failed");
        hipLaunchKernelGGL(k_prng_ternary, dim3((unsigned)((n / 16 + 255) / 256), (unsigned)(limbs < 8 ? limbs : 8)),
                           dim3(256), 0, st, s, byte_offset, out, primes, limbs, log_n, state_dev);
        hipLaunchKernelGGL(k_prng_ternary_fix, dim3(1), dim3(64), 0, st, s, byte_offset, out, primes, limbs, log_n,
                           state_dev);
    }
    else if (kind == MHE_SAMPLE_CBD)
        hipLaunchKernelGGL(k_prng_cbd, dim3((unsigned)((n + kCbdCoeffs - 1) / kCbdCoeffs), (unsigned)(limbs < 4 ? limbs : 4)),
                           dim3(256), 0, st, s, byte_offset, (const u32 *)state_dev, out, primes, limbs, log_n);
    else
        return mhe_internal_fail(MHE_ERR_ARG, "unknown distribution");
    return launch_check("sampling kernel launch failed");
}
