/*
 * seal_random.c -- CPU restatement of SEAL's randomness and key/encryption generation.
 * TEST INFRASTRUCTURE ONLY (included by mhe_oracle.c; see its header).
 *
 * Follows, sequentially and byte for byte (paths relative to
 * seal-modified-3.6.6/native/src/seal/):
 *   util/blake2b.c (BLAKE2b, RFC 7693), util/blake2xb.c:37-180 (BLAKE2Xb),
 *   randomgen.h:200-270 + randomgen.cpp:160-195 (Blake2xbPRNG: 4096-byte buffers, counter),
 *   randomtostd.h (32-bit URBG adapter) and libstdc++ 11's uniform_int_distribution
 *   (bits/uniform_int_dist.h:246-330: Lemire downscaling for a 32-bit URBG),
 *   util/rlwe.cpp:21-162 (sample_poly_ternary / _sparse_ternary / _cbd / _uniform),
 *   util/rlwe.cpp:220-373 (encrypt_zero_asymmetric / encrypt_zero_symmetric, NTT form),
 *   encryptor.cpp:88-166 (asymmetric encryption at the previous level, then divide-and-round),
 *   keygenerator.cpp:62-112,115-149,384-414 (secret key, public key, relinearization and
 *   Galois key-switching keys).
 * Pinning: BLAKE2Xb is checked against Python's hashlib.blake2b (tests/test_seal_random.py).
 */

/* ------------------------------------------------------------------ BLAKE2b (blake2b.c) */
static const uint64_t or_b2_iv[8] = { 0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                      0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                      0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL };
static const uint8_t or_b2_sigma[12][16] = {
    { 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15 }, { 14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3 },
    { 11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4 }, { 7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8 },
    { 9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13 }, { 2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9 },
    { 12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11 }, { 13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10 },
    { 6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5 }, { 10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0 },
    { 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15 }, { 14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3 },
};

typedef struct
{
    uint64_t h[8], t[2], f[2];
    uint8_t buf[128];
    size_t buflen, outlen;
} or_b2_state;

/* the 64-byte parameter block (blake2.h:114-127) */
typedef struct
{
    uint8_t digest_length, key_length, fanout, depth;
    uint32_t leaf_length, node_offset, xof_length;
    uint8_t node_depth, inner_length;
} or_b2_param;

static uint64_t or_load64(const uint8_t *p)
{
    uint64_t v = 0;
    for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
    return v;
}

static uint64_t or_rotr64(uint64_t x, int r) { return (x >> r) | (x << (64 - r)); }

static void or_b2_compress(or_b2_state *S, const uint8_t block[128])
{
    uint64_t m[16], v[16];
    for (int i = 0; i < 16; i++) m[i] = or_load64(block + 8 * i);
    for (int i = 0; i < 8; i++) v[i] = S->h[i];
    for (int i = 0; i < 8; i++) v[8 + i] = or_b2_iv[i];
    v[12] ^= S->t[0];
    v[13] ^= S->t[1];
    v[14] ^= S->f[0];
    v[15] ^= S->f[1];
#define OR_G(r, i, a, b, c, d)                                                                                          \
    do                                                                                                                  \
    {                                                                                                                   \
        a = a + b + m[or_b2_sigma[r][2 * i]];                                                                           \
        d = or_rotr64(d ^ a, 32);                                                                                       \
        c = c + d;                                                                                                      \
        b = or_rotr64(b ^ c, 24);                                                                                       \
        a = a + b + m[or_b2_sigma[r][2 * i + 1]];                                                                       \
        d = or_rotr64(d ^ a, 16);                                                                                       \
        c = c + d;                                                                                                      \
        b = or_rotr64(b ^ c, 63);                                                                                       \
    } while (0)
    for (int r = 0; r < 12; r++)
    {
        OR_G(r, 0, v[0], v[4], v[8], v[12]);
        OR_G(r, 1, v[1], v[5], v[9], v[13]);
        OR_G(r, 2, v[2], v[6], v[10], v[14]);
        OR_G(r, 3, v[3], v[7], v[11], v[15]);
        OR_G(r, 4, v[0], v[5], v[10], v[15]);
        OR_G(r, 5, v[1], v[6], v[11], v[12]);
        OR_G(r, 6, v[2], v[7], v[8], v[13]);
        OR_G(r, 7, v[3], v[4], v[9], v[14]);
    }
#undef OR_G
    for (int i = 0; i < 8; i++) S->h[i] ^= v[i] ^ v[i + 8];
}

static void or_b2_init_param(or_b2_state *S, const or_b2_param *P)
{
    uint8_t pb[64];
    memset(pb, 0, sizeof(pb));
    pb[0] = P->digest_length;
    pb[1] = P->key_length;
    pb[2] = P->fanout;
    pb[3] = P->depth;
    for (int i = 0; i < 4; i++)
    {
        pb[4 + i] = (uint8_t)(P->leaf_length >> (8 * i));
        pb[8 + i] = (uint8_t)(P->node_offset >> (8 * i));
        pb[12 + i] = (uint8_t)(P->xof_length >> (8 * i));
    }
    pb[16] = P->node_depth;
    pb[17] = P->inner_length;
    memset(S, 0, sizeof(*S));
    for (int i = 0; i < 8; i++) S->h[i] = or_b2_iv[i] ^ or_load64(pb + 8 * i);
    S->outlen = P->digest_length;
}

static void or_b2_update(or_b2_state *S, const uint8_t *in, size_t inlen)
{
    /* blake2b_update: the last block is kept for final */
    if (!inlen) return;
    size_t left = S->buflen, fill = 128 - left;
    if (inlen > fill)
    {
        S->buflen = 0;
        memcpy(S->buf + left, in, fill);
        S->t[0] += 128;
        if (S->t[0] < 128) S->t[1]++;
        or_b2_compress(S, S->buf);
        in += fill;
        inlen -= fill;
        while (inlen > 128)
        {
            S->t[0] += 128;
            if (S->t[0] < 128) S->t[1]++;
            or_b2_compress(S, in);
            in += 128;
            inlen -= 128;
        }
    }
    memcpy(S->buf + S->buflen, in, inlen);
    S->buflen += inlen;
}

static void or_b2_final(or_b2_state *S, uint8_t *out, size_t outlen)
{
    S->t[0] += S->buflen;
    if (S->t[0] < S->buflen) S->t[1]++;
    S->f[0] = ~0ULL;
    memset(S->buf + S->buflen, 0, 128 - S->buflen);
    or_b2_compress(S, S->buf);
    uint8_t full[64];
    for (int i = 0; i < 8; i++)
        for (int b = 0; b < 8; b++) full[8 * i + b] = (uint8_t)(S->h[i] >> (8 * b));
    memcpy(out, full, outlen);
}

/* blake2xb (blake2xb.c:143-168 with init_key :37-80 and final :88-141) */
OR_API int or_blake2xb(uint8_t *out, size_t outlen, const uint8_t *in, size_t inlen, const uint8_t *key, size_t keylen)
{
    if (!outlen || outlen > 0xFFFFFFFFUL || keylen > 64) return -1;
    or_b2_state S;
    or_b2_param P = { 64, (uint8_t)keylen, 1, 1, 0, 0, (uint32_t)outlen, 0, 0 };
    or_b2_init_param(&S, &P);
    if (keylen)
    {
        uint8_t block[128];
        memset(block, 0, sizeof(block));
        memcpy(block, key, keylen);
        or_b2_update(&S, block, 128);
    }
    or_b2_update(&S, in, inlen);
    uint8_t root[64];
    or_b2_final(&S, root, 64);
    or_b2_param C = P;
    C.key_length = 0;
    C.fanout = 0;
    C.depth = 0;
    C.leaf_length = 64;
    C.inner_length = 64;
    C.node_depth = 0;
    for (size_t i = 0; outlen > 0; i++)
    {
        const size_t block_size = outlen < 64 ? outlen : 64;
        C.digest_length = (uint8_t)block_size;
        C.node_offset = (uint32_t)i;
        or_b2_state T;
        or_b2_init_param(&T, &C);
        or_b2_update(&T, root, 64);
        or_b2_final(&T, out + i * 64, block_size);
        outlen -= block_size;
    }
    return 0;
}

/* ------------------------------------------------------------------ Blake2xbPRNG */
typedef struct
{
    uint8_t seed[64];
    uint8_t buf[4096];
    size_t head;
    uint64_t counter;
} or_prng;

static void or_prng_init(or_prng *g, const uint64_t seed[8])
{
    for (int i = 0; i < 8; i++)
        for (int b = 0; b < 8; b++) g->seed[8 * i + b] = (uint8_t)(seed[i] >> (8 * b));
    g->head = 4096; /* buffer_head_ = buffer_end_ */
    g->counter = 0;
}

static void or_prng_refill(or_prng *g)
{
    uint8_t ctr[8];
    for (int b = 0; b < 8; b++) ctr[b] = (uint8_t)(g->counter >> (8 * b));
    or_blake2xb(g->buf, 4096, ctr, 8, g->seed, 64);
    g->counter++;
}

static void or_prng_generate(or_prng *g, size_t count, uint8_t *dst)
{
    while (count)
    {
        size_t cur = 4096 - g->head;
        if (cur > count) cur = count;
        memcpy(dst, g->buf + g->head, cur);
        g->head += cur;
        dst += cur;
        count -= cur;
        if (g->head == 4096)
        {
            or_prng_refill(g);
            g->head = 0;
        }
    }
}

static uint32_t or_prng_u32(or_prng *g)
{
    uint8_t b[4];
    or_prng_generate(g, 4, b);
    return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
}

/* std::uniform_int_distribution<uint64_t>(a, b)(RandomToStandardAdapter) in libstdc++ 11:
 * range < 2^32 -> _S_nd<uint64_t>(urng, uint32 range + 1) (Lemire) */
static uint64_t or_uniform_int(or_prng *g, uint64_t a, uint64_t b)
{
    const uint32_t erange = (uint32_t)(b - a + 1);
    uint64_t product = (uint64_t)or_prng_u32(g) * erange;
    uint32_t low = (uint32_t)product;
    if (low < erange)
    {
        const uint32_t threshold = (uint32_t)(-erange) % erange;
        while (low < threshold)
        {
            product = (uint64_t)or_prng_u32(g) * erange;
            low = (uint32_t)product;
        }
    }
    return (product >> 32) + a;
}

OR_API void or_prng_bytes(const uint64_t seed[8], size_t count, uint8_t *out)
{
    or_prng g;
    or_prng_init(&g, seed);
    or_prng_generate(&g, count, out);
}

/* ------------------------------------------------------------------ samplers (rlwe.cpp) */
static void or_put_small(int64_t v, const or_ctx *c, int limbs, size_t i, uint64_t *out)
{
    for (int l = 0; l < limbs; l++)
    {
        const uint64_t q = c->mod[l].value;
        out[(size_t)l * c->n + i] = v >= 0 ? (uint64_t)v : q - (uint64_t)(-v);
    }
}

static void or_sample_ternary(or_prng *g, const or_ctx *c, int limbs, uint64_t *out)
{
    for (size_t i = 0; i < c->n; i++) or_put_small((int64_t)or_uniform_int(g, 0, 2) - 1, c, limbs, i, out);
}

static void or_sample_sparse_ternary(or_prng *g, const or_ctx *c, int limbs, size_t hw, uint64_t *out)
{
    const size_t n = c->n, total = (size_t)limbs * n;
    memset(out, 0, total * 8);
    (void)total;
    size_t w = 0;
    while (w < hw)
    {
        /* inclusive range: n can be drawn.  SEAL then writes coefficient 0 of limbs 1.. with the
         * previous prime's residue (and one word past the array), which is not a ring element;
         * the engine redraws it (seal/random.cpp), and so does this restatement */
        const size_t index = (size_t)or_uniform_int(g, 0, n);
        if (index >= n || out[index] != 0) continue;
        const uint64_t r = 2 * or_uniform_int(g, 0, 1);
        for (int j = 0; j < limbs; j++) out[index + (size_t)j * n] = r == 0 ? c->mod[j].value - 1 : r - 1;
        w++;
    }
}

static void or_sample_cbd(or_prng *g, const or_ctx *c, int limbs, uint64_t *out)
{
    for (size_t i = 0; i < c->n; i++)
    {
        uint8_t x[6];
        or_prng_generate(g, 6, x);
        x[2] &= 0x1F;
        x[5] &= 0x1F;
        const int noise = __builtin_popcount(x[0]) + __builtin_popcount(x[1]) + __builtin_popcount(x[2]) -
                          __builtin_popcount(x[3]) - __builtin_popcount(x[4]) - __builtin_popcount(x[5]);
        or_put_small(noise, c, limbs, i, out);
    }
}

/* sample_poly_uniform over limbs 0..limbs-1 of the context */
static void or_sample_uniform(or_prng *g, const or_ctx *c, int limbs, uint64_t *out)
{
    const size_t n = c->n;
    or_prng_generate(g, (size_t)limbs * n * 8, (uint8_t *)out); /* little-endian host */
    for (int j = 0; j < limbs; j++)
    {
        const uint64_t q = c->mod[j].value;
        const uint64_t max_multiple = ~0ULL - or_barrett64(~0ULL, &c->mod[j]) - 1;
        for (size_t i = 0; i < n; i++)
        {
            uint64_t r = out[(size_t)j * n + i];
            while (r >= max_multiple) or_prng_generate(g, 8, (uint8_t *)&r);
            out[(size_t)j * n + i] = or_barrett64(r, &c->mod[j]);
        }
        (void)q;
    }
}

/* kind: 0 uniform, 1 ternary, 2 sparse ternary (hw), 3 cbd; output [limbs][n] */
OR_API void or_ctx_sample(const or_ctx *c, const uint64_t seed[8], int kind, int limbs, size_t hw, uint64_t *out)
{
    or_prng g;
    or_prng_init(&g, seed);
    switch (kind)
    {
    case 0: or_sample_uniform(&g, c, limbs, out); break;
    case 1: or_sample_ternary(&g, c, limbs, out); break;
    case 2: or_sample_sparse_ternary(&g, c, limbs, hw, out); break;
    default: or_sample_cbd(&g, c, limbs, out); break;
    }
}

/* ------------------------------------------------------------------ encryption / keys */
/* encrypt_zero_symmetric (rlwe.cpp:289-373), NTT form, no seed saved, at `limbs` limbs.
 * sk: NTT form over at least `limbs` limbs (first limbs used). out: [2][limbs][n]. */
OR_API void or_ctx_encrypt_zero_symmetric(const or_ctx *c, const uint64_t seed[8], const uint64_t *sk, int limbs,
                                          uint64_t *out)
{
    const size_t n = c->n, ps = (size_t)limbs * n;
    or_prng boot;
    or_prng_init(&boot, seed);
    uint64_t pub[8];
    or_prng_generate(&boot, 64, (uint8_t *)pub);
    or_prng cg;
    or_prng_init(&cg, pub);
    uint64_t *c0 = out, *c1 = out + ps;
    or_sample_uniform(&cg, c, limbs, c1);
    uint64_t *noise = (uint64_t *)malloc(ps * 8);
    or_sample_cbd(&boot, c, limbs, noise);
    or_ctx_dyadic(c, sk, c1, c0, limbs);
    or_ctx_ntt(c, noise, 1, limbs, 0);
    or_ctx_addsub(c, noise, c0, c0, 1, limbs, 0);
    or_ctx_addsub(c, c0, NULL, c0, 1, limbs, 2);
    free(noise);
}

/* encrypt_zero_asymmetric (rlwe.cpp:220-286) at m limbs with pk [2][K][n] (first m limbs),
 * then, when m > L, divide_and_round_q_last_ntt_inplace per poly (encryptor.cpp:120-140).
 * out: [2][L][n]; L = m or m - 1. */
OR_API void or_ctx_encrypt_zero_asymmetric(const or_ctx *c, const uint64_t seed[8], const uint64_t *pk, int m,
                                           int L, uint64_t *out)
{
    const size_t n = c->n, ps = (size_t)m * n, K = (size_t)c->k;
    or_prng g;
    or_prng_init(&g, seed);
    uint64_t *u = (uint64_t *)malloc(ps * 8), *e = (uint64_t *)malloc(ps * 8), *ct = (uint64_t *)malloc(2 * ps * 8);
    or_sample_ternary(&g, c, m, u);
    or_ctx_ntt(c, u, 1, m, 0);
    for (int j = 0; j < 2; j++) or_ctx_dyadic(c, u, pk + (size_t)j * K * n, ct + (size_t)j * ps, m);
    for (int j = 0; j < 2; j++)
    {
        or_sample_cbd(&g, c, m, e);
        or_ctx_ntt(c, e, 1, m, 0);
        or_ctx_addsub(c, e, ct + (size_t)j * ps, ct + (size_t)j * ps, 1, m, 0);
    }
    if (L == m)
        memcpy(out, ct, 2 * ps * 8);
    else
        or_ctx_rescale(c, ct, out, 2, m);
    free(u);
    free(e);
    free(ct);
}

/* KeyGenerator secret key (keygenerator.cpp:62-84): sparse ternary (hw > 0) or ternary over the
 * key level, NTT form.  out: [K][n]. */
OR_API void or_ctx_keygen_secret(const or_ctx *c, const uint64_t seed[8], size_t hw, uint64_t *out)
{
    or_prng g;
    or_prng_init(&g, seed);
    if (hw)
        or_sample_sparse_ternary(&g, c, c->k, hw, out);
    else
        or_sample_ternary(&g, c, c->k, out);
    or_ctx_ntt(c, out, 1, c->k, 0);
}

/* generate_one_kswitch_key (keygenerator.cpp:384-414) with a seeded factory: every digit's
 * encrypt_zero_symmetric draws its bootstrap PRNG from the same seed.  new_key: [K][n] NTT;
 * out: [K-1][2][K][n]. */
OR_API void or_ctx_kswitch_key(const or_ctx *c, const uint64_t seed[8], const uint64_t *sk, const uint64_t *new_key,
                               uint64_t *out)
{
    const size_t n = c->n, K = (size_t)c->k;
    for (size_t j = 0; j + 1 < K; j++)
    {
        uint64_t *d = out + j * 2 * K * n;
        or_ctx_encrypt_zero_symmetric(c, seed, sk, (int)K, d);
        const uint64_t factor = or_barrett64(c->mod[K - 1].value, &c->mod[j]);
        for (size_t i = 0; i < n; i++)
        {
            const uint64_t t = or_mulmod(new_key[j * n + i], factor, &c->mod[j]);
            uint64_t r = d[j * n + i] + t;
            d[j * n + i] = r >= c->mod[j].value ? r - c->mod[j].value : r;
        }
    }
}
