/*
 * mhe_oracle.c -- CPU restatement of the reference's RNS-CKKS evaluator hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP engine in
 * fhe-gpt-2_amd/csrc.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it; the product path never links or calls it.
 *
 * It restates, function by function, the modified Microsoft SEAL 3.6.6 shipped in the
 * reference (paths below are relative to
 * /root/reference/cnn_ckks/cpu-ckks/single-key/seal-modified-3.6.6/native/src/seal/).
 * Every function cites the file:line it follows.  The algorithms are re-written from
 * reading the reference, not copied; the loop structure (lazy ranges, reduction points)
 * is kept so that lazy intermediate values match SEAL's bit for bit where that matters.
 *
 * Pinning (see DESIGN.md "Oracle"): the reference SEAL cannot be built here without its
 * CMake-generated config.h and the absent GSL/zstd headers, so oracle/_ref is not built.
 * This restatement is pinned instead by the reference's own known-answer tests
 * (native/tests/seal/util/{ntt,galois,rns,uintarithsmallmod,numth}.cpp), replayed in
 * tests/test_oracle_kat.py from the fixtures in tests/golden/.
 */
#define _GNU_SOURCE /* sincos */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

typedef unsigned __int128 u128;

#define OR_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------------------------
 * Modulus + primitives
 * ------------------------------------------------------------------------------------------ */

/* Modulus::set_value const_ratio = floor(2^128 / q) (modulus.cpp:66-98). */
typedef struct
{
    uint64_t value;
    uint64_t ratio0, ratio1; /* low / high words of floor(2^128/q) */
} or_mod;

static void or_mod_init(or_mod *m, uint64_t q)
{
    m->value = q;
    /* floor(2^128 / q) = floor((2^128 - 1) / q) unless q divides 2^128 (q a power of two). */
    u128 r = (~(u128)0) / q;
    if ((q & (q - 1)) == 0) r += 1;
    m->ratio0 = (uint64_t)r;
    m->ratio1 = (uint64_t)(r >> 64);
}

/* barrett_reduce_128 (util/uintarithsmallmod.h:166-200). */
static inline uint64_t or_barrett128(uint64_t in0, uint64_t in1, const or_mod *m)
{
    uint64_t carry = (uint64_t)(((u128)in0 * m->ratio0) >> 64);
    u128 t2 = (u128)in0 * m->ratio1;
    uint64_t tmp1 = (uint64_t)t2 + carry;
    uint64_t tmp3 = (uint64_t)(t2 >> 64) + (tmp1 < carry);
    t2 = (u128)in1 * m->ratio0;
    uint64_t lo = (uint64_t)t2;
    uint64_t s = tmp1 + lo;
    carry = (uint64_t)(t2 >> 64) + (s < lo);
    tmp1 = in1 * m->ratio1 + tmp3 + carry;
    tmp3 = in0 - tmp1 * m->value;
    return tmp3 >= m->value ? tmp3 - m->value : tmp3;
}

/* barrett_reduce_64 (util/uintarithsmallmod.h:206-224). */
static inline uint64_t or_barrett64(uint64_t x, const or_mod *m)
{
    uint64_t hi = (uint64_t)(((u128)x * m->ratio1) >> 64);
    uint64_t t = x - hi * m->value;
    return t >= m->value ? t - m->value : t;
}

/* multiply_uint_mod(a, b) (util/uintarithsmallmod.h:230-242). */
static inline uint64_t or_mulmod(uint64_t a, uint64_t b, const or_mod *m)
{
    u128 z = (u128)a * b;
    return or_barrett128((uint64_t)z, (uint64_t)(z >> 64), m);
}

/* MultiplyUIntModOperand (util/uintarithsmallmod.h:249-279): quotient = floor(w * 2^64 / q). */
typedef struct
{
    uint64_t operand, quotient;
} or_shoup;

static inline or_shoup or_shoup_make(uint64_t w, uint64_t q)
{
    or_shoup s;
    s.operand = w;
    s.quotient = (uint64_t)(((u128)w << 64) / q);
    return s;
}

/* multiply_uint_mod(x, MultiplyUIntModOperand) (util/uintarithsmallmod.h:286-299). */
static inline uint64_t or_mulmod_shoup(uint64_t x, or_shoup y, uint64_t p)
{
    uint64_t hi = (uint64_t)(((u128)x * y.quotient) >> 64);
    uint64_t t = y.operand * x - hi * p;
    return t >= p ? t - p : t;
}

/* multiply_uint_mod_lazy (util/uintarithsmallmod.h:306-318): result in [0, 2p). */
static inline uint64_t or_mulmod_shoup_lazy(uint64_t x, or_shoup y, uint64_t p)
{
    uint64_t hi = (uint64_t)(((u128)x * y.quotient) >> 64);
    return y.operand * x - hi * p;
}

static uint64_t or_powmod(uint64_t base, uint64_t e, const or_mod *m)
{
    uint64_t r = 1 % m->value;
    base = or_barrett64(base, m);
    while (e)
    {
        if (e & 1) r = or_mulmod(r, base, m);
        base = or_mulmod(base, base, m);
        e >>= 1;
    }
    return r;
}

/* try_invert_uint_mod via xgcd (util/numth.h:78-145). Returns 0 if not invertible. */
static int or_invmod(uint64_t a, uint64_t q, uint64_t *res)
{
    uint64_t r0 = q, r1 = a % q;
    if (r1 == 0) return 0;
    /* extended Euclid with signed Bezout coefficients (|s| < q < 2^62 fits) */
    __int128 s0 = 0, s1 = 1;
    while (r1 != 0)
    {
        uint64_t qt = r0 / r1;
        uint64_t r2 = r0 - qt * r1;
        __int128 s2 = s0 - (__int128)qt * s1;
        r0 = r1;
        r1 = r2;
        s0 = s1;
        s1 = s2;
    }
    if (r0 != 1) return 0;
    __int128 v = s0 % (__int128)q;
    if (v < 0) v += q;
    *res = (uint64_t)v;
    return 1;
}

static uint32_t or_reverse_bits(uint32_t x, int bits)
{
    uint32_t r = 0;
    for (int i = 0; i < bits; i++)
    {
        r = (r << 1) | (x & 1);
        x >>= 1;
    }
    return r;
}

/* ------------------------------------------------------------------------------------------
 * Prime selection (util/numth.cpp:179-317, modulus.cpp:143-185)
 * ------------------------------------------------------------------------------------------ */

/* is_prime (util/numth.cpp:179-277).  SEAL runs 40 Miller-Rabin rounds with random bases;
 * for 64-bit inputs the fixed base set below is deterministic and decides identically. */
OR_API int or_is_prime(uint64_t value)
{
    if (value < 2) return 0;
    static const uint64_t small[] = { 2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37 };
    for (int i = 0; i < 12; i++)
    {
        if (value == small[i]) return 1;
        if (value % small[i] == 0) return 0;
    }
    or_mod m;
    or_mod_init(&m, value);
    uint64_t d = value - 1;
    int r = 0;
    while (!(d & 1))
    {
        d >>= 1;
        r++;
    }
    for (int i = 0; i < 12; i++)
    {
        uint64_t x = or_powmod(small[i], d, &m);
        if (x == 1 || x == value - 1) continue;
        int cont = 0;
        for (int c = 0; c < r - 1; c++)
        {
            x = or_mulmod(x, x, &m);
            if (x == value - 1)
            {
                cont = 1;
                break;
            }
        }
        if (!cont) return 0;
    }
    return 1;
}

/* get_primes (util/numth.cpp:279-317): scan 2^bits - 2n + 1 downwards in steps of 2n,
 * output in descending order.  Returns number found. */
OR_API int or_get_primes(uint64_t ntt_size, int bit_size, int count, uint64_t *out)
{
    uint64_t factor = 2 * ntt_size;
    uint64_t value = (((uint64_t)1) << bit_size) - factor + 1;
    uint64_t lower = ((uint64_t)1) << (bit_size - 1);
    int found = 0;
    while (found < count && value > lower)
    {
        if (or_is_prime(value)) out[found++] = value;
        value -= factor;
    }
    return found;
}

/* CoeffModulus::Create (modulus.cpp:143-185): for every bit size the primes are generated
 * descending and handed out from the back (smallest first). */
OR_API int or_coeff_modulus_create(uint64_t n, const int *bit_sizes, int count, uint64_t *out)
{
    int cursor[64] = { 0 };
    int total[64] = { 0 };
    uint64_t *tables[64] = { 0 };
    for (int i = 0; i < count; i++)
    {
        if (bit_sizes[i] < 2 || bit_sizes[i] > 60) return -1;
        total[bit_sizes[i]]++;
    }
    for (int b = 0; b < 64; b++)
    {
        if (!total[b]) continue;
        tables[b] = (uint64_t *)malloc(sizeof(uint64_t) * total[b]);
        if (or_get_primes(n, b, total[b], tables[b]) != total[b])
        {
            for (int c = 0; c <= b; c++) free(tables[c]);
            return -2;
        }
        cursor[b] = total[b];
    }
    for (int i = 0; i < count; i++)
    {
        int b = bit_sizes[i];
        out[i] = tables[b][--cursor[b]];
    }
    for (int b = 0; b < 64; b++) free(tables[b]);
    return 0;
}

/* try_minimal_primitive_root (util/numth.cpp:352-424): the smallest primitive degree-th root.
 * SEAL starts from a random primitive root g and scans g^(2i+1); the minimum over all odd
 * powers is the same whatever g it started from, so a deterministic start is used here. */
OR_API uint64_t or_minimal_primitive_root(uint64_t degree, uint64_t q)
{
    or_mod m;
    or_mod_init(&m, q);
    uint64_t quotient = (q - 1) / degree;
    if (quotient * degree != q - 1) return 0;
    uint64_t root = 0;
    for (uint64_t cand = 2; cand < q; cand++)
    {
        uint64_t g = or_powmod(cand, quotient, &m);
        /* is_primitive_root (util/numth.cpp:325-350): g^(degree/2) == -1 */
        if (g != 0 && or_powmod(g, degree >> 1, &m) == q - 1)
        {
            root = g;
            break;
        }
    }
    if (!root) return 0;
    uint64_t gsq = or_mulmod(root, root, &m);
    uint64_t cur = root, best = root;
    for (uint64_t i = 0; i < degree; i++)
    {
        if (cur < best) best = cur;
        cur = or_mulmod(cur, gsq, &m);
    }
    return best;
}

/* ------------------------------------------------------------------------------------------
 * NTT tables + Harvey NTT (util/ntt.cpp:30-89,183-209; util/ntt.h:24-71,235-296,336-358;
 * util/dwthandler.h:94-356)
 * ------------------------------------------------------------------------------------------ */

typedef struct
{
    int log_n;
    size_t n;
    or_mod mod;
    uint64_t root, inv_root;
    or_shoup *root_powers;     /* bit-reversed powers of psi, [0] = 1 */
    or_shoup *inv_root_powers; /* scrambled powers of psi^-1: slot rev(i-1)+1 holds psi^-i */
    or_shoup inv_degree;
} or_ntt_tables;

/* NTTTables::initialize (util/ntt.cpp:30-89). */
static int or_ntt_tables_init(or_ntt_tables *t, int log_n, uint64_t q)
{
    t->log_n = log_n;
    t->n = (size_t)1 << log_n;
    or_mod_init(&t->mod, q);
    t->root = or_minimal_primitive_root(2 * t->n, q);
    if (!t->root) return -1;
    if (!or_invmod(t->root, q, &t->inv_root)) return -1;
    t->root_powers = (or_shoup *)malloc(sizeof(or_shoup) * t->n);
    t->inv_root_powers = (or_shoup *)malloc(sizeof(or_shoup) * t->n);
    uint64_t power = t->root;
    for (size_t i = 1; i < t->n; i++)
    {
        t->root_powers[or_reverse_bits((uint32_t)i, log_n)] = or_shoup_make(power, q);
        power = or_mulmod(power, t->root, &t->mod);
    }
    t->root_powers[0] = or_shoup_make(1, q);
    power = t->inv_root;
    for (size_t i = 1; i < t->n; i++)
    {
        t->inv_root_powers[or_reverse_bits((uint32_t)(i - 1), log_n) + 1] = or_shoup_make(power, q);
        power = or_mulmod(power, t->inv_root, &t->mod);
    }
    t->inv_root_powers[0] = or_shoup_make(1, q);
    uint64_t invn;
    if (!or_invmod((uint64_t)t->n, q, &invn)) return -1;
    t->inv_degree = or_shoup_make(invn, q);
    return 0;
}

static void or_ntt_tables_free(or_ntt_tables *t)
{
    free(t->root_powers);
    free(t->inv_root_powers);
    t->root_powers = t->inv_root_powers = NULL;
}

/* DWTHandler::transform_to_rev with Arithmetic<u64, MultiplyUIntModOperand> (dwthandler.h:94-191,
 * ntt.h:24-71): Cooley-Tukey, inputs in [0,4q), outputs in [0,4q), bit-reversed order. */
static void or_ntt_fwd_lazy(uint64_t *values, const or_ntt_tables *t)
{
    const uint64_t q = t->mod.value, two_q = q << 1;
    const or_shoup *roots = t->root_powers;
    size_t n = t->n, gap = n >> 1, m = 1;
    for (; m < (n >> 1); m <<= 1)
    {
        size_t offset = 0;
        for (size_t i = 0; i < m; i++)
        {
            or_shoup r = *++roots;
            uint64_t *x = values + offset, *y = x + gap;
            for (size_t j = 0; j < gap; j++)
            {
                uint64_t u = *x >= two_q ? *x - two_q : *x; /* guard */
                uint64_t v = or_mulmod_shoup_lazy(*y, r, q);
                *x++ = u + v;
                *y++ = u + two_q - v;
            }
            offset += gap << 1;
        }
        gap >>= 1;
    }
    for (size_t i = 0; i < m; i++)
    {
        or_shoup r = *++roots;
        uint64_t u = values[0] >= two_q ? values[0] - two_q : values[0];
        uint64_t v = or_mulmod_shoup_lazy(values[1], r, q);
        values[0] = u + v;
        values[1] = u + two_q - v;
        values += 2;
    }
}

/* ntt_negacyclic_harvey (util/ntt.h:235-264): lazy NTT then reduce [0,4q) -> [0,q). */
static void or_ntt_fwd(uint64_t *values, const or_ntt_tables *t)
{
    or_ntt_fwd_lazy(values, t);
    const uint64_t q = t->mod.value, two_q = q << 1;
    for (size_t i = 0; i < t->n; i++)
    {
        uint64_t v = values[i];
        if (v >= two_q) v -= two_q;
        if (v >= q) v -= q;
        values[i] = v;
    }
}

/* DWTHandler::transform_from_rev with scalar = n^-1 (dwthandler.h:202-314, ntt.cpp:197-209):
 * Gentleman-Sande, inputs bit-reversed in [0,2q), outputs natural order in [0,2q). */
static void or_ntt_inv_lazy(uint64_t *values, const or_ntt_tables *t)
{
    const uint64_t q = t->mod.value, two_q = q << 1;
    const or_shoup *roots = t->inv_root_powers;
    size_t n = t->n, gap = 1, m = n >> 1;
    for (; m > 1; m >>= 1)
    {
        size_t offset = 0;
        for (size_t i = 0; i < m; i++)
        {
            or_shoup r = *++roots;
            uint64_t *x = values + offset, *y = x + gap;
            for (size_t j = 0; j < gap; j++)
            {
                uint64_t u = *x, v = *y;
                uint64_t s = u + v;
                *x++ = s >= two_q ? s - two_q : s;
                *y++ = or_mulmod_shoup_lazy(u + two_q - v, r, q);
            }
            offset += gap << 1;
        }
        gap <<= 1;
    }
    /* last stage merged with n^-1 (mul_root_scalar / mul_scalar, ntt.h:49-60) */
    or_shoup r = *++roots;
    or_shoup scaled = or_shoup_make(or_mulmod_shoup(r.operand, t->inv_degree, q), q);
    uint64_t *x = values, *y = values + gap;
    for (size_t j = 0; j < gap; j++)
    {
        uint64_t u = *x >= two_q ? *x - two_q : *x;
        uint64_t v = *y;
        uint64_t s = u + v;
        s = s >= two_q ? s - two_q : s;
        *x++ = or_mulmod_shoup_lazy(s, t->inv_degree, q);
        *y++ = or_mulmod_shoup_lazy(u + two_q - v, scaled, q);
    }
}

/* inverse_ntt_negacyclic_harvey (util/ntt.h:336-358): lazy INTT then reduce to [0,q). */
static void or_ntt_inv(uint64_t *values, const or_ntt_tables *t)
{
    or_ntt_inv_lazy(values, t);
    const uint64_t q = t->mod.value;
    for (size_t i = 0; i < t->n; i++)
        if (values[i] >= q) values[i] -= q;
}

/* ------------------------------------------------------------------------------------------
 * Standalone entry points used by the known-answer tests
 * ------------------------------------------------------------------------------------------ */

OR_API uint64_t or_barrett_reduce_64(uint64_t x, uint64_t q)
{
    or_mod m;
    or_mod_init(&m, q);
    return or_barrett64(x, &m);
}

OR_API uint64_t or_barrett_reduce_128(uint64_t lo, uint64_t hi, uint64_t q)
{
    or_mod m;
    or_mod_init(&m, q);
    return or_barrett128(lo, hi, &m);
}

OR_API uint64_t or_multiply_uint_mod(uint64_t a, uint64_t b, uint64_t q)
{
    or_mod m;
    or_mod_init(&m, q);
    return or_mulmod(a, b, &m);
}

OR_API uint64_t or_shoup_quotient(uint64_t w, uint64_t q)
{
    return or_shoup_make(w, q).quotient;
}

OR_API uint64_t or_multiply_uint_mod_shoup(uint64_t x, uint64_t w, uint64_t q)
{
    return or_mulmod_shoup(x, or_shoup_make(w, q), q);
}

OR_API int or_try_invert_uint_mod(uint64_t a, uint64_t q, uint64_t *res)
{
    return or_invmod(a, q, res);
}

/* Writes root_powers[i].operand and inv_root_powers[i].operand for i < n. */
OR_API int or_ntt_root_powers(int log_n, uint64_t q, uint64_t *roots, uint64_t *inv_roots)
{
    or_ntt_tables t;
    if (or_ntt_tables_init(&t, log_n, q)) return -1;
    for (size_t i = 0; i < t.n; i++)
    {
        roots[i] = t.root_powers[i].operand;
        inv_roots[i] = t.inv_root_powers[i].operand;
    }
    or_ntt_tables_free(&t);
    return 0;
}

/* mode: 0 = ntt_negacyclic_harvey, 1 = _lazy, 2 = inverse, 3 = inverse_lazy.  count polys. */
OR_API int or_ntt(uint64_t *data, int log_n, uint64_t q, int count, int mode)
{
    or_ntt_tables t;
    if (or_ntt_tables_init(&t, log_n, q)) return -1;
    for (int c = 0; c < count; c++)
    {
        uint64_t *p = data + (size_t)c * t.n;
        switch (mode)
        {
        case 0: or_ntt_fwd(p, &t); break;
        case 1: or_ntt_fwd_lazy(p, &t); break;
        case 2: or_ntt_inv(p, &t); break;
        default: or_ntt_inv_lazy(p, &t); break;
        }
    }
    or_ntt_tables_free(&t);
    return 0;
}

/* ------------------------------------------------------------------------------------------
 * Context: the key-level modulus chain q_0 .. q_{L_top-1}, P (special prime last), as
 * SEALContext::key_context_data holds it (context.cpp:422-523).
 * ------------------------------------------------------------------------------------------ */

typedef struct
{
    int log_n;
    size_t n;
    int k;        /* number of key-level primes (data limbs + 1 special) */
    or_mod *mod;  /* [k] */
    or_ntt_tables *ntt; /* [k] */
} or_ctx;

OR_API or_ctx *or_ctx_create(int log_n, const uint64_t *moduli, int count)
{
    or_ctx *c = (or_ctx *)calloc(1, sizeof(or_ctx));
    c->log_n = log_n;
    c->n = (size_t)1 << log_n;
    c->k = count;
    c->mod = (or_mod *)malloc(sizeof(or_mod) * count);
    c->ntt = (or_ntt_tables *)calloc(count, sizeof(or_ntt_tables));
    for (int i = 0; i < count; i++)
    {
        or_mod_init(&c->mod[i], moduli[i]);
        if (or_ntt_tables_init(&c->ntt[i], log_n, moduli[i]))
        {
            for (int j = 0; j <= i; j++) or_ntt_tables_free(&c->ntt[j]);
            free(c->ntt);
            free(c->mod);
            free(c);
            return NULL;
        }
    }
    return c;
}

OR_API void or_ctx_destroy(or_ctx *c)
{
    if (!c) return;
    for (int i = 0; i < c->k; i++) or_ntt_tables_free(&c->ntt[i]);
    free(c->ntt);
    free(c->mod);
    free(c);
}

/* Per-limb NTT on an RNS polynomial array [polys][limbs][n] restricted to limbs
 * [limb_begin, limb_begin+limb_count) of the key chain; mode as in or_ntt. */
OR_API void or_ctx_ntt(const or_ctx *c, uint64_t *data, int polys, int limbs, int mode)
{
    for (int p = 0; p < polys; p++)
        for (int l = 0; l < limbs; l++)
        {
            uint64_t *v = data + ((size_t)p * limbs + l) * c->n;
            switch (mode)
            {
            case 0: or_ntt_fwd(v, &c->ntt[l]); break;
            case 1: or_ntt_fwd_lazy(v, &c->ntt[l]); break;
            case 2: or_ntt_inv(v, &c->ntt[l]); break;
            default: or_ntt_inv_lazy(v, &c->ntt[l]); break;
            }
        }
}

/* dyadic_product_coeffmod (util/polyarithsmallmod.cpp:111-165) over [limbs][n]. */
OR_API void or_ctx_dyadic(const or_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, int limbs)
{
    for (int l = 0; l < limbs; l++)
    {
        const or_mod *m = &c->mod[l];
        for (size_t i = 0; i < c->n; i++)
        {
            size_t o = (size_t)l * c->n + i;
            out[o] = or_mulmod(a[o], b[o], m);
        }
    }
}

/* add_poly_coeffmod / sub_poly_coeffmod / negate_poly_coeffmod (util/polyarithsmallmod.h:190-300)
 * over [polys][limbs][n].  op: 0 add, 1 sub, 2 negate (b unused). */
OR_API void or_ctx_addsub(const or_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, int polys, int limbs, int op)
{
    for (int p = 0; p < polys; p++)
        for (int l = 0; l < limbs; l++)
        {
            uint64_t q = c->mod[l].value;
            size_t base = ((size_t)p * limbs + l) * c->n;
            for (size_t i = 0; i < c->n; i++)
            {
                uint64_t x = a[base + i], r;
                if (op == 0)
                {
                    r = x + b[base + i];
                    r = r >= q ? r - q : r;
                }
                else if (op == 1)
                {
                    uint64_t y = b[base + i];
                    r = x >= y ? x - y : x + q - y;
                }
                else
                    r = x ? q - x : 0;
                out[base + i] = r;
            }
        }
}

/* Evaluator::ckks_multiply, size-2 x size-2 tile path (evaluator.cpp:673-773).
 * a, b: [2][L][n]; out: [3][L][n] (out may alias a's storage only if sized for 3). */
OR_API void or_ctx_ckks_multiply(const or_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, int L)
{
    size_t n = c->n, ps = (size_t)L * n;
    for (int l = 0; l < L; l++)
    {
        const or_mod *m = &c->mod[l];
        uint64_t q = m->value;
        for (size_t i = 0; i < n; i++)
        {
            size_t o = (size_t)l * n + i;
            uint64_t x0 = a[o], x1 = a[ps + o], y0 = b[o], y1 = b[ps + o];
            uint64_t c2 = or_mulmod(x1, y1, m);
            uint64_t t = or_mulmod(x1, y0, m);
            uint64_t c1 = or_mulmod(x0, y1, m) + t;
            c1 = c1 >= q ? c1 - q : c1;
            out[o] = or_mulmod(x0, y0, m);
            out[ps + o] = c1;
            out[2 * ps + o] = c2;
        }
    }
}

/* Evaluator::ckks_square (evaluator.cpp:1000-1059): (c0^2, 2 c0 c1, c1^2). */
OR_API void or_ctx_ckks_square(const or_ctx *c, const uint64_t *a, uint64_t *out, int L)
{
    size_t n = c->n, ps = (size_t)L * n;
    for (int l = 0; l < L; l++)
    {
        const or_mod *m = &c->mod[l];
        uint64_t q = m->value;
        for (size_t i = 0; i < n; i++)
        {
            size_t o = (size_t)l * n + i;
            uint64_t x0 = a[o], x1 = a[ps + o];
            uint64_t c2 = or_mulmod(x1, x1, m);
            uint64_t c1 = or_mulmod(x0, x1, m);
            c1 = c1 + c1;
            c1 = c1 >= q ? c1 - q : c1;
            out[o] = or_mulmod(x0, x0, m);
            out[ps + o] = c1;
            out[2 * ps + o] = c2;
        }
    }
}

/* Evaluator::switch_key_inplace, CKKS branch (evaluator.cpp:2281-2525).
 *   ct:     [2][L][n] NTT form, modified in place (ct += KS(target))
 *   target: [L][n] NTT form
 *   key:    one KSwitchKeys entry, [decomp][2][key_limbs][n] with key_limbs = c->k, special last
 *           (keygenerator.cpp:384-414 layout: vector<PublicKey> of size-2 ciphertexts)
 *   L:      data limbs of ct (decomp_modulus_size)                                          */
OR_API int or_ctx_switch_key(const or_ctx *c, uint64_t *ct, const uint64_t *target, const uint64_t *key, int L)
{
    const size_t n = c->n;
    const int K = c->k;                 /* key_modulus_size */
    const int R = L + 1;                /* rns_modulus_size */
    if (L < 1 || L > K - 1) return -1;
    const size_t key_comp = (size_t)K * n, key_digit = 2 * key_comp;

    /* t_target = INTT(target) (:2345-2354) */
    uint64_t *t_target = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)L * n);
    memcpy(t_target, target, sizeof(uint64_t) * (size_t)L * n);
    for (int j = 0; j < L; j++) or_ntt_inv(t_target + (size_t)j * n, &c->ntt[j]);

    uint64_t *t_poly_prod = (uint64_t *)calloc((size_t)2 * R * n, sizeof(uint64_t)); /* [2][R][n] */
    uint64_t *lazy = (uint64_t *)malloc(sizeof(uint64_t) * 2 * 2 * n);                 /* [2][n][2] */
    uint64_t *t_ntt = (uint64_t *)malloc(sizeof(uint64_t) * n);

    for (int I = 0; I < R; I++)
    {
        int key_index = (I == L) ? K - 1 : I;
        const or_mod *km = &c->mod[key_index];
        const size_t bound = 256; /* SEAL_MULTIPLY_ACCUMULATE_USER_MOD_MAX (util/defines.h:63) */
        size_t counter = bound;
        memset(lazy, 0, sizeof(uint64_t) * 4 * n);
        for (int J = 0; J < L; J++)
        {
            const uint64_t *op;
            if (I == J)
                op = target + (size_t)J * n; /* reuse RNS-NTT form (:2380-2384) */
            else
            {
                if (c->mod[J].value <= km->value)
                    memcpy(t_ntt, t_target + (size_t)J * n, sizeof(uint64_t) * n);
                else
                    for (size_t i = 0; i < n; i++) t_ntt[i] = or_barrett64(t_target[(size_t)J * n + i], km);
                or_ntt_fwd_lazy(t_ntt, &c->ntt[key_index]);
                op = t_ntt;
            }
            for (int k = 0; k < 2; k++)
            {
                const uint64_t *kp = key + (size_t)J * key_digit + (size_t)k * key_comp + (size_t)key_index * n;
                uint64_t *acc = lazy + (size_t)k * 2 * n;
                for (size_t i = 0; i < n; i++)
                {
                    u128 prod = (u128)op[i] * kp[i];
                    u128 s = prod + (((u128)acc[2 * i + 1] << 64) | acc[2 * i]);
                    if (!counter)
                    {
                        acc[2 * i] = or_barrett128((uint64_t)s, (uint64_t)(s >> 64), km);
                        acc[2 * i + 1] = 0;
                    }
                    else
                    {
                        acc[2 * i] = (uint64_t)s;
                        acc[2 * i + 1] = (uint64_t)(s >> 64);
                    }
                }
            }
            if (!--counter) counter = bound;
        }
        for (int k = 0; k < 2; k++)
        {
            uint64_t *dst = t_poly_prod + ((size_t)k * R + I) * n;
            const uint64_t *acc = lazy + (size_t)k * 2 * n;
            for (size_t i = 0; i < n; i++)
                dst[i] = (counter == bound) ? acc[2 * i] : or_barrett128(acc[2 * i], acc[2 * i + 1], km);
        }
    }

    /* Modulus switching with scaling by P^-1 (:2466-2524) */
    const or_mod *pm = &c->mod[K - 1];
    const uint64_t qk = pm->value, qk_half = qk >> 1;
    for (int k = 0; k < 2; k++)
    {
        uint64_t *t_last = t_poly_prod + ((size_t)k * R + L) * n;
        or_ntt_inv_lazy(t_last, &c->ntt[K - 1]);
        for (size_t i = 0; i < n; i++) t_last[i] = or_barrett64(t_last[i] + qk_half, pm);
        for (int j = 0; j < L; j++)
        {
            const or_mod *qm = &c->mod[j];
            uint64_t qi = qm->value;
            if (qk > qi)
                for (size_t i = 0; i < n; i++) t_ntt[i] = or_barrett64(t_last[i], qm);
            else
                memcpy(t_ntt, t_last, sizeof(uint64_t) * n);
            uint64_t fix = qi - or_barrett64(qk_half, qm);
            for (size_t i = 0; i < n; i++) t_ntt[i] += fix;
            or_ntt_fwd_lazy(t_ntt, &c->ntt[j]);
            uint64_t qi_lazy = qi << 2;
            uint64_t inv_p = 0;
            or_invmod(qk, qi, &inv_p); /* key rns_tool inv_q_last_mod_q (util/rns.cpp:686-693) */
            or_shoup sp = or_shoup_make(inv_p, qi);
            uint64_t *prod = t_poly_prod + ((size_t)k * R + j) * n;
            uint64_t *dst = ct + ((size_t)k * L + j) * n;
            for (size_t i = 0; i < n; i++)
            {
                uint64_t v = prod[i] + qi_lazy - t_ntt[i];
                v = or_mulmod_shoup(v, sp, qi);
                v = v + dst[i];
                dst[i] = v >= qi ? v - qi : v;
            }
        }
    }
    free(t_ntt);
    free(lazy);
    free(t_poly_prod);
    free(t_target);
    return 0;
}

/* Evaluator::relinearize_internal for a size-3 ciphertext (evaluator.cpp:1061-1116):
 * switch_key(ct[0..1], target = ct[2], relin key index 0), drop c2.
 * ct: [3][L][n] -> the first [2][L][n] hold the result. */
OR_API int or_ctx_relinearize(const or_ctx *c, uint64_t *ct, const uint64_t *key, int L)
{
    return or_ctx_switch_key(c, ct, ct + (size_t)2 * L * c->n, key, L);
}

/* RNSTool::divide_and_round_q_last_ntt_inplace (util/rns.cpp:737-808) for every component,
 * then the copy-down of mod_switch_scale_to_next (evaluator.cpp:1118-1181).
 * in: [size][L][n] (unchanged); out: [size][L-1][n]. */
OR_API int or_ctx_rescale(const or_ctx *c, const uint64_t *in, uint64_t *out, int size, int L)
{
    const size_t n = c->n;
    if (L < 2) return -1;
    const or_mod *lm = &c->mod[L - 1];
    const uint64_t half = lm->value >> 1;
    uint64_t *last = (uint64_t *)malloc(sizeof(uint64_t) * n);
    uint64_t *temp = (uint64_t *)malloc(sizeof(uint64_t) * n);
    for (int s = 0; s < size; s++)
    {
        memcpy(last, in + ((size_t)s * L + (L - 1)) * n, sizeof(uint64_t) * n);
        or_ntt_inv(last, &c->ntt[L - 1]);
        /* add_poly_scalar_coeffmod(last, half) */
        for (size_t i = 0; i < n; i++)
        {
            uint64_t v = last[i] + half;
            last[i] = v >= lm->value ? v - lm->value : v;
        }
        for (int i = 0; i < L - 1; i++)
        {
            const or_mod *qm = &c->mod[i];
            const uint64_t qi = qm->value;
            if (qi < lm->value)
                for (size_t j = 0; j < n; j++) temp[j] = or_barrett64(last[j], qm);
            else
                memcpy(temp, last, sizeof(uint64_t) * n);
            uint64_t neg_half_mod = qi - or_barrett64(half, qm);
            for (size_t j = 0; j < n; j++) temp[j] += neg_half_mod;
            uint64_t qi_lazy = qi << 2;
            or_ntt_fwd_lazy(temp, &c->ntt[i]);
            uint64_t inv = 0;
            or_invmod(lm->value, qi, &inv);
            or_shoup sp = or_shoup_make(inv, qi);
            const uint64_t *src = in + ((size_t)s * L + i) * n;
            uint64_t *dst = out + ((size_t)s * (L - 1) + i) * n;
            for (size_t j = 0; j < n; j++) dst[j] = or_mulmod_shoup(src[j] + qi_lazy - temp[j], sp, qi);
        }
    }
    free(temp);
    free(last);
    return 0;
}

/* GaloisTool::get_elt_from_step (util/galois.cpp:53-95), generator_ = 5 (util/galois.h:169). */
OR_API uint32_t or_galois_elt_from_step(uint64_t n, int step)
{
    uint64_t m = 2 * n;
    if (step == 0) return (uint32_t)(m - 1);
    int sign = step < 0;
    uint64_t pos = (uint64_t)(step < 0 ? -step : step);
    if (pos >= (n >> 1)) return 0;
    pos &= m - 1;
    uint64_t s = sign ? (n >> 1) - pos : pos;
    uint64_t elt = 1;
    while (s--)
    {
        elt *= 5;
        elt &= m - 1;
    }
    return (uint32_t)elt;
}

/* GaloisTool::generate_table_ntt (util/galois.cpp:18-51). */
OR_API void or_galois_table_ntt(int log_n, uint32_t galois_elt, uint32_t *table)
{
    uint32_t n = 1u << log_n, mask = n - 1;
    for (uint32_t i = n; i < (n << 1); i++)
    {
        uint32_t reversed = or_reverse_bits(i, log_n + 1);
        uint64_t idx = ((uint64_t)galois_elt * reversed) >> 1;
        idx &= mask;
        *table++ = or_reverse_bits((uint32_t)idx, log_n);
    }
}

/* GaloisTool::apply_galois_ntt (util/galois.cpp:192-218) over [limbs][n]. */
OR_API void or_apply_galois_ntt(const uint64_t *in, int log_n, int limbs, uint32_t galois_elt, uint64_t *out)
{
    size_t n = (size_t)1 << log_n;
    uint32_t *table = (uint32_t *)malloc(sizeof(uint32_t) * n);
    or_galois_table_ntt(log_n, galois_elt, table);
    for (int l = 0; l < limbs; l++)
        for (size_t i = 0; i < n; i++) out[(size_t)l * n + i] = in[(size_t)l * n + table[i]];
    free(table);
}

/* Evaluator::apply_galois_inplace, CKKS branch (evaluator.cpp:2120-2222):
 * c0 <- perm(c0); temp <- perm(c1); c1 <- 0; switch_key(ct, temp).  ct: [2][L][n]. */
OR_API int or_ctx_apply_galois(const or_ctx *c, uint64_t *ct, uint32_t galois_elt, const uint64_t *key, int L)
{
    size_t ps = (size_t)L * c->n;
    uint64_t *temp = (uint64_t *)malloc(sizeof(uint64_t) * ps);
    or_apply_galois_ntt(ct, c->log_n, L, galois_elt, temp);
    memcpy(ct, temp, sizeof(uint64_t) * ps);
    or_apply_galois_ntt(ct + ps, c->log_n, L, galois_elt, temp);
    memset(ct + ps, 0, sizeof(uint64_t) * ps);
    int r = or_ctx_switch_key(c, ct, temp, key, L);
    free(temp);
    return r;
}

/* Evaluator::multiply_plain_ntt (evaluator.cpp:1891-1930): ct[s] (.) pt per limb. */
OR_API void or_ctx_multiply_plain(const or_ctx *c, uint64_t *ct, const uint64_t *pt, int size, int L)
{
    size_t ps = (size_t)L * c->n;
    for (int s = 0; s < size; s++) or_ctx_dyadic(c, ct + s * ps, pt, ct + s * ps, L);
}

/* One HMult: multiply_inplace + relinearize_inplace + rescale_to_next_inplace.
 * a, b: [2][L][n]; out: [2][L-1][n]; scratch allocated internally. */
OR_API int or_ctx_hmult(const or_ctx *c, const uint64_t *a, const uint64_t *b, const uint64_t *key, uint64_t *out, int L)
{
    size_t ps = (size_t)L * c->n;
    uint64_t *t3 = (uint64_t *)malloc(sizeof(uint64_t) * 3 * ps);
    or_ctx_ckks_multiply(c, a, b, t3, L);
    int r = or_ctx_relinearize(c, t3, key, L);
    if (!r) r = or_ctx_rescale(c, t3, out, 2, L);
    free(t3);
    return r;
}

/* Batched HMults for the CPU baseline (bench.py cpu_baseline leg): B independent
 * HMults over the same key, one per OpenMP thread, as the reference runs one image per
 * OpenMP thread (cnn/infer_seal.cpp:404).  Returns the number of threads used. */
#include <omp.h>
OR_API int or_ctx_hmult_batch(const or_ctx *c, const uint64_t *a, const uint64_t *b, const uint64_t *key, uint64_t *out,
                              int L, int batch, int threads)
{
    size_t in_stride = (size_t)2 * L * c->n, out_stride = (size_t)2 * (L - 1) * c->n;
    if (threads > 0) omp_set_num_threads(threads);
    int used = 1;
#pragma omp parallel
    {
#pragma omp single
        used = omp_get_num_threads();
#pragma omp for schedule(dynamic, 1)
        for (int i = 0; i < batch; i++)
            or_ctx_hmult(c, a + i * in_stride, b + i * in_stride, key, out + i * out_stride, L);
    }
    return used;
}

/* The same over every host core: `batch` independent HMults drawn cyclically from `distinct`
 * input pairs (so B can be the core count without B distinct inputs in memory); the output of
 * HMult i goes to the slot of the thread that ran it (out: [threads][2][L-1][n]). */
OR_API int or_ctx_hmult_batch_cyclic(const or_ctx *c, const uint64_t *a, const uint64_t *b, int distinct,
                                     const uint64_t *key, uint64_t *out, int L, int batch, int threads)
{
    size_t in_stride = (size_t)2 * L * c->n, out_stride = (size_t)2 * (L - 1) * c->n;
    if (threads > 0) omp_set_num_threads(threads);
    int used = 1;
#pragma omp parallel
    {
#pragma omp single
        used = omp_get_num_threads();
        uint64_t *o = out + (size_t)omp_get_thread_num() * out_stride;
#pragma omp for schedule(dynamic, 1)
        for (int i = 0; i < batch; i++)
            or_ctx_hmult(c, a + (i % distinct) * in_stride, b + (i % distinct) * in_stride, key, o, L);
    }
    return used;
}

/* ------------------------------------------------------------------------------------------
 * CKKS encoder (ckks.cpp:10-60 constructor tables, ckks.h:457-640 encode_internal,
 * ckks.cpp:78-200 encode_internal(double), util/croots.cpp ComplexRoots,
 * util/dwthandler.h:202-314 transform_from_rev over complex<double> with
 * Arithmetic<complex<double>> (ckks.h:46-81)).  Built with -ffp-contract=off: the reference
 * encodes without FMA (SEAL library at -O3 for baseline x86-64, cnn driver at -O0), so the
 * double results here are bit-identical to SEAL's for the same libm.
 * ------------------------------------------------------------------------------------------ */
typedef struct
{
    double re, im;
} or_cplx;

static or_cplx or_c(double re, double im)
{
    or_cplx z = { re, im };
    return z;
}
static or_cplx or_cmul(or_cplx a, or_cplx b) /* std::complex operator* (finite path) */
{
    return or_c(a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re);
}
static or_cplx or_cadd(or_cplx a, or_cplx b)
{
    return or_c(a.re + b.re, a.im + b.im);
}
static or_cplx or_csub(or_cplx a, or_cplx b)
{
    return or_c(a.re - b.re, a.im - b.im);
}
static or_cplx or_cscale(or_cplx a, double s)
{
    return or_c(a.re * s, a.im * s);
}

/* ComplexRoots (util/croots.cpp:17-66) for degree m = 2n. */
typedef struct
{
    size_t m;
    or_cplx *roots; /* m/8 + 1 entries */
} or_croots;

static void or_croots_init(or_croots *c, size_t m)
{
    const double PI_ = 3.1415926535897932384626433832795028842;
    c->m = m;
    c->roots = (or_cplx *)malloc(sizeof(or_cplx) * (m / 8 + 1));
    for (size_t i = 0; i <= m / 8; i++)
    {
        /* polar<double>(1.0, theta): SEAL's Release build with GCC lowers the cos/sin pair of
         * std::polar to one sincos() call, which differs from separate cos()/sin() in the last
         * bit for a few angles (e.g. i = 487 at m = 8192); sincos is called explicitly so the
         * tables do not depend on the optimisation level. */
        double th = 2 * PI_ * (double)i / (double)m, sn, cs;
        sincos(th, &sn, &cs);
        c->roots[i] = or_c(cs, sn);
    }
}

static or_cplx or_croot(const or_croots *c, size_t index)
{
    size_t m = c->m;
    index &= m - 1;
    if (index <= m / 8) return c->roots[index];
    if (index <= m / 4)
    {
        or_cplx a = c->roots[m / 4 - index];
        return or_c(a.im, a.re); /* mirror */
    }
    if (index <= m / 2)
    {
        or_cplx a = or_croot(c, m / 2 - index);
        return or_c(-a.re, a.im); /* -conj(a) */
    }
    if (index <= 3 * m / 4)
    {
        or_cplx a = or_croot(c, index - m / 2);
        return or_c(-a.re, -a.im);
    }
    or_cplx a = or_croot(c, m - index);
    return or_c(a.re, -a.im); /* conj */
}

/* CKKSEncoder constructor tables: matrix_reps_index_map_ (5^i), root_powers_ (bit-reversed),
 * inv_root_powers_ (scrambled, conjugated). */
typedef struct
{
    int log_n;
    size_t n, slots;
    size_t *index_map;
    or_cplx *root_powers, *inv_root_powers;
} or_encoder;

OR_API or_encoder *or_encoder_create(int log_n)
{
    or_encoder *e = (or_encoder *)calloc(1, sizeof(or_encoder));
    size_t n = (size_t)1 << log_n, m = n << 1;
    e->log_n = log_n;
    e->n = n;
    e->slots = n >> 1;
    e->index_map = (size_t *)malloc(sizeof(size_t) * n);
    uint64_t pos = 1;
    for (size_t i = 0; i < e->slots; i++)
    {
        uint64_t index1 = (pos - 1) >> 1, index2 = (m - pos - 1) >> 1;
        e->index_map[i] = or_reverse_bits((uint32_t)index1, log_n);
        e->index_map[e->slots | i] = or_reverse_bits((uint32_t)index2, log_n);
        pos *= 5;
        pos &= (m - 1);
    }
    e->root_powers = (or_cplx *)calloc(n, sizeof(or_cplx));
    e->inv_root_powers = (or_cplx *)calloc(n, sizeof(or_cplx));
    or_croots cr;
    or_croots_init(&cr, m);
    for (size_t i = 1; i < n; i++)
    {
        e->root_powers[i] = or_croot(&cr, or_reverse_bits((uint32_t)i, log_n));
        or_cplx r = or_croot(&cr, or_reverse_bits((uint32_t)(i - 1), log_n) + 1);
        e->inv_root_powers[i] = or_c(r.re, -r.im);
    }
    free(cr.roots);
    return e;
}

OR_API void or_encoder_destroy(or_encoder *e)
{
    if (!e) return;
    free(e->index_map);
    free(e->root_powers);
    free(e->inv_root_powers);
    free(e);
}

/* DWTHandler<complex<double>, complex<double>, double>::transform_from_rev with scalar. */
static void or_fft_from_rev(or_cplx *values, int log_n, const or_cplx *roots, double scalar)
{
    size_t n = (size_t)1 << log_n, gap = 1, m = n >> 1;
    for (; m > 1; m >>= 1)
    {
        size_t offset = 0;
        for (size_t i = 0; i < m; i++)
        {
            or_cplx r = *++roots;
            or_cplx *x = values + offset, *y = x + gap;
            for (size_t j = 0; j < gap; j++)
            {
                or_cplx u = *x, v = *y;
                *x++ = or_cadd(u, v);
                *y++ = or_cmul(or_csub(u, v), r);
            }
            offset += gap << 1;
        }
        gap <<= 1;
    }
    or_cplx r = *++roots;
    or_cplx scaled_r = or_cscale(r, scalar);
    or_cplx *x = values, *y = values + gap;
    for (size_t j = 0; j < gap; j++)
    {
        or_cplx u = *x, v = *y;
        *x++ = or_cscale(or_cadd(u, v), scalar);
        *y++ = or_cmul(or_csub(u, v), scaled_r);
    }
}

/* Multi-word decomposition of a non-negative integer given as little-endian words into RNS
 * (RNSBase::decompose, util/rns.cpp): value mod q_j by Horner from the top word. */
static uint64_t or_words_mod(const uint64_t *w, int nw, const or_mod *m)
{
    uint64_t r = 0;
    for (int k = nw - 1; k >= 0; k--) r = or_barrett128(w[k], r, m);
    return r;
}

/* encode_internal for complex values (ckks.h:457-640), at a level with `limbs` primes of the
 * context: writes the NTT-form plaintext [limbs][n].  total_bits = total coeff modulus bit
 * count of that level (for the SEAL range checks).  Returns 0, -1 scale out of bounds,
 * -2 values too large. */
OR_API int or_ckks_encode(const or_encoder *e, const or_ctx *c, const double *re, const double *im, size_t count,
                          double scale, int limbs, int total_bits, uint64_t *out)
{
    size_t n = e->n;
    if (scale <= 0 || ((int)log2(scale)) + 1 >= total_bits) return -1;
    or_cplx *cv = (or_cplx *)calloc(n, sizeof(or_cplx));
    for (size_t i = 0; i < count; i++)
    {
        or_cplx v = or_c(re[i], im ? im[i] : 0.0);
        cv[e->index_map[i]] = v;
        cv[e->index_map[i + e->slots]] = or_c(v.re, -v.im);
    }
    double fix = scale / (double)n;
    or_fft_from_rev(cv, e->log_n, e->inv_root_powers, fix);
    double max_coeff = 0;
    for (size_t i = 0; i < n; i++) max_coeff = fmax(max_coeff, fabs(cv[i].re));
    int max_bits = (int)ceil(log2(fmax(max_coeff, 1.0))) + 1;
    if (max_bits >= total_bits)
    {
        free(cv);
        return -2;
    }
    const double two64 = pow(2.0, 64);
    for (size_t i = 0; i < n; i++)
    {
        double cd = round(cv[i].re);
        int neg = signbit(cd) ? 1 : 0;
        cd = fabs(cd);
        uint64_t w[64] = { 0 };
        int nw;
        if (max_bits <= 64)
        {
            w[0] = (uint64_t)cd;
            nw = 1;
        }
        else if (max_bits <= 128)
        {
            w[0] = (uint64_t)fmod(cd, two64);
            w[1] = (uint64_t)(cd / two64);
            nw = 2;
        }
        else
        {
            nw = 0;
            while (cd >= 1)
            {
                w[nw++] = (uint64_t)fmod(cd, two64);
                cd /= two64;
            }
            if (!nw) nw = 1;
        }
        for (int j = 0; j < limbs; j++)
        {
            const or_mod *m = &c->mod[j];
            uint64_t r = (nw == 1) ? or_barrett64(w[0], m) : or_words_mod(w, nw, m);
            out[(size_t)j * n + i] = (neg && r) ? m->value - r : r;
        }
    }
    free(cv);
    for (int j = 0; j < limbs; j++) or_ntt_fwd(out + (size_t)j * n, &c->ntt[j]);
    return 0;
}

/* encode_internal(double value, ...) (ckks.cpp:78-200): a constant polynomial, written as
 * one residue per limb (the plaintext is that residue in every coefficient, NTT of a
 * constant is the constant).  Returns the SEAL error codes as or_ckks_encode. */
OR_API int or_ckks_encode_scalar(const or_ctx *c, double value, double scale, int limbs, int total_bits,
                                 uint64_t *residues)
{
    if (scale <= 0 || ((int)log2(scale)) >= total_bits) return -1;
    value *= scale;
    int coeff_bits = (int)log2(fabs(value)) + 2;
    if (coeff_bits >= total_bits) return -2;
    const double two64 = pow(2.0, 64);
    double cd = round(value);
    int neg = signbit(cd) ? 1 : 0;
    cd = fabs(cd);
    uint64_t w[64] = { 0 };
    int nw;
    if (coeff_bits <= 64)
    {
        w[0] = (uint64_t)fabs(cd);
        nw = 1;
    }
    else if (coeff_bits <= 128)
    {
        w[0] = (uint64_t)fmod(cd, two64);
        w[1] = (uint64_t)(cd / two64);
        nw = 2;
    }
    else
    {
        nw = 0;
        while (cd >= 1)
        {
            w[nw++] = (uint64_t)fmod(cd, two64);
            cd /= two64;
        }
        if (!nw) nw = 1;
    }
    for (int j = 0; j < limbs; j++)
    {
        const or_mod *m = &c->mod[j];
        uint64_t r = (nw == 1) ? or_barrett64(w[0], m) : or_words_mod(w, nw, m);
        residues[j] = (neg && r) ? m->value - r : r;
    }
    return 0;
}

/* --------------------------------------------------------------------------------------------
 * CKKS decode (ckks.h:644-761): inverse NTT per limb, CRT compose (RNSBase::compose_array,
 * util/rns.cpp:354-400), sparse-slot masking (modified SEAL, ckks.h:704-713), SEAL's
 * word-by-word conversion to double (ckks.h:715-753), transform_to_rev with root_powers_
 * (util/dwthandler.h:94-190), slot gather through matrix_reps_index_map_.
 * ------------------------------------------------------------------------------------------ */
static void or_mp_mul_scalar(const uint64_t *a, int L, uint64_t s, uint64_t *out) /* multiply_uint, truncated to L words */
{
    uint64_t carry = 0;
    for (int k = 0; k < L; k++)
    {
        u128 p = (u128)a[k] * s + carry;
        out[k] = (uint64_t)p;
        carry = (uint64_t)(p >> 64);
    }
}

static int or_mp_geq(const uint64_t *a, const uint64_t *b, int L)
{
    for (int k = L - 1; k >= 0; k--)
        if (a[k] != b[k]) return a[k] > b[k];
    return 1;
}

static void or_mp_sub(uint64_t *a, const uint64_t *b, int L) /* a -= b */
{
    uint64_t borrow = 0;
    for (int k = 0; k < L; k++)
    {
        uint64_t d = a[k] - b[k];
        uint64_t b2 = (a[k] < b[k]) | (d < borrow);
        a[k] = d - borrow;
        borrow = b2;
    }
}

static void or_mp_add_mod(uint64_t *acc, const uint64_t *b, const uint64_t *Q, int L) /* add_uint_uint_mod */
{
    uint64_t carry = 0;
    for (int k = 0; k < L; k++)
    {
        u128 s = (u128)acc[k] + b[k] + carry;
        acc[k] = (uint64_t)s;
        carry = (uint64_t)(s >> 64);
    }
    if (carry || or_mp_geq(acc, Q, L)) or_mp_sub(acc, Q, L);
}

static void or_fft_to_rev(or_cplx *values, int log_n, const or_cplx *roots)
{
    size_t n = (size_t)1 << log_n, gap = n >> 1, m = 1;
    for (; m < (n >> 1); m <<= 1)
    {
        size_t offset = 0;
        for (size_t i = 0; i < m; i++)
        {
            or_cplx r = *++roots;
            or_cplx *x = values + offset, *y = x + gap;
            for (size_t j = 0; j < gap; j++)
            {
                or_cplx u = *x, v = or_cmul(*y, r);
                *x++ = or_cadd(u, v);
                *y++ = or_csub(u, v);
            }
            offset += gap << 1;
        }
        gap >>= 1;
    }
    for (size_t i = 0; i < m; i++)
    {
        or_cplx r = *++roots;
        or_cplx u = values[0], v = or_cmul(values[1], r);
        values[0] = or_cadd(u, v);
        values[1] = or_csub(u, v);
        values += 2;
    }
}

/* plain: NTT-form [limbs][n] at a level of `limbs` primes; total_bits of that level; writes
 * sparse_slots values (sparse_slots = 0 means n/2).  Returns 0 or -1 (scale out of bounds). */
static int or_ckks_decode_impl(const or_encoder *e, const or_ctx *c, const uint64_t *plain, int limbs, double scale,
                               int total_bits, size_t sparse_slots, double *re, double *im, double *coeffs_out);

/* The real-valued coefficients before transform_to_rev (ckks.h:715-753), for testing the
 * conversion step alone. */
OR_API int or_ckks_decode_coeffs(const or_encoder *e, const or_ctx *c, const uint64_t *plain, int limbs, double scale,
                                 int total_bits, size_t sparse_slots, double *coeffs)
{
    return or_ckks_decode_impl(e, c, plain, limbs, scale, total_bits, sparse_slots, NULL, NULL, coeffs);
}

OR_API int or_ckks_decode(const or_encoder *e, const or_ctx *c, const uint64_t *plain, int limbs, double scale,
                          int total_bits, size_t sparse_slots, double *re, double *im)
{
    return or_ckks_decode_impl(e, c, plain, limbs, scale, total_bits, sparse_slots, re, im, NULL);
}

static int or_ckks_decode_impl(const or_encoder *e, const or_ctx *c, const uint64_t *plain, int limbs, double scale,
                               int total_bits, size_t sparse_slots, double *re, double *im, double *coeffs_out)
{
    const size_t n = e->n, L = (size_t)limbs;
    if (scale <= 0 || ((int)log2(scale)) >= total_bits) return -1;
    if (!sparse_slots) sparse_slots = e->slots;
    uint64_t *x = (uint64_t *)malloc(sizeof(uint64_t) * n * L);
    memcpy(x, plain, sizeof(uint64_t) * n * L);
    for (size_t j = 0; j < L; j++) or_ntt_inv(x + j * n, &c->ntt[j]);

    /* base constants (RNSBase::initialize, util/rns.cpp): Q, Q/q_j, (Q/q_j)^{-1} mod q_j */
    uint64_t *Q = (uint64_t *)calloc(L, sizeof(uint64_t));
    uint64_t *punct = (uint64_t *)calloc(L * L, sizeof(uint64_t));
    uint64_t *inv_punct = (uint64_t *)calloc(L, sizeof(uint64_t));
    uint64_t *tmp = (uint64_t *)calloc(L + 1, sizeof(uint64_t));
    Q[0] = 1;
    for (size_t j = 0; j < L; j++)
    {
        or_mp_mul_scalar(Q, (int)L, c->mod[j].value, tmp);
        memcpy(Q, tmp, sizeof(uint64_t) * L);
    }
    for (size_t j = 0; j < L; j++)
    {
        uint64_t *p = punct + j * L;
        p[0] = 1;
        uint64_t pm = 1; /* punctured product mod q_j */
        for (size_t k = 0; k < L; k++)
        {
            if (k == j) continue;
            or_mp_mul_scalar(p, (int)L, c->mod[k].value, tmp);
            memcpy(p, tmp, sizeof(uint64_t) * L);
            pm = or_mulmod(pm, or_barrett64(c->mod[k].value, &c->mod[j]), &c->mod[j]);
        }
        if (L == 1) pm = 1;
        or_invmod(pm, c->mod[j].value, &inv_punct[j]);
    }

    /* compose: value_i = sum_j [x_ij * inv_j]_{q_j} * (Q/q_j) mod Q */
    uint64_t *comp = (uint64_t *)calloc(n * L, sizeof(uint64_t));
    for (size_t i = 0; i < n; i++)
    {
        uint64_t *acc = comp + i * L;
        if (L == 1)
        {
            acc[0] = x[i];
            continue;
        }
        for (size_t j = 0; j < L; j++)
        {
            uint64_t t = or_mulmod(x[j * n + i], inv_punct[j], &c->mod[j]);
            or_mp_mul_scalar(punct + j * L, (int)L, t, tmp);
            or_mp_add_mod(acc, tmp, Q, (int)L);
        }
    }
    if (sparse_slots != e->slots)
    {
        size_t sparsity = e->slots / sparse_slots;
        for (size_t i = 0; i < n; i++)
            if (((i - 1) & (sparsity - 1)) != sparsity - 1) memset(comp + i * L, 0, sizeof(uint64_t) * L);
    }

    /* upper_half_threshold = (Q + 1) / 2 */
    uint64_t *thr = (uint64_t *)calloc(L, sizeof(uint64_t));
    {
        uint64_t carry = 1;
        for (size_t k = 0; k < L; k++)
        {
            thr[k] = Q[k] + carry;
            carry = (carry && thr[k] == 0) ? 1 : 0;
        }
        for (size_t k = 0; k < L; k++) thr[k] = (thr[k] >> 1) | ((k + 1 < L) ? (thr[k + 1] << 63) : ((uint64_t)carry << 63));
    }
    const double two64 = pow(2.0, 64), inv_scale = 1.0 / scale;
    or_cplx *res = (or_cplx *)calloc(n, sizeof(or_cplx));
    for (size_t i = 0; i < n; i++)
    {
        const uint64_t *v = comp + i * L;
        double acc = 0.0, s64 = inv_scale;
        if (or_mp_geq(v, thr, (int)L))
        {
            for (size_t j = 0; j < L; j++, s64 *= two64)
            {
                if (v[j] > Q[j])
                {
                    uint64_t diff = v[j] - Q[j];
                    acc += diff ? (double)diff * s64 : 0.0;
                }
                else
                {
                    uint64_t diff = Q[j] - v[j];
                    acc -= diff ? (double)diff * s64 : 0.0;
                }
            }
        }
        else
        {
            for (size_t j = 0; j < L; j++, s64 *= two64)
            {
                uint64_t cc = v[j];
                acc += cc ? (double)cc * s64 : 0.0;
            }
        }
        res[i] = or_c(acc, 0.0);
        if (coeffs_out) coeffs_out[i] = acc;
    }
    if (!coeffs_out) or_fft_to_rev(res, e->log_n, e->root_powers);
    for (size_t i = 0; i < sparse_slots && re; i++)
    {
        or_cplx z = res[e->index_map[i]];
        re[i] = z.re;
        if (im) im[i] = z.im;
    }
    free(x);
    free(Q);
    free(punct);
    free(inv_punct);
    free(tmp);
    free(comp);
    free(thr);
    free(res);
    return 0;
}

/* SEAL randomness, keys and encryption (test infrastructure) */
#include "seal_random.c"
