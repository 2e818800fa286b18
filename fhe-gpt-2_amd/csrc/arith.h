// Device-side 64-bit modular arithmetic for gfx950.
//
// Residues are u64 in [0, q) with q < 2^61 (SEAL caps user moduli at 60 bits,
// util/defines.h:40).  gfx950 has no 64x64 multiplier: every 64-bit product below lowers
// to v_mul_lo_u32 / v_mul_hi_u32 / v_mad_u64_u32 sequences, so the formulas are chosen to
// minimise full 64x64->128 products:
//   * twiddle / scalar products use Shoup's precomputed quotient (one mulhi + two mullo),
//     exactly SEAL's MultiplyUIntModOperand (util/uintarithsmallmod.h:249-318);
//   * variable x variable products use SEAL's 128-bit Barrett with const_ratio =
//     floor(2^128/q) (util/uintarithsmallmod.h:166-200).
// Any exact reduction gives the same canonical residue, so outputs are bit-identical to
// SEAL's; only the internal lazy ranges are ours.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint64_t u64;
typedef uint32_t u32;
typedef ulonglong2 Tw; // (w, floor(w 2^64 / q)): a Shoup operand

// Per-prime constants, one entry per key-level prime, resident in HBM.
struct PrimeDev
{
    u64 q;        // modulus
    u64 two_q;    // 2q
    u64 four_q;   // 4q
    u64 r0, r1;   // floor(2^128 / q) (Modulus::const_ratio, modulus.cpp:66-98)
    u64 ninv;     // n^-1 mod q
    u64 ninv_q;   // Shoup quotient of ninv
    u64 last_w;   // psi^-1 (itw[1]) * n^-1 mod q: last INTT stage twiddle (dwthandler.h:273-314)
    u64 last_wq;
    double qd, qi; // q and fl(1/q) as doubles: the elementwise kernels' FP64 products (q < 2^51)
};

// Table reads through the constant address space: with a uniform index they become scalar loads.  A
// kernel that also stores makes the compiler read a table behind a plain pointer with vector loads,
// and their s_waitcnt vmcnt also waits for every store in flight (one counter for both): in a column
// pass's output-prime loop, each prime's setup waited for the previous prime's stores.  The tables
// (primes, inverse factors) are never written while a kernel runs.
typedef const __attribute__((address_space(4))) u64 *const_u64_p;
static_assert(sizeof(PrimeDev) % 8 == 0, "PrimeDev is read as 64-bit words");
__device__ __forceinline__ PrimeDev prime_at(const PrimeDev *t, int i)
{
    constexpr int W = (int)(sizeof(PrimeDev) / 8);
    const const_u64_p w = (const_u64_p)t + (size_t)i * W;
    PrimeDev r;
    u64 *d = reinterpret_cast<u64 *>(&r);
#pragma unroll
    for (int k = 0; k < W; k++) d[k] = w[k];
    return r;
}
__device__ __forceinline__ Tw tw_at(const Tw *t, size_t i)
{
    const const_u64_p w = (const_u64_p)t + 2 * i;
    Tw r;
    r.x = w[0];
    r.y = w[1];
    return r;
}

// 64-bit products built only from v_mad_u64_u32 (32x32+64 -> 64), which gfx950 issues at
// half rate.  The default lowering of u64 '*' and __umul64hi uses v_mul_lo_u32 / v_mul_hi_u32,
// which are quarter rate (measured: scripts/ubench_valu.hip, DESIGN.md "Arithmetic"), and
// LLVM re-forms a wide multiply from any schoolbook expansion written in C.  So the single
// instruction is pinned with inline asm; the carry-out goes to a scratch SGPR pair that is
// never read, and operand/pair assembly stays with the compiler.
__device__ __forceinline__ u64 mad32(u32 a, u32 b, u64 c)
{
    u64 d, sc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(sc) : "v"(a), "v"(b), "v"(c));
    return d;
}

__device__ __forceinline__ u64 mul32(u32 a, u32 b)
{
    u64 d, sc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(d), "=s"(sc) : "v"(a), "v"(b));
    return d;
}

// floor(a * b / 2^64), exact: 4 v_mad_u64_u32 (b is the possibly-uniform operand).
__device__ __forceinline__ u64 mulhi64(u64 a, u64 b)
{
    const u32 a0 = (u32)a, a1 = (u32)(a >> 32), b0 = (u32)b, b1 = (u32)(b >> 32);
    const u64 p00 = mul32(b0, a0);
    const u64 p01 = mad32(b1, a0, p00 >> 32);
    const u64 p10 = mad32(b0, a1, (u32)p01);
    return mad32(b1, a1, (p01 >> 32) + (p10 >> 32));
}

// a * b mod 2^64: 3 v_mad_u64_u32 (the cross terms only feed the high word, so their
// addends may carry garbage above bit 31).
__device__ __forceinline__ u64 mullo64(u64 a, u64 b)
{
    const u32 a0 = (u32)a, a1 = (u32)(a >> 32), b0 = (u32)b, b1 = (u32)(b >> 32);
    const u32 cross = (u32)mad32(b0, a1, mul32(b1, a0));
    return mad32(b0, a0, (u64)cross << 32);
}

// full 128-bit product (lo, hi): 4 v_mad_u64_u32.
__device__ __forceinline__ void mul128(u64 a, u64 b, u64 &lo, u64 &hi)
{
    const u32 a0 = (u32)a, a1 = (u32)(a >> 32), b0 = (u32)b, b1 = (u32)(b >> 32);
    const u64 p00 = mul32(a0, b0);
    const u64 p01 = mad32(a0, b1, p00 >> 32);
    const u64 p10 = mad32(a1, b0, (u32)p01);
    lo = ((u64)(u32)p10 << 32) | (u32)p00;
    hi = mad32(a1, b1, (p01 >> 32) + (p10 >> 32));
}

// multiply_uint_mod_lazy: x * w mod q in [0, 2q) for any 64-bit x.
__device__ __forceinline__ u64 mul_shoup_lazy(u64 x, u64 w, u64 wq, u64 q)
{
    const u64 h = mulhi64(x, wq);
    const u64 nq = 0 - q; // w x - h q = w x + h (2^64 - q) (mod 2^64)
    const u32 x0 = (u32)x, x1 = (u32)(x >> 32), w0 = (u32)w, w1 = (u32)(w >> 32);
    const u32 h0 = (u32)h, h1 = (u32)(h >> 32), n0 = (u32)nq, n1 = (u32)(nq >> 32);
    u64 c = mul32(w0, x1);
    c = mad32(w1, x0, c);
    c = mad32(n1, h0, c);
    c = mad32(n0, h1, c); // low word = cross terms of both products (mod 2^32)
    return mad32(w0, x0, mul32(n0, h0)) + (c << 32); // one v_lshl_add_u64, garbage shifts out
}

// NB independent Shoup lazy products x[i] * w[i] (mod q, in [0, 2q)), computed step by step
// across the batch.  The schedule is written out explicitly: hipcc does not know the latency
// of the inline-asm v_mad_u64_u32, so it would otherwise emit one product's dependent chain
// back to back (an s_nop per link) instead of interleaving independent products.
template <int NB>
__device__ __forceinline__ void mul_shoup_lazy_batch(const u64 (&x)[NB], const Tw *const (&w)[NB], u64 q,
                                                     u64 (&out)[NB])
{
    const u64 nq = 0 - q;
    const u32 n0 = (u32)nq, n1 = (u32)(nq >> 32);
    u32 x0[NB], x1[NB], w0[NB], w1[NB], v0[NB], v1[NB];
    u64 t[NB], u[NB], h[NB], c[NB];
#pragma unroll
    for (int i = 0; i < NB; i++)
    {
        const Tw tw = *w[i];
        x0[i] = (u32)x[i];
        x1[i] = (u32)(x[i] >> 32);
        w0[i] = (u32)tw.x;
        w1[i] = (u32)(tw.x >> 32);
        v0[i] = (u32)tw.y;
        v1[i] = (u32)(tw.y >> 32);
    }
    // h = floor(x * w' / 2^64)
#pragma unroll
    for (int i = 0; i < NB; i++) t[i] = mul32(v0[i], x0[i]);
#pragma unroll
    for (int i = 0; i < NB; i++) t[i] = mad32(v1[i], x0[i], t[i] >> 32);
#pragma unroll
    for (int i = 0; i < NB; i++) u[i] = mad32(v0[i], x1[i], (u32)t[i]);
#pragma unroll
    for (int i = 0; i < NB; i++) h[i] = mad32(v1[i], x1[i], (t[i] >> 32) + (u[i] >> 32));
    // w x - h q (mod 2^64): cross terms of both products in one chain, then the low parts
#pragma unroll
    for (int i = 0; i < NB; i++) c[i] = mul32(w0[i], x1[i]);
#pragma unroll
    for (int i = 0; i < NB; i++) c[i] = mad32(w1[i], x0[i], c[i]);
#pragma unroll
    for (int i = 0; i < NB; i++) c[i] = mad32(n1, (u32)h[i], c[i]);
#pragma unroll
    for (int i = 0; i < NB; i++) c[i] = mad32(n0, (u32)(h[i] >> 32), c[i]);
#pragma unroll
    for (int i = 0; i < NB; i++) t[i] = mul32(n0, (u32)h[i]);
#pragma unroll
    for (int i = 0; i < NB; i++) t[i] = mad32(w0[i], x0[i], t[i]);
#pragma unroll
    for (int i = 0; i < NB; i++) out[i] = t[i] + (c[i] << 32);
}

__device__ __forceinline__ u64 csub(u64 x, u64 m)
{
    return x >= m ? x - m : x;
}

__device__ __forceinline__ u64 mul_shoup(u64 x, u64 w, u64 wq, u64 q)
{
    return csub(mul_shoup_lazy(x, w, wq, q), q);
}

// barrett_reduce_128 (util/uintarithsmallmod.h:166-200): (hi:lo) mod q, exact for q < 2^63.
__device__ __forceinline__ u64 barrett128(u64 lo, u64 hi, const PrimeDev &p)
{
    u64 carry = mulhi64(lo, p.r0);
    u64 t2lo, t2hi;
    mul128(lo, p.r1, t2lo, t2hi);
    u64 tmp1 = t2lo + carry;
    u64 tmp3 = t2hi + (tmp1 < carry);
    u64 u2lo, u2hi;
    mul128(hi, p.r0, u2lo, u2hi);
    u64 s = tmp1 + u2lo;
    carry = u2hi + (s < u2lo);
    tmp1 = mullo64(hi, p.r1) + tmp3 + carry;
    return csub(lo - mullo64(tmp1, p.q), p.q);
}

// barrett_reduce_64 (util/uintarithsmallmod.h:206-224).
__device__ __forceinline__ u64 barrett64(u64 x, const PrimeDev &p)
{
    return csub(x - mullo64(mulhi64(x, p.r1), p.q), p.q);
}

// multiply_uint_mod (util/uintarithsmallmod.h:230-242).
__device__ __forceinline__ u64 mulmod(u64 a, u64 b, const PrimeDev &p)
{
    u64 lo, hi;
    mul128(a, b, lo, hi);
    return barrett128(lo, hi, p);
}

__device__ __forceinline__ u64 addmod(u64 a, u64 b, u64 q)
{
    return csub(a + b, q);
}

__device__ __forceinline__ u64 submod(u64 a, u64 b, u64 q)
{
    return a >= b ? a - b : a + q - b;
}

// 128-bit accumulator for key-switching inner products (evaluator.cpp:2412-2441).
struct Acc128
{
    u64 lo, hi;
};

__device__ __forceinline__ void mac128(Acc128 &acc, u64 a, u64 b)
{
    u64 plo, phi;
    mul128(a, b, plo, phi);
    u64 s = acc.lo + plo;
    acc.hi += phi + (s < plo);
    acc.lo = s;
}
