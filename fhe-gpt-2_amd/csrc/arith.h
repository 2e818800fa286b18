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
};

__device__ __forceinline__ u64 mulhi64(u64 a, u64 b)
{
    return __umul64hi(a, b);
}

// multiply_uint_mod_lazy: x * w mod q in [0, 2q) for any 64-bit x.
__device__ __forceinline__ u64 mul_shoup_lazy(u64 x, u64 w, u64 wq, u64 q)
{
    return w * x - mulhi64(x, wq) * q;
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
    u64 t2lo = lo * p.r1, t2hi = mulhi64(lo, p.r1);
    u64 tmp1 = t2lo + carry;
    u64 tmp3 = t2hi + (tmp1 < carry);
    u64 u2lo = hi * p.r0, u2hi = mulhi64(hi, p.r0);
    u64 s = tmp1 + u2lo;
    carry = u2hi + (s < u2lo);
    tmp1 = hi * p.r1 + tmp3 + carry;
    return csub(lo - tmp1 * p.q, p.q);
}

// barrett_reduce_64 (util/uintarithsmallmod.h:206-224).
__device__ __forceinline__ u64 barrett64(u64 x, const PrimeDev &p)
{
    return csub(x - mulhi64(x, p.r1) * p.q, p.q);
}

// multiply_uint_mod (util/uintarithsmallmod.h:230-242).
__device__ __forceinline__ u64 mulmod(u64 a, u64 b, const PrimeDev &p)
{
    return barrett128(a * b, mulhi64(a, b), p);
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
    u64 plo = a * b, phi = mulhi64(a, b);
    u64 s = acc.lo + plo;
    acc.hi += phi + (s < plo);
    acc.lo = s;
}
