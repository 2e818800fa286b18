// FP64-FMA modular arithmetic for primes q < 2^51 (gfx950).
//
// gfx950 has no 64x64 integer multiplier: a Shoup product costs 9-10 v_mad_u64_u32 plus
// 64-bit carries, ~35 VALU instructions per Harvey butterfly.  The FP64 pipe runs v_fma_f64 at
// the same rate as v_mad_u64_u32, and for q < 2^51 a residue and a 102-bit product are exact
// in doubles:
//     h = y*w (rounded), l = fma(y, w, -h)      -> y*w = h + l exactly
//     k = rint(y * w')  with w' = w/q           -> quotient estimate, |y*w/q - k| <= 1
//     r = fma(-k, q, h) + l                     -> r = y*w - k*q exactly, |r| <= 1.5q
// so a butterfly is ~11 full-rate FP64 operations.  Values are kept as doubles in the signed
// range |v| <= 2q between stages; the first load converts canonical/lazy u64 residues, the last
// store canonicalises.  Every output that leaves a transform is canonical, so results are the
// same residues SEAL's integer Harvey butterflies produce.
//
// Bounds (q < 2^51, |inputs| <= B = 2q < 2^52):
//   rint(y*w') errs by at most 2*B*2^-53 + 1/2 <= 1, so |r| <= 1.5q; |h - k*q| <= 1.5q + ulp(h)/2
//   <= 1.5q + 2^50 < 2^53, so the fma result is exact; a centered reduction x - rint(x/q)*q of
//   |x| <= 2^53 is within [-q/2 - 1, q/2 + 1].  Forward: x' = red(x) + r, y' = red(x) - r, so
//   |.| <= 2q + 1 is preserved.  Inverse: x' = red(x + y), y' = mulmod(red(x - y), w), |.| <= q.
//   (scripts/ubench_bfly.hip checks 1536 random stages at q ~ 2^51 against the integer path.)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Twiddle as (w, w/q).
typedef double2 TwF;

__device__ __forceinline__ double fp_rint(double x)
{
    return __builtin_rint(x);
}

// y*w mod q in (-1.5q, 1.5q) for |y| <= 4q, w in [0, q), ws = w/q.
__device__ __forceinline__ double fp_mulmod(double y, double w, double ws, double q)
{
    const double h = y * w;
    const double l = __builtin_fma(y, w, -h);
    const double k = fp_rint(y * ws);
    return __builtin_fma(-k, q, h) + l;
}

// a*b mod q in (-1.25q, 1.25q) for a general b in [0, q) (no precomputed b/q) and |a| <= 2^51:
// the quotient estimate rint(fl(a*b) * fl(1/q)) errs by at most 3*2^-53*|ab/q| + 1/2 <= 0.875.
// For |a| <= 2^52 (q < 2^51, a not reduced) it errs by at most 2: |result| <= 2q.
__device__ __forceinline__ double fp_mulmod_gen(double a, double b, double q, double qinv)
{
    const double h = a * b;
    const double l = __builtin_fma(a, b, -h);
    const double k = fp_rint(h * qinv);
    return __builtin_fma(-k, q, h) + l;
}

// centered reduction: x - rint(x/q)*q, |result| <= q/2 + 1 for |x| <= 2^52.
__device__ __forceinline__ double fp_reduce(double x, double q, double qinv)
{
    return __builtin_fma(-fp_rint(x * qinv), q, x);
}

// 2^52: a double in [2^52, 2^53) holds the integer d - 2^52 in its 52 mantissa bits
#define FP_TWO52 4503599627370496.0

// canonical [0, q) from |x| <= 2^53, as u64.  The centered residue r is shifted into [2^52, 2^53)
// (r + 2^52, or r + q + 2^52 when negative: exact integers below 2^53), whose mantissa field IS
// the residue -- one add and a mask instead of gfx950's multi-instruction f64 -> u64 conversion.
__device__ __forceinline__ uint64_t fp_canon(double x, double q, double qinv)
{
    const double r = fp_reduce(x, q, qinv); // [-q/2 - 1, q/2 + 1]
    const double d = r + (r < 0 ? q + FP_TWO52 : FP_TWO52);
    return (uint64_t)__double_as_longlong(d) & 0x000FFFFFFFFFFFFFull;
}

// exact double of a u64 < 2^53
__device__ __forceinline__ double fp_from_u64(uint64_t x)
{
    return (double)x;
}

// exact double of a u64 < 2^52 (every canonical residue of a prime below 2^51): the exponent of
// 2^52 OR-ed over x gives 2^52 + x, one subtraction leaves x -- instead of two u32 conversions,
// an ldexp and an add
__device__ __forceinline__ double fp_from_u52(uint64_t x)
{
    return __longlong_as_double((long long)(x | 0x4330000000000000ull)) - FP_TWO52;
}

// The packed ModUp intermediate of the FP path (ntt.h tile16, primes q < 2^48) holds the centred
// residue r = x - rint(x/q) q, |r| <= q/2 + 1 < 2^47, as 48-bit two's complement: r + 1.5 2^52 is a
// double in [2^52, 2^53) whose mantissa is r + 2^51, and its low 48 bits are r mod 2^48 -- one add
// instead of fp_canon's select and add.  Only the low 48 bits of the returned word are meaningful.
__device__ __forceinline__ uint64_t fp_to_s48(double x, double q, double qinv)
{
    const double r = fp_reduce(x, q, qinv);
    return (uint64_t)__double_as_longlong(r + 6755399441055744.0); // 1.5 * 2^52
}

// ... and back: flipping bit 47 of r mod 2^48 gives r + 2^47 in [0, 2^48); OR-ed under the exponent
// of 2^52 (one XOR with both) and less 2^52 + 2^47, that is r exactly.
__device__ __forceinline__ double fp_from_s48(uint64_t v48)
{
    return __longlong_as_double((long long)(v48 ^ 0x4330800000000000ull)) - 4644337115725824.0; // 2^52 + 2^47
}

// Forward Cooley-Tukey butterfly (the mathematics of dwthandler.h:122-125).
__device__ __forceinline__ void fwd_bfly_f(double &x, double &y, const TwF w, double q, double qinv)
{
    const double r = fp_mulmod(y, w.x, w.y, q);
    const double u = fp_reduce(x, q, qinv);
    x = u + r;
    y = u - r;
}

// Forward butterfly without reducing x, for q < 2^47: within one pass (<= 8 stages) |x| grows
// from <= 4q by <= 1.5q per stage to <= 16q <= 2^51, which keeps every product's quotient
// estimate within 1 (|y| <= 2^51) -- so the centered reduction of x can be skipped.
__device__ __forceinline__ void fwd_bfly_f_lazy(double &x, double &y, const TwF w, double q)
{
    const double r = fp_mulmod(y, w.x, w.y, q);
    const double u = x;
    x = u + r;
    y = u - r;
}

// Inverse Gentleman-Sande butterfly (dwthandler.h:230-233).  |x|,|y| <= 2q + 1: the
// difference is reduced first so the product's quotient estimate stays within 1.
__device__ __forceinline__ void inv_bfly_f(double &x, double &y, const TwF w, double q, double qinv)
{
    const double s = x + y, d = x - y;
    x = fp_reduce(s, q, qinv);
    y = fp_mulmod(fp_reduce(d, q, qinv), w.x, w.y, q);
}

// Last inverse stage with n^-1 merged (dwthandler.h:273-314): x' = (u+v) n^-1, y' = (u-v) w_last.
__device__ __forceinline__ void inv_bfly_last_f(double &x, double &y, double ninv, double ninv_s, double lw,
                                                double lws, double q, double qinv)
{
    const double s = x + y, d = x - y;
    x = fp_mulmod(fp_reduce(s, q, qinv), ninv, ninv_s, q);
    y = fp_mulmod(fp_reduce(d, q, qinv), lw, lws, q);
}

// One forward stage over the E values of a lane (pairs (e, e+gap), gap bit clear); LAZY (only
// for q < 2^47) drops the reduction of x.
template <int E, bool LAZY, class TwOf>
__device__ __forceinline__ void fwd_stage_f(double (&v)[E], int gap, TwOf tw_of, double q, double qinv)
{
#pragma unroll
    for (int e = 0; e < E; e++)
        if (!(e & gap))
        {
            if (LAZY)
                fwd_bfly_f_lazy(v[e], v[e + gap], *tw_of(e), q);
            else
                fwd_bfly_f(v[e], v[e + gap], *tw_of(e), q, qinv);
        }
}

template <int E, class TwOf>
__device__ __forceinline__ void inv_stage_f(double (&v)[E], int gap, TwOf tw_of, double q, double qinv)
{
#pragma unroll
    for (int e = 0; e < E; e++)
        if (!(e & gap)) inv_bfly_f(v[e], v[e + gap], *tw_of(e), q, qinv);
}
