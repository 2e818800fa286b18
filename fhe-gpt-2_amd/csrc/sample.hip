// On-device sampling of the random polynomials of key generation and encryption
// (SEAL/util/rlwe.cpp sample_poly_uniform / sample_poly_ternary / sample_poly_normal), written
// straight into RNS form on the GPU: no host loops, no host->device upload, no stream sync.
//
// Randomness: Philox4x32-10 (Salmon et al., SC'11), counter = (element index, polynomial tag),
// key = 64-bit seed.  Distributions:
//   uniform mod q_l : 128 random bits reduced by Barrett (statistical distance < q / 2^128);
//   ternary         : 64 random bits mod 3, minus 1;
//   normal          : Box-Muller, sigma = 3.2, rejected outside 6 sigma (ClippedNormal),
//                     truncated to an integer as sample_poly_normal does.
// These are SEAL's distributions, not SEAL's bits (SEAL uses Blake2xb): keys and ciphertexts
// differ from SEAL's for the same seed; every operation on them is bit-exact.
#include <hip/hip_runtime.h>

#include "../../include/mhe.h"
#include "arith.h"

int mhe_internal_fail(int code, const char *msg);
int mhe_internal_primes(mhe_ctx *c, const PrimeDev **dev, const uint64_t **host, int *count, int *log_n);

namespace
{
__device__ __forceinline__ void philox10(u32 (&ctr)[4], u32 k0, u32 k1)
{
#pragma unroll
    for (int r = 0; r < 10; r++)
    {
        const u64 p0 = (u64)0xD2511F53u * ctr[0], p1 = (u64)0xCD9E8D57u * ctr[2];
        const u32 h0 = (u32)(p0 >> 32), l0 = (u32)p0, h1 = (u32)(p1 >> 32), l1 = (u32)p1;
        const u32 n0 = h1 ^ ctr[1] ^ k0, n2 = h0 ^ ctr[3] ^ k1;
        ctr[0] = n0;
        ctr[1] = l1;
        ctr[2] = n2;
        ctr[3] = l0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// 128 random bits for (element, tag, draw)
__device__ __forceinline__ void rand128(u64 idx, u64 tag, u32 draw, u64 seed, u64 &lo, u64 &hi)
{
    u32 ctr[4] = { (u32)idx, (u32)(idx >> 32) ^ (draw << 24), (u32)tag, (u32)(tag >> 32) };
    philox10(ctr, (u32)seed, (u32)(seed >> 32));
    lo = ((u64)ctr[1] << 32) | ctr[0];
    hi = ((u64)ctr[3] << 32) | ctr[2];
}

enum Kind
{
    UNIFORM = 0,
    TERNARY = 1,
    NORMAL = 2
};

__global__ void k_sample_uniform(u64 *out, const PrimeDev *primes, int limbs, int log_n, u64 seed, u64 tag)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t total = (size_t)limbs << log_n;
    if (i >= total) return;
    u64 lo, hi;
    rand128(i, tag, 0, seed, lo, hi);
    out[i] = barrett128(lo, hi, primes[i >> log_n]);
}

__global__ void k_sample_small(u64 *out, const PrimeDev *primes, int limbs, int log_n, int kind, u64 seed, u64 tag)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t n = (size_t)1 << log_n;
    if (i >= n) return;
    long long v;
    if (kind == TERNARY)
    {
        u64 lo, hi;
        rand128(i, tag, 0, seed, lo, hi);
        v = (long long)(lo % 3) - 1;
    }
    else
    {
        // Box-Muller with rejection outside 6 sigma (rare: p ~ 2e-9); every draw uses its own
        // counter, so the loop is bounded in practice and deterministic
        const double sigma = 3.2, bound = 6 * 3.2, two_pi = 6.283185307179586476925286766559;
        double z = 0;
        for (u32 d = 0; d < 64; d++)
        {
            u64 lo, hi;
            rand128(i, tag, d, seed, lo, hi);
            const double u1 = ((lo >> 11) + 1) * 0x1.0p-53; // (0, 1]
            const double u2 = (hi >> 11) * 0x1.0p-53;       // [0, 1)
            z = sigma * sqrt(-2.0 * log(u1)) * cos(two_pi * u2);
            if (fabs(z) <= bound) break;
            z = 0;
        }
        v = (long long)z; // truncation, as sample_poly_normal's static_cast<int64_t>
    }
    for (int l = 0; l < limbs; l++)
    {
        const u64 q = primes[l].q;
        out[((size_t)l << log_n) + i] = v >= 0 ? (u64)v : q - (u64)(-v);
    }
}
} // namespace

extern "C" __attribute__((visibility("default"))) int mhe_sample_poly(mhe_ctx *c, uint64_t *out, int limbs, int kind,
                                                                     uint64_t seed, uint64_t tag, void *stream)
{
    const PrimeDev *primes;
    const uint64_t *q;
    int K, log_n;
    if (mhe_internal_primes(c, &primes, &q, &K, &log_n)) return mhe_internal_fail(MHE_ERR_ARG, "context is not valid");
    if (!out || limbs < 1 || limbs > K) return mhe_internal_fail(MHE_ERR_ARG, "invalid polynomial arguments");
    hipStream_t st = (hipStream_t)stream;
    if (kind == UNIFORM)
    {
        const size_t total = (size_t)limbs << log_n;
        hipLaunchKernelGGL(k_sample_uniform, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, out, primes,
                           limbs, log_n, seed, tag);
    }
    else if (kind == TERNARY || kind == NORMAL)
    {
        const size_t n = (size_t)1 << log_n;
        hipLaunchKernelGGL(k_sample_small, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out, primes, limbs,
                           log_n, kind, seed, tag);
    }
    else
        return mhe_internal_fail(MHE_ERR_ARG, "unknown distribution");
    if (hipGetLastError() != hipSuccess) return mhe_internal_fail(MHE_ERR_DEVICE, "sampling kernel launch failed");
    return MHE_OK;
}
