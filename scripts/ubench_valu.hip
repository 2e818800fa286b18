// Microbenchmark of the VALU instruction classes a 64-bit modular butterfly is built from,
// on gfx950: 32-bit integer multiplies (v_mul_lo_u32 / v_mul_hi_u32 / v_mad_u64_u32),
// 64-bit integer add, FP64 fma / mul, and a full Shoup mulmod.  Prints ops/s per class so the
// NTT butterfly can be priced (DESIGN.md "Arithmetic").
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 4096
#define CHAINS 8

template <int KIND>
__global__ __launch_bounds__(256) void k_bench(uint64_t *out, uint64_t seed)
{
    uint64_t a[CHAINS];
    uint32_t x[CHAINS];
    double d[CHAINS];
    const uint64_t tid = blockIdx.x * 256 + threadIdx.x;
#pragma unroll
    for (int c = 0; c < CHAINS; c++)
    {
        a[c] = seed * (tid + 3 * c + 1) | 1;
        d[c] = (double)(a[c] & 0xffffff) + 0.5;
        x[c] = (uint32_t)a[c];
    }
    const uint32_t m32 = (uint32_t)seed | 3;
    const uint64_t m64 = seed | 0x100000001ull;
    const uint64_t q = 0x7fffffffe0001ull, wq = 0x123456789abcdefull;
    const double dm = 1.0000001, da = 0.5;
    for (int it = 0; it < ITERS; it++)
    {
#pragma unroll
        for (int c = 0; c < CHAINS; c++)
        {
            if (KIND == 0) x[c] = x[c] * (m32 + c) ^ x[c];                                      // v_mul_lo_u32
            if (KIND == 1) x[c] = __umulhi(x[c], m32 + c) ^ x[c];                               // v_mul_hi_u32
            if (KIND == 2) a[c] = (uint64_t)(uint32_t)a[c] * m32 + a[c];                        // v_mad_u64_u32
            if (KIND == 3) a[c] = a[c] + m64;                                                   // 64-bit add
            if (KIND == 4) d[c] = fma(d[c], dm, da);                                            // v_fma_f64
            if (KIND == 5) a[c] = a[c] * (wq + c) - __umul64hi(a[c], wq) * q;                   // Shoup lazy mulmod
            if (KIND == 6) d[c] = d[c] * dm;                                                    // v_mul_f64
            if (KIND == 7) a[c] = (uint64_t)((uint32_t)a[c] * 2654435761u) ^ a[c];              // lo-mul + xor
            if (KIND == 8) d[c] = __builtin_rint(d[c] * dm);                                    // v_mul_f64 + v_rndne_f64
            if (KIND == 9) d[c] = __builtin_fma(d[c], dm, 6755399441055744.0) - 6755399441055744.0; // fma + add (magic rounding)
            if (KIND == 10) d[c] = d[c] + da;                                                   // v_add_f64
        }
    }
    uint64_t s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; c++) s += a[c] + (uint64_t)d[c] + x[c];
    if (s == 42) out[tid] = s;
}

template <int KIND>
static void run(const char *name, uint64_t *out)
{
    const int blocks = 256 * 16;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k_bench<KIND>, dim3(blocks), dim3(256), 0, 0, out, 12345);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k_bench<KIND>, dim3(blocks), dim3(256), 0, 0, out, 12345 + r);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    double ops = 5.0 * blocks * 256.0 * ITERS * CHAINS;
    printf("%-28s %8.3f ms  %9.2f Gop/s (lane-ops)\n", name, ms, ops / (ms * 1e-3) / 1e9);
}

int main()
{
    uint64_t *out;
    (void)hipMalloc(&out, 256 * 16 * 256 * sizeof(uint64_t));
    run<0>("v_mul_lo_u32 (+add)", out);
    run<1>("v_mul_hi_u32 (+add)", out);
    run<2>("v_mad_u64_u32", out);
    run<3>("u64 add", out);
    run<4>("v_fma_f64", out);
    run<5>("shoup_lazy mulmod (64b)", out);
    run<6>("v_mul_f64", out);
    run<7>("mul_lo+xor", out);
    run<8>("v_mul_f64 + v_rndne_f64", out);
    run<9>("v_fma_f64 + v_add_f64 (magic)", out);
    run<10>("v_add_f64", out);
    (void)hipFree(out);
    return 0;
}
