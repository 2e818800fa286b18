// Butterfly throughput: SEAL-style integer Harvey/Shoup butterflies (arith.h/ntt.h) against the
// FP64-FMA butterflies (fparith.h), on register-resident data (8 residues per lane, 3 stages per
// round), plus a correctness check of the FP64 path against the integer one for q ~ 2^51 and
// q ~ 2^46.  Build: hipcc -O3 --offload-arch=gfx950 -I fhe-gpt-2_amd/csrc scripts/ubench_bfly.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "ntt.h"
#include "fparith.h"

#define ROUNDS 512
#define E 8

__global__ __launch_bounds__(256) void k_int(uint64_t *data, const Tw *tw, PrimeDev p, int rounds)
{
    const size_t base = ((size_t)blockIdx.x * 256 + threadIdx.x) * E;
    u64 v[E];
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = data[base + e];
    for (int it = 0; it < rounds; it++)
    {
#pragma unroll
        for (int s = 0; s < 3; s++)
            fwd_stage<E>(v, 1 << (2 - s), [&](int e) { return &tw[(1 << s) + (e >> (3 - s)) + 8 * (it & 7)]; }, p.q,
                         p.two_q);
    }
#pragma unroll
    for (int e = 0; e < E; e++)
    {
        u64 x = v[e];
        x = csub(x, p.two_q);
        x = csub(x, p.q);
        data[base + e] = x;
    }
}

__global__ __launch_bounds__(256) void k_fp(uint64_t *data, const TwF *tw, PrimeF p, int rounds)
{
    const size_t base = ((size_t)blockIdx.x * 256 + threadIdx.x) * E;
    double v[E];
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = fp_from_u64(data[base + e]);
    for (int it = 0; it < rounds; it++)
    {
#pragma unroll
        for (int s = 0; s < 3; s++)
        {
            const int gap = 1 << (2 - s);
#pragma unroll
            for (int e = 0; e < E; e++)
                if (!(e & gap)) fwd_bfly_f(v[e], v[e + gap], tw[(1 << s) + (e >> (3 - s)) + 8 * (it & 7)], p.q, p.qinv);
        }
    }
#pragma unroll
    for (int e = 0; e < E; e++) data[base + e] = fp_canon(v[e], p.q, p.qinv);
}

static uint64_t mulmod_h(uint64_t a, uint64_t b, uint64_t q)
{
    return (uint64_t)((unsigned __int128)a * b % q);
}

int main()
{
    const int blocks = 256 * 16;
    const size_t cnt = (size_t)blocks * 256 * E;
    uint64_t *h = (uint64_t *)malloc(cnt * 8), *g1 = (uint64_t *)malloc(cnt * 8), *g2 = (uint64_t *)malloc(cnt * 8);
    uint64_t *d;
    Tw *dtw;
    TwF *dtf;
    (void)hipMalloc(&d, cnt * 8);
    (void)hipMalloc(&dtw, 128 * sizeof(Tw));
    (void)hipMalloc(&dtf, 128 * sizeof(TwF));
    const uint64_t qs[2] = { 2251799813554177ull /* < 2^51 */, 70368744210433ull /* ~2^46 */ };
    for (int qi = 0; qi < 2; qi++)
    {
        const uint64_t q = qs[qi];
        PrimeDev p = {};
        p.q = q;
        p.two_q = 2 * q;
        p.four_q = 4 * q;
        PrimeF pf = { (double)q, 1.0 / (double)q, 0, 0, 0, 0 };
        Tw tw[128];
        TwF tf[128];
        uint64_t s = 88172645463325252ull + qi;
        for (int i = 0; i < 128; i++)
        {
            s ^= s << 13, s ^= s >> 7, s ^= s << 17;
            const uint64_t w = s % q;
            tw[i].x = w;
            tw[i].y = (uint64_t)(((unsigned __int128)w << 64) / q);
            tf[i].x = (double)w;
            tf[i].y = (double)w / (double)q;
        }
        for (size_t i = 0; i < cnt; i++)
        {
            s ^= s << 13, s ^= s >> 7, s ^= s << 17;
            h[i] = s % q;
        }
        (void)hipMemcpy(dtw, tw, sizeof(tw), hipMemcpyHostToDevice);
        (void)hipMemcpy(dtf, tf, sizeof(tf), hipMemcpyHostToDevice);
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        float ms_i = 0, ms_f = 0;
        // correctness (few rounds) then timing (many)
        for (int pass = 0; pass < 2; pass++)
        {
            const int rounds = pass ? ROUNDS : 5;
            (void)hipMemcpy(d, h, cnt * 8, hipMemcpyHostToDevice);
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k_int, dim3(blocks), dim3(256), 0, 0, d, dtw, p, rounds);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms_i, e0, e1);
            (void)hipMemcpy(g1, d, cnt * 8, hipMemcpyDeviceToHost);
            (void)hipMemcpy(d, h, cnt * 8, hipMemcpyHostToDevice);
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k_fp, dim3(blocks), dim3(256), 0, 0, d, dtf, pf, rounds);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms_f, e0, e1);
            (void)hipMemcpy(g2, d, cnt * 8, hipMemcpyDeviceToHost);
            size_t bad = 0;
            for (size_t i = 0; i < cnt; i++) bad += g1[i] != g2[i];
            if (pass == 0)
            {
                // host check of the first lane's 8 values for one round of the integer path
                printf("q=%llu correctness: %zu mismatches of %zu (int vs fp, %d rounds)\n", (unsigned long long)q,
                       bad, cnt, rounds);
            }
            else
            {
                const double bfly = (double)blocks * 256 * rounds * 3 * (E / 2);
                printf("q=%llu  int: %.3f ms (%.1f Gbfly/s)   fp64: %.3f ms (%.1f Gbfly/s)   speedup %.2fx  mismatches %zu\n",
                       (unsigned long long)q, ms_i, bfly / ms_i / 1e6, ms_f, bfly / ms_f / 1e6, ms_i / ms_f, bad);
            }
        }
        (void)mulmod_h;
    }
    return 0;
}
