// Batched 64-bit negacyclic NTT / INTT for gfx950.
//
// Mathematically the transforms are SEAL's ntt_negacyclic_harvey(_lazy) and
// inverse_ntt_negacyclic_harvey(_lazy) (util/ntt.cpp:183-209, util/dwthandler.h:94-356):
// Cooley-Tukey forward with psi^rev(i) twiddles, output in bit-reversed order; Gentleman-
// Sande inverse with n^-1 merged into the last stage.  Butterflies are Harvey's lazy forms
// (forward values in [0,4q), inverse in [0,2q)).
//
// Decomposition (not SEAL's loop order): a size-2^K transform is run as two passes.
//   * column pass: stages 0..k1-1.  Sub-transform c (c < 2^(K-k1)) is the strided set
//     x = c + 2^(K-k1) * r, r < 2^k1, and uses twiddles tw[2^s + (r >> (k1-s))].
//   * row pass: stages k1..K-1.  Sub-transform b is the contiguous block x = 2^k2 * b + j and
//     uses twiddles tw[2^s * (2^k1 + b) + (j >> (k2-s))] for local stage s.
// Inside a pass one workgroup (256 lanes) owns S = 256/TPS sub-transforms; each lane holds
// E = R/TPS residues in VGPRs and runs log2(E) butterfly stages in registers, then one LDS
// transpose, then the remaining log2(TPS) stages.  So one HBM round trip per pass and a
// single LDS exchange per pass (two when coalescing needs a transpose back).
//
// Each pass is a template over a Job: Job::view(blockIdx.y) yields the prime, twiddle row,
// and load()/store() hooks.  Key switching and rescale fuse their digit lift / (c - t)*q^-1
// epilogues into these hooks, so the lifted digits never take an extra HBM round trip.
#pragma once
#include "arith.h"

typedef ulonglong2 Tw; // (w, floor(w 2^64 / q))

// Forward Harvey butterfly (dwthandler.h:122-125 with ntt.h:34-65 arithmetic).
__device__ __forceinline__ void fwd_bfly(u64 &x, u64 &y, const Tw w, u64 q, u64 q2)
{
    u64 u = csub(x, q2);
    u64 v = mul_shoup_lazy(y, w.x, w.y, q);
    x = u + v;
    y = u + q2 - v;
}

// Inverse Gentleman-Sande butterfly (dwthandler.h:230-233).
__device__ __forceinline__ void inv_bfly(u64 &x, u64 &y, const Tw w, u64 q, u64 q2)
{
    u64 u = x, v = y;
    x = csub(u + v, q2);
    y = mul_shoup_lazy(u + q2 - v, w.x, w.y, q);
}

// Last inverse stage with n^-1 merged (dwthandler.h:273-314).
__device__ __forceinline__ void inv_bfly_last(u64 &x, u64 &y, const PrimeDev &p)
{
    u64 u = csub(x, p.two_q), v = y;
    x = mul_shoup_lazy(csub(u + v, p.two_q), p.ninv, p.ninv_q, p.q);
    y = mul_shoup_lazy(u + p.two_q - v, p.last_w, p.last_wq, p.q);
}

template <int LOGR, int LOGT>
struct Shape
{
    static constexpr int R = 1 << LOGR;    // sub-transform size
    static constexpr int TPS = 1 << LOGT;  // lanes per sub-transform
    static constexpr int LOGE = LOGR - LOGT;
    static constexpr int E = 1 << LOGE;    // residues per lane
    static constexpr int S = 256 / TPS;    // sub-transforms per workgroup
    static constexpr int LD = R + 1;       // padded LDS row (breaks power-of-two strides)
    static_assert(LOGT <= LOGE, "second phase must stay inside a lane");
};

// ------------------------------------------------------------------ forward, column pass
template <int LOGR, int LOGT, class Job>
__global__ __launch_bounds__(256) void k_fwd_col(Job job, int log_n)
{
    using SH = Shape<LOGR, LOGT>;
    constexpr int E = SH::E, TPS = SH::TPS, LOGE = SH::LOGE, S = SH::S, LD = SH::LD;
    __shared__ u64 lds[S * LD];
    const int tid = threadIdx.x, sl = tid % S, t = tid / S;
    const int logC = log_n - LOGR;
    const u32 c = blockIdx.x * S + sl;
    const auto V = job.view(blockIdx.y);
    if (V.skip) return; // uniform per workgroup, before any barrier
    const u64 q = V.p.q, q2 = V.p.two_q;
    const Tw *tw = V.tw;
    u64 v[E];
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = V.load(c + ((u32)(t + TPS * e) << logC));
#pragma unroll
    for (int s = 0; s < LOGE; s++)
    {
        const int gap = 1 << (LOGE - 1 - s);
#pragma unroll
        for (int e = 0; e < E; e++)
            if (!(e & gap)) fwd_bfly(v[e], v[e + gap], tw[(1 << s) + (e >> (LOGE - s))], q, q2);
    }
#pragma unroll
    for (int e = 0; e < E; e++) lds[sl * LD + t + TPS * e] = v[e];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = lds[sl * LD + E * t + e];
#pragma unroll
    for (int s = LOGE; s < LOGR; s++)
    {
        const int gap = 1 << (LOGR - 1 - s);
#pragma unroll
        for (int e = 0; e < E; e++)
            if (!(e & gap)) fwd_bfly(v[e], v[e + gap], tw[(1 << s) + ((E * t + e) >> (LOGR - s))], q, q2);
    }
#pragma unroll
    for (int e = 0; e < E; e++) V.store(c + ((u32)(E * t + e) << logC), v[e]);
}

// --------------------------------------------------------------------- forward, row pass
template <int LOGR, int LOGT, class Job>
__global__ __launch_bounds__(256) void k_fwd_row(Job job, int log_n)
{
    using SH = Shape<LOGR, LOGT>;
    constexpr int E = SH::E, TPS = SH::TPS, LOGE = SH::LOGE, S = SH::S, LD = SH::LD;
    __shared__ u64 lds[S * LD];
    const int tid = threadIdx.x, t = tid % TPS, sl = tid / TPS;
    const u32 b = blockIdx.x * S + sl;
    const u32 base = b << LOGR;
    const u32 rb = (1u << (log_n - LOGR)) + b; // 2^k1 + b
    const auto V = job.view(blockIdx.y);
    if (V.skip) return; // uniform per workgroup, before any barrier
    const u64 q = V.p.q, q2 = V.p.two_q;
    const Tw *tw = V.tw;
    u64 v[E];
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = V.load(base + t + TPS * e);
#pragma unroll
    for (int s = 0; s < LOGE; s++)
    {
        const int gap = 1 << (LOGE - 1 - s);
#pragma unroll
        for (int e = 0; e < E; e++)
            if (!(e & gap)) fwd_bfly(v[e], v[e + gap], tw[(rb << s) + (e >> (LOGE - s))], q, q2);
    }
#pragma unroll
    for (int e = 0; e < E; e++) lds[sl * LD + t + TPS * e] = v[e];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = lds[sl * LD + E * t + e];
#pragma unroll
    for (int s = LOGE; s < LOGR; s++)
    {
        const int gap = 1 << (LOGR - 1 - s);
#pragma unroll
        for (int e = 0; e < E; e++)
            if (!(e & gap)) fwd_bfly(v[e], v[e + gap], tw[(rb << s) + ((E * t + e) >> (LOGR - s))], q, q2);
    }
    // transpose back so stores (and epilogue reads) are coalesced
#pragma unroll
    for (int e = 0; e < E; e++) lds[sl * LD + E * t + e] = v[e];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; e++) V.store(base + t + TPS * e, lds[sl * LD + t + TPS * e]);
}

// --------------------------------------------------------------------- inverse, row pass
template <int LOGR, int LOGT, class Job>
__global__ __launch_bounds__(256) void k_inv_row(Job job, int log_n)
{
    using SH = Shape<LOGR, LOGT>;
    constexpr int E = SH::E, TPS = SH::TPS, LOGE = SH::LOGE, S = SH::S, LD = SH::LD;
    __shared__ u64 lds[S * LD];
    const int tid = threadIdx.x, t = tid % TPS, sl = tid / TPS;
    const u32 b = blockIdx.x * S + sl;
    const u32 base = b << LOGR;
    const u32 rb = (1u << (log_n - LOGR)) + b;
    const auto V = job.view(blockIdx.y);
    if (V.skip) return; // uniform per workgroup, before any barrier
    const u64 q = V.p.q, q2 = V.p.two_q;
    const Tw *tw = V.tw;
    u64 v[E];
#pragma unroll
    for (int e = 0; e < E; e++) lds[sl * LD + t + TPS * e] = V.load(base + t + TPS * e);
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = lds[sl * LD + E * t + e];
#pragma unroll
    for (int s = LOGR - 1; s >= LOGE; s--)
    {
        const int gap = 1 << (LOGR - 1 - s);
#pragma unroll
        for (int e = 0; e < E; e++)
            if (!(e & gap)) inv_bfly(v[e], v[e + gap], tw[(rb << s) + ((E * t + e) >> (LOGR - s))], q, q2);
    }
#pragma unroll
    for (int e = 0; e < E; e++) lds[sl * LD + E * t + e] = v[e];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = lds[sl * LD + t + TPS * e];
#pragma unroll
    for (int s = LOGE - 1; s >= 0; s--)
    {
        const int gap = 1 << (LOGE - 1 - s);
#pragma unroll
        for (int e = 0; e < E; e++)
            if (!(e & gap)) inv_bfly(v[e], v[e + gap], tw[(rb << s) + (e >> (LOGE - s))], q, q2);
    }
#pragma unroll
    for (int e = 0; e < E; e++) V.store(base + t + TPS * e, v[e]);
}

// ------------------------------------------------------------------ inverse, column pass
template <int LOGR, int LOGT, class Job>
__global__ __launch_bounds__(256) void k_inv_col(Job job, int log_n)
{
    using SH = Shape<LOGR, LOGT>;
    constexpr int E = SH::E, TPS = SH::TPS, LOGE = SH::LOGE, S = SH::S, LD = SH::LD;
    __shared__ u64 lds[S * LD];
    const int tid = threadIdx.x, sl = tid % S, t = tid / S;
    const int logC = log_n - LOGR;
    const u32 c = blockIdx.x * S + sl;
    const auto V = job.view(blockIdx.y);
    if (V.skip) return; // uniform per workgroup, before any barrier
    const u64 q = V.p.q, q2 = V.p.two_q;
    const Tw *tw = V.tw;
    u64 v[E];
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = V.load(c + ((u32)(E * t + e) << logC));
#pragma unroll
    for (int s = LOGR - 1; s >= LOGE; s--)
    {
        const int gap = 1 << (LOGR - 1 - s);
#pragma unroll
        for (int e = 0; e < E; e++)
            if (!(e & gap)) inv_bfly(v[e], v[e + gap], tw[(1 << s) + ((E * t + e) >> (LOGR - s))], q, q2);
    }
#pragma unroll
    for (int e = 0; e < E; e++) lds[sl * LD + E * t + e] = v[e];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = lds[sl * LD + t + TPS * e];
#pragma unroll
    for (int s = LOGE - 1; s >= 1; s--)
    {
        const int gap = 1 << (LOGE - 1 - s);
#pragma unroll
        for (int e = 0; e < E; e++)
            if (!(e & gap)) inv_bfly(v[e], v[e + gap], tw[(1 << s) + (e >> (LOGE - s))], q, q2);
    }
    {
        constexpr int gap = E / 2;
#pragma unroll
        for (int e = 0; e < gap; e++) inv_bfly_last(v[e], v[e + gap], V.p);
    }
#pragma unroll
    for (int e = 0; e < E; e++) V.store(c + ((u32)(t + TPS * e) << logC), v[e]);
}

// --------------------------------------------------------------------------- dispatch
// Pass split: column pass takes ceil(K/2) stages, row pass floor(K/2).
enum PassKind
{
    FWD_COL,
    FWD_ROW,
    INV_ROW,
    INV_COL
};

template <int PASS, int LOGR, class Job>
static inline void launch_pass(const Job &job, int log_n, int jobs, hipStream_t st)
{
    constexpr int LOGT = LOGR <= 7 ? 3 : 4;
    using SH = Shape<LOGR, LOGT>;
    const int subs = 1 << (log_n - LOGR);
    dim3 grid(subs / SH::S, jobs);
    if (PASS == FWD_COL) hipLaunchKernelGGL((k_fwd_col<LOGR, LOGT, Job>), grid, dim3(256), 0, st, job, log_n);
    if (PASS == FWD_ROW) hipLaunchKernelGGL((k_fwd_row<LOGR, LOGT, Job>), grid, dim3(256), 0, st, job, log_n);
    if (PASS == INV_ROW) hipLaunchKernelGGL((k_inv_row<LOGR, LOGT, Job>), grid, dim3(256), 0, st, job, log_n);
    if (PASS == INV_COL) hipLaunchKernelGGL((k_inv_col<LOGR, LOGT, Job>), grid, dim3(256), 0, st, job, log_n);
}

template <int PASS, class Job>
static inline void launch_col(const Job &job, int log_n, int jobs, hipStream_t st)
{
    switch ((log_n + 1) / 2)
    {
    case 6: launch_pass<PASS, 6>(job, log_n, jobs, st); break;
    case 7: launch_pass<PASS, 7>(job, log_n, jobs, st); break;
    case 8: launch_pass<PASS, 8>(job, log_n, jobs, st); break;
    }
}

template <int PASS, class Job>
static inline void launch_row(const Job &job, int log_n, int jobs, hipStream_t st)
{
    switch (log_n / 2)
    {
    case 6: launch_pass<PASS, 6>(job, log_n, jobs, st); break;
    case 7: launch_pass<PASS, 7>(job, log_n, jobs, st); break;
    case 8: launch_pass<PASS, 8>(job, log_n, jobs, st); break;
    }
}

template <class Job> static inline void fwd_col(const Job &j, int log_n, int jobs, hipStream_t st) { launch_col<FWD_COL>(j, log_n, jobs, st); }
template <class Job> static inline void fwd_row(const Job &j, int log_n, int jobs, hipStream_t st) { launch_row<FWD_ROW>(j, log_n, jobs, st); }
template <class Job> static inline void inv_row(const Job &j, int log_n, int jobs, hipStream_t st) { launch_row<INV_ROW>(j, log_n, jobs, st); }
template <class Job> static inline void inv_col(const Job &j, int log_n, int jobs, hipStream_t st) { launch_col<INV_COL>(j, log_n, jobs, st); }
