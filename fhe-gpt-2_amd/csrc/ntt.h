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
#include <type_traits>

#include "arith.h"
#include "fparith.h"

// Batched launches: one launch of a key-switch / rescale kernel serves up to MHE_MAXB independent
// ciphertexts of the same level (per-entry pointers in the kernel arguments, entry = a grid
// dimension), so small-level work from independent rotations or images fills the chip.
#ifndef MHE_MAXB
#define MHE_MAXB 8
#endif


// Streaming (non-temporal) access for the key-switch streams, selected at build time (MHE_NT bit 0:
// ModUp intermediate stores, bit 1: key loads, bit 2: intermediate loads in the fused MAC).
#ifndef MHE_NT
#define MHE_NT 5 // measured: +5% HMult/s (scripts/gpu_nt.sh; key loads NT lost 5%)
#endif
template <int BIT, class T>
__device__ __forceinline__ void st_nt(T *p, T v)
{
    if constexpr ((MHE_NT >> BIT) & 1)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}
template <int BIT, class T>
__device__ __forceinline__ T ld_nt(const T *p)
{
    if constexpr ((MHE_NT >> BIT) & 1)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}

// Packed ModUp intermediate (key switch at n = 2^16, output prime q < 2^48): the canonical
// residues need 48 bits, so a limb slot holds a 32-bit plane [n] followed by a 16-bit plane [n]
// (6 of its 8 bytes per residue).  Both planes are laid out as 16 x 16 tiles of the 256 x 256
// (row = index >> 8, column = index & 255) matrix the two NTT passes see: a column-pass lane
// writes 16 consecutive rows of one column and a row-pass wave reads whole tile rows, so both
// sides move contiguous 64-128 B runs.
__device__ __forceinline__ u32 tile16(u32 idx)
{
    const u32 r = idx >> 8, c = idx & 255;
    return ((((r >> 4) << 4) | (c >> 4)) << 8) | ((r & 15) << 4) | (c & 15);
}
// Prepared key (mhe_key_prepare): every limb slot of a prime below 2^51 (the FP64 path's primes)
// holds its residues as IEEE doubles -- the FP64 key MAC's operand, loaded with no unpacking (-0.0
// for a zero residue).  Every such word is >= 2^61, which no residue of a SEAL key reaches (primes
// of at most 60 bits), so the key MAC tells a prepared slot from SEAL's layout by any one word.
#define KEY_PREP_MIN (1ull << 61)
__host__ __device__ __forceinline__ bool key_word_prepared(u64 w)
{
    return w >= KEY_PREP_MIN;
}
// The second prepared format, for keys streamed by one ciphertext at a time (where the MAC's key
// bytes matter more than its unpacking): a slot of a prime below 2^48 holds a 32-bit plane [n], a
// 16-bit plane [n] and, in its unused last quarter, this tag (6 B per residue).
#define KEY_PACK_TAG 0xF0E1D2C3B4A59687ull
// a slot's format from its last word: 0 SEAL's layout, 1 doubles, 2 48-bit planes
__host__ __device__ __forceinline__ int key_slot_format(u64 last_word)
{
    return last_word == KEY_PACK_TAG ? 2 : key_word_prepared(last_word) ? 1 : 0;
}
// a prepared word as the residue's double / as the u64 residue (integer kernels): 2^52 + x holds x
// in its mantissa field (-0.0 + 2^52 = 2^52)
__device__ __forceinline__ double key_word_f(u64 w)
{
    return __longlong_as_double((long long)w);
}
__device__ __forceinline__ u64 key_word_u(u64 w)
{
    return (u64)__double_as_longlong(__longlong_as_double((long long)w) + 4503599627370496.0) & 0x000FFFFFFFFFFFFFull;
}
// The 16-bit plane pairs rows instead: in a tile, u32 word (r/2, c) holds the high halves of rows
// r and r+1 of column c (u16 index returned), so a column-pass lane, which holds both rows, writes
// one u32 per row pair and 16 lanes fill a whole 64-byte segment (2-byte stores left 32-byte
// half-segments and ~0.17 GB of extra write traffic per HMult).
__device__ __forceinline__ u32 tile16h(u32 idx)
{
    const u32 r = idx >> 8, c = idx & 255;
    return ((((r >> 4) << 4) | (c >> 4)) << 8) | (((r & 15) >> 1) << 5) | ((c & 15) << 1) | (r & 1);
}
__device__ __forceinline__ bool inter_packed(int pack, u64 q)
{
    return pack && q < (1ull << 48);
}

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

// One forward stage on the E residues of a lane: butterflies (e, e+gap) for every e with the
// gap bit clear, twiddle pointer tw_of(e).  The E/2 twiddle products are computed as a batch.
template <int E, class TwOf>
__device__ __forceinline__ void fwd_stage(u64 (&v)[E], int gap, TwOf tw_of, u64 q, u64 q2)
{
    constexpr int NB = E / 2;
    u64 y[NB], m[NB];
    const Tw *w[NB];
    int k = 0;
#pragma unroll
    for (int e = 0; e < E; e++)
        if (!(e & gap))
        {
            y[k] = v[e + gap];
            w[k] = tw_of(e);
            k++;
        }
    mul_shoup_lazy_batch<NB>(y, w, q, m);
    k = 0;
#pragma unroll
    for (int e = 0; e < E; e++)
        if (!(e & gap))
        {
            const u64 u = csub(v[e], q2);
            v[e] = u + m[k];
            v[e + gap] = u + q2 - m[k];
            k++;
        }
}

// One inverse (Gentleman-Sande) stage, batched like fwd_stage.
template <int E, class TwOf>
__device__ __forceinline__ void inv_stage(u64 (&v)[E], int gap, TwOf tw_of, u64 q, u64 q2)
{
    constexpr int NB = E / 2;
    u64 y[NB], m[NB];
    const Tw *w[NB];
    int k = 0;
#pragma unroll
    for (int e = 0; e < E; e++)
        if (!(e & gap))
        {
            const u64 a = v[e], b = v[e + gap];
            v[e] = csub(a + b, q2);
            y[k] = a + q2 - b;
            w[k] = tw_of(e);
            k++;
        }
    mul_shoup_lazy_batch<NB>(y, w, q, m);
    k = 0;
#pragma unroll
    for (int e = 0; e < E; e++)
        if (!(e & gap)) v[e + gap] = m[k++];
}

// Arithmetic policy of a transform pass.  NttArith<false>: SEAL's integer Harvey butterflies
// (u64 values in lazy ranges).  NttArith<true>: FP64-FMA butterflies (fparith.h) for primes
// < 2^51, values held as doubles inside the pass; loads convert exact u64 -> double and stores
// hand canonical u64 to the job's store hook (canonical lies inside every lazy range the hooks
// accept).  The FP twiddle tables mirror the integer ones entry for entry (16 B each), so the
// job's integer twiddle pointer plus a fixed byte offset addresses the FP table.
template <bool FP>
struct NttArith;

template <>
struct NttArith<false>
{
    using T = u64;
    using TW = Tw;
    u64 q, q2;
    const Tw *tw;
    __device__ NttArith(const PrimeDev &p, const Tw *t, long long) : q(p.q), q2(p.two_q), tw(t) {}
    __device__ T in(u64 x) const { return x; }
    __device__ T in52(u64 x) const { return x; }
    __device__ u64 out(T x) const { return x; }
    __device__ u64 canon(T x) const { return csub(csub(x, q2), q); }
    template <int E, class Ix>
    __device__ void fwd(T (&v)[E], int gap, Ix ix) const
    {
        fwd_stage<E>(v, gap, [&](int e) { return &tw[ix(e)]; }, q, q2);
    }
    template <int E, class Ix>
    __device__ void fwd_tab(T (&v)[E], int gap, const TW *tab, Ix ix) const
    {
        fwd_stage<E>(v, gap, [&](int e) { return &tab[ix(e)]; }, q, q2);
    }
    template <int E, class Ix>
    __device__ void inv(T (&v)[E], int gap, Ix ix) const
    {
        inv_stage<E>(v, gap, [&](int e) { return &tw[ix(e)]; }, q, q2);
    }
    template <int E, class Ix>
    __device__ void inv_tab(T (&v)[E], int gap, const TW *tab, Ix ix) const
    {
        inv_stage<E>(v, gap, [&](int e) { return &tab[ix(e)]; }, q, q2);
    }
    __device__ void inv_last(T &x, T &y, const PrimeDev &p) const { inv_bfly_last(x, y, p); }
};

template <bool LAZY>
struct NttArithF
{
    using T = double;
    using TW = TwF;
    double q, qinv;
    const TwF *tw;
    __device__ NttArithF(const PrimeDev &p, const Tw *t, long long delta)
        : q((double)p.q), qinv(1.0 / (double)p.q), tw(reinterpret_cast<const TwF *>(reinterpret_cast<const char *>(t) + delta))
    {
    }
    __device__ T in(u64 x) const { return (double)x; }
    __device__ T in52(u64 x) const { return fp_from_u52(x); } // x < 2^52: a canonical residue
    __device__ u64 out(T x) const { return fp_canon(x, q, qinv); }
    __device__ u64 canon(T x) const { return fp_canon(x, q, qinv); }
    template <int E, class Ix>
    __device__ void fwd(T (&v)[E], int gap, Ix ix) const
    {
        fwd_stage_f<E, LAZY>(v, gap, [&](int e) { return &tw[ix(e)]; }, q, qinv);
    }
    template <int E, class Ix>
    __device__ void fwd_tab(T (&v)[E], int gap, const TW *tab, Ix ix) const
    {
        fwd_stage_f<E, LAZY>(v, gap, [&](int e) { return &tab[ix(e)]; }, q, qinv);
    }
    template <int E, class Ix>
    __device__ void inv(T (&v)[E], int gap, Ix ix) const
    {
        inv_stage_f<E>(v, gap, [&](int e) { return &tw[ix(e)]; }, q, qinv);
    }
    template <int E, class Ix>
    __device__ void inv_tab(T (&v)[E], int gap, const TW *tab, Ix ix) const
    {
        inv_stage_f<E>(v, gap, [&](int e) { return &tab[ix(e)]; }, q, qinv);
    }
    __device__ void inv_last(T &x, T &y, const PrimeDev &p) const
    {
        const double ni = (double)p.ninv, lw = (double)p.last_w;
        inv_bfly_last_f(x, y, ni, ni / q, lw, lw / q, q, qinv);
    }
};

// FP64 with the reduction of x in every forward stage (any q < 2^51).  The two hot key-switch
// kernels pick NttArithF<true> per workgroup when q < 2^47 (fparith.h fwd_bfly_f_lazy).
template <>
struct NttArith<true> : NttArithF<false>
{
    using NttArithF<false>::NttArithF;
};

// Per-launch arithmetic selection: fp = every prime of the context is < 2^51; the deltas are
// the byte offsets from the integer to the FP forward / inverse twiddle tables.
struct NttMode
{
    int fp = 0;
    long long dfwd = 0, dinv = 0;
};

// A block of R = 2^LOGR residues is held by TPS = R/8 <= 32 lanes, i.e. inside one wave, so
// its LDS transposes never cross waves: a wave's LDS accesses execute in program order, and
// only the compiler must be kept from moving them across each other.
__device__ __forceinline__ void wave_lds_fence()
{
    asm volatile("" ::: "memory");
}

// Workgroup barrier on LDS only (s_waitcnt lgkmcnt(0) + s_barrier): __syncthreads() also waits for
// every outstanding global memory operation (vmcnt(0)), which serialises a kernel's stores with the
// compute that follows them (cdna_hip_programming.md §8).
__device__ __forceinline__ void lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
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
template <int LOGR, int LOGT, class Job, bool FP>
__global__ __launch_bounds__(256) void k_fwd_col(Job job, int log_n, long long twd)
{
    using SH = Shape<LOGR, LOGT>;
    using A = NttArith<FP>;
    using T = typename A::T;
    constexpr int E = SH::E, TPS = SH::TPS, LOGE = SH::LOGE, S = SH::S, LD = SH::LD;
    __shared__ T lds[S * LD];
    const int tid = threadIdx.x, sl = tid % S, t = tid / S;
    const int logC = log_n - LOGR;
    const u32 c = blockIdx.x * S + sl;
    const auto V = job.view(blockIdx.y);
    if (V.skip) return; // uniform per workgroup, before any barrier
    const A ar(V.p, V.tw, twd);
    T v[E];
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = ar.in(V.load(c + ((u32)(t + TPS * e) << logC)));
    // the per-lane twiddles of the first two stages after the barrier, loaded with the data (the
    // barrier would otherwise hold their loads back; cf. k_fwd_row): entries (1 << s) + (E t >> (LOGR - s)) + j
    using TWT = typename A::TW;
    constexpr int C0 = E >> (LOGR - LOGE), C1 = E >> (LOGR - LOGE - 1);
    TWT p0[C0], p1[C1];
#pragma unroll
    for (int j = 0; j < C0; j++) p0[j] = ar.tw[(1 << LOGE) + ((E * t) >> (LOGR - LOGE)) + j];
#pragma unroll
    for (int j = 0; j < C1; j++) p1[j] = ar.tw[(1 << (LOGE + 1)) + ((E * t) >> (LOGR - LOGE - 1)) + j];
#pragma unroll
    for (int s = 0; s < LOGE; s++)
        ar.template fwd<E>(v, 1 << (LOGE - 1 - s), [&](int e) { return (1 << s) + (e >> (LOGE - s)); });
#pragma unroll
    for (int e = 0; e < E; e++) lds[sl * LD + t + TPS * e] = v[e];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = lds[sl * LD + E * t + e];
#pragma unroll
    for (int s = LOGE; s < LOGR; s++)
    {
        if (s == LOGE)
            ar.template fwd_tab<E>(v, 1 << (LOGR - 1 - s), p0, [&](int e) { return e >> (LOGR - s); });
        else if (s == LOGE + 1)
            ar.template fwd_tab<E>(v, 1 << (LOGR - 1 - s), p1, [&](int e) { return e >> (LOGR - s); });
        else
            ar.template fwd<E>(v, 1 << (LOGR - 1 - s), [&](int e) { return (1 << s) + ((E * t + e) >> (LOGR - s)); });
    }
#pragma unroll
    for (int e = 0; e < E; e++) V.store(c + ((u32)(E * t + e) << logC), ar.out(v[e]));
}

// Row-pass epilogue operands.  A View whose store() reads other buffers (the ModDown / rescale
// epilogues read acc and ct at the stored index) declares `Pre` and pre(x): the pass loads those
// operands for all its E indices right after its own loads, so their latency hides behind the
// butterflies, and hands them to store(x, v, pre).  Without it each store's loads wait for the
// previous store (the compiler cannot move a load above a store that may alias it): E serialised
// HBM round trips per lane at the end of the kernel.
#ifndef MHE_ROW_PRE
#define MHE_ROW_PRE 1
#endif
template <class V, class = void>
struct PreOf
{
    using type = char;
    static constexpr bool value = false;
};
template <class V>
struct PreOf<V, std::void_t<typename V::Pre>>
{
    using type = typename V::Pre;
    static constexpr bool value = MHE_ROW_PRE != 0;
};

// A View with `static constexpr bool brev = true` stores position x of each 256-slot block from slot
// brev8(x & 255) of the block (hoisted rotations, hoist.h): with 256-slot rows (LOGR = 8) the row
// pass reads its LDS row at the bit-reversed index and its stores stay contiguous.
template <class V, class = void>
struct BrevOf
{
    static constexpr bool value = false;
};
template <class V>
struct BrevOf<V, std::void_t<decltype(V::brev)>>
{
    static constexpr bool value = V::brev;
};
__device__ __forceinline__ u32 brev8_ntt(u32 x)
{
    return __builtin_bitreverse32(x) >> 24;
}

// LDS image of a row pass's transposes.  The in-lane phase writes position t + TPS e and the
// cross-lane phase reads E t + e (and back); with a plain padded row the second pattern puts the
// 16 lanes of a sub-transform on a stride of E 8-byte words, an 8-way bank conflict at LOGR = 8
// (SQ_LDS_BANK_CONFLICT 6.5x the LDS busy cycles, profiles/r03k).  XOR-ing the low LOGE bits with
// the high ones and a row pitch of R + TPS words makes both patterns conflict-free for every row
// shape (bank model of MI355X_MICROARCH.md §LDS: 64 banks, 32-lane groups for ds_*_b64).
#ifndef MHE_ROW_SWZ
#define MHE_ROW_SWZ 1
#endif
template <int LOGR, int LOGT>
struct RowLds
{
    static constexpr int R = 1 << LOGR, TPS = 1 << LOGT, LOGE = LOGR - LOGT, E = 1 << LOGE;
    static constexpr int LD = MHE_ROW_SWZ ? R + TPS : R + 1;
    __device__ static __forceinline__ int at(int sl, int p)
    {
        return sl * LD + (MHE_ROW_SWZ ? (p ^ ((p >> LOGE) & (E - 1))) : p);
    }
};

// Bijective LDS index swizzle: conflict-free ds_write_b64 / ds_read_b64 for all three
// transpose layouts (bank model of MI355X_MICROARCH.md §LDS; checked in scripts).
__device__ __forceinline__ u32 swz(u32 r)
{
    return r ^ ((r >> 3) & 3) ^ (((r >> 5) & 7) << 2);
}

// Residue index held in slot e by lane t for a layout whose 3 in-lane bits start at b_lo.
__device__ __forceinline__ u32 lay(u32 t, int e, int b_lo)
{
    return ((t >> b_lo) << (b_lo + 3)) | ((u32)e << b_lo) | (t & ((1u << b_lo) - 1));
}

// Row passes load the twiddles of the first stage(s) after their transpose together with the data
// (MHE_ROW_TWPF=0: where the stage uses them)
#ifndef MHE_ROW_TWPF
#define MHE_ROW_TWPF 1
#endif
// row passes at n = 2^16 in FP64 run k_fwd_row3 / k_inv_row3 (8 residues per lane, three phases)
#ifndef MHE_ROW3
#define MHE_ROW3 1
#endif

// --------------------------------------------------------------------- forward, row pass
// FP with the up-front prefetch: 3 waves/SIMD (<= 168 VGPRs)
template <int LOGR, int LOGT, class Job, bool FP, bool PRE_ON = true>
__global__ __launch_bounds__(256, (FP && PRE_ON) ? 3 : 1) void k_fwd_row(Job job, int log_n, long long twd)
{
    using SH = Shape<LOGR, LOGT>;
    using A = NttArith<FP>;
    using T = typename A::T;
    using RL = RowLds<LOGR, LOGT>;
    constexpr int E = SH::E, TPS = SH::TPS, LOGE = SH::LOGE, S = SH::S;
    __shared__ T lds[S * RL::LD];
    const int tid = threadIdx.x, t = tid % TPS, sl = tid / TPS;
    const u32 b = blockIdx.x * S + sl;
    const u32 base = b << LOGR;
    const u32 rb = (1u << (log_n - LOGR)) + b; // 2^k1 + b
    const auto V = job.view(blockIdx.y);
    if (V.skip) return; // uniform per workgroup, before any barrier
    using VW = std::remove_cv_t<decltype(V)>;
    constexpr bool PRE = PreOf<VW>::value && PRE_ON;
    const A ar(V.p, V.tw, twd);
    T v[E];
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = ar.in(V.load(base + t + TPS * e));
    [[maybe_unused]] typename PreOf<VW>::type pr[E];
    if constexpr (PRE)
    {
#pragma unroll
        for (int e = 0; e < E; e++) pr[e] = V.pre(base + t + TPS * e);
    }
    // The twiddles of the first two stages after the transpose, loaded here with the data: the
    // transpose's fence keeps the compiler from issuing them earlier, and each was a serialised L2
    // round trip in the middle of the workgroup's life (3 workgroups per CU do not hide it).  Stage
    // s >= LOGE uses entries (rb << s) + (E t >> (LOGR - s)) + (e >> (LOGR - s)).
    using TWT = typename A::TW;
    constexpr int C0 = E >> (LOGR - LOGE), C1 = E >> (LOGR - LOGE - 1);
    [[maybe_unused]] TWT p0[C0], p1[C1];
    if constexpr (MHE_ROW_TWPF)
    {
#pragma unroll
        for (int j = 0; j < C0; j++) p0[j] = ar.tw[(rb << LOGE) + ((E * t) >> (LOGR - LOGE)) + j];
#pragma unroll
        for (int j = 0; j < C1; j++) p1[j] = ar.tw[(rb << (LOGE + 1)) + ((E * t) >> (LOGR - LOGE - 1)) + j];
    }
#pragma unroll
    for (int s = 0; s < LOGE; s++)
        ar.template fwd<E>(v, 1 << (LOGE - 1 - s), [&](int e) { return (rb << s) + (e >> (LOGE - s)); });
#pragma unroll
    for (int e = 0; e < E; e++) lds[RL::at(sl, t + TPS * e)] = v[e];
    wave_lds_fence(); // a sub-transform is TPS <= 16 consecutive lanes of one wave
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = lds[RL::at(sl, E * t + e)];
#pragma unroll
    for (int s = LOGE; s < LOGR; s++)
    {
        if (MHE_ROW_TWPF && s == LOGE)
            ar.template fwd_tab<E>(v, 1 << (LOGR - 1 - s), p0, [&](int e) { return e >> (LOGR - s); });
        else if (MHE_ROW_TWPF && s == LOGE + 1)
            ar.template fwd_tab<E>(v, 1 << (LOGR - 1 - s), p1, [&](int e) { return e >> (LOGR - s); });
        else
            ar.template fwd<E>(v, 1 << (LOGR - 1 - s), [&](int e) { return (rb << s) + ((E * t + e) >> (LOGR - s)); });
    }
    // transpose back so stores (and epilogue reads) are coalesced
#pragma unroll
    for (int e = 0; e < E; e++) lds[RL::at(sl, E * t + e)] = v[e];
    wave_lds_fence(); // a sub-transform is TPS <= 16 consecutive lanes of one wave
    if constexpr (!PRE && PreOf<VW>::value)
    {
        // Large launches run without the up-front prefetch (4 instead of 3 waves/SIMD), and a plain
        // store(x, o) would load its operands after the previous store: E serialised round trips.
        // Groups of 4 instead, the next group's operands loaded before this group's stores.
        constexpr int G = 4;
        static_assert(E % G == 0, "epilogue groups");
        using PT = typename PreOf<VW>::type;
        PT cur[G], nxt[G];
#pragma unroll
        for (int k = 0; k < G; k++) cur[k] = V.pre(base + t + TPS * k);
#pragma unroll
        for (int e0 = 0; e0 < E; e0 += G)
        {
            if (e0 + G < E)
            {
#pragma unroll
                for (int k = 0; k < G; k++) nxt[k] = V.pre(base + t + TPS * (e0 + G + k));
            }
#pragma unroll
            for (int k = 0; k < G; k++)
            {
                const int e = e0 + k;
                int src = t + TPS * e;
                if constexpr (BrevOf<VW>::value && LOGR == 8) src = (int)brev8_ntt((u32)src);
                V.store(base + t + TPS * e, ar.out(lds[RL::at(sl, src)]), cur[k]);
            }
#pragma unroll
            for (int k = 0; k < G; k++) cur[k] = nxt[k];
        }
        return;
    }
#pragma unroll
    for (int e = 0; e < E; e++)
    {
        int src = t + TPS * e;
        if constexpr (BrevOf<VW>::value && LOGR == 8) src = (int)brev8_ntt((u32)src); // launched at LOGR 8 only
        const u64 o = ar.out(lds[RL::at(sl, src)]);
        if constexpr (PRE)
            V.store(base + t + TPS * e, o, pr[e]);
        else
            V.store(base + t + TPS * e, o);
    }
}

// The twiddles of stage s of a 2^8-point row in layout lay(t, e, b_lo) (b_lo + s <= 8): entry
// (rb << s) + (hi >> (8 - s)) + (e >> (8 - s - b_lo)), hi the lane's bits above the layout's e
// bits -- 2^(b_lo + s - 5) distinct values (at least 1), loaded ahead of the stage's turn.
#ifndef MHE_ROW3_PF
#define MHE_ROW3_PF 1
#endif
template <int S_, int BLO, class AR>
__device__ __forceinline__ void row3_tw(const AR &ar, u32 rb, u32 t, typename AR::TW (&w)[4])
{
    constexpr int C = 1 << ((BLO + S_ - 5) > 0 ? (BLO + S_ - 5) : 0);
    const u32 hi = (t >> BLO) << (BLO + 3);
    const u32 b0 = (rb << S_) + (hi >> (8 - S_));
#pragma unroll
    for (int j = 0; j < C; j++) w[j] = ar.tw[b0 + j];
}

// ------------------------------------------- forward row pass, 2^8-point rows, three phases
// k_fwd_row holds 16 residues per lane (two register phases, one transpose): with an epilogue
// prefetch that is ~150 VGPRs, 3 waves/SIMD, and each workgroup does one load-compute-store round,
// so the latency of the small launches shows.  Here 8 residues per lane in three register phases
// of 3, 3 and 2 stages (k_ks_row_mac's layouts: positions lay(t, e, 5), lay(t, e, 2) and 8t + e,
// wave-local swizzled transposes), 8 rows of 32 lanes per workgroup: about 100 VGPRs and 16 KB of
// LDS.  A third transpose returns to the first layout, in which loads, epilogue operands and
// stores are coalesced across lanes.  n = 2^16, FP64.
template <class Job>
__global__ __launch_bounds__(256) void k_fwd_row3(Job job, int log_n, long long twd)
{
    constexpr int LOGR = 8, R = 256, TPS = 32, S = 8, B_A = 5, B_B = 2;
    using A = NttArith<true>;
    using T = double;
    __shared__ T lds[S * R];
    const int tid = threadIdx.x, t = tid % TPS, sl = tid / TPS;
    const u32 b = blockIdx.x * S + sl;
    const u32 base = b << LOGR;
    const u32 rb = (1u << (log_n - LOGR)) + b;
    const auto V = job.view(blockIdx.y);
    if (V.skip) return; // uniform per workgroup
    using VW = std::remove_cv_t<decltype(V)>;
    constexpr bool PRE = PreOf<VW>::value;
    const A ar(V.p, V.tw, twd);
    T *x = &lds[sl * R];
    T v[8];
#pragma unroll
    for (int e = 0; e < 8; e++) v[e] = ar.in(V.load(base + lay(t, e, B_A)));
    [[maybe_unused]] typename PreOf<VW>::type pr[8];
    if constexpr (PRE)
    {
#pragma unroll
        for (int e = 0; e < 8; e++) pr[e] = V.pre(base + lay(t, e, B_A));
    }
    auto stages = [&](int b_lo, int s0, int s1) {
#pragma unroll
        for (int s = s0; s < s1; s++)
            ar.template fwd<8>(v, 1 << (LOGR - 1 - s - b_lo), [&](int e) { return (rb << s) + (lay(t, e, b_lo) >> (LOGR - s)); });
    };
    auto transpose = [&](int from, int to) {
        wave_lds_fence(); // the previous transpose's reads come first
#pragma unroll
        for (int e = 0; e < 8; e++) x[swz(lay(t, e, from))] = v[e];
        wave_lds_fence(); // a row is 32 lanes of one wave
#pragma unroll
        for (int e = 0; e < 8; e++) v[e] = x[swz(lay(t, e, to))];
    };
    if constexpr (MHE_ROW3_PF)
    {
        // the first stage of each later phase takes twiddles loaded a phase ahead: the transposes'
        // fences would otherwise hold their loads back to the stage itself
        using TWT = typename A::TW;
        TWT w3[4], w6[4];
        row3_tw<3, B_B>(ar, rb, t, w3);
        stages(B_A, 0, 3);
        row3_tw<6, 0>(ar, rb, t, w6);
        transpose(B_A, B_B);
        ar.template fwd_tab<8>(v, 1 << (LOGR - 1 - 3 - B_B), w3, [&](int e) { return e >> (8 - 3 - B_B); });
        stages(B_B, 4, 6);
        transpose(B_B, 0);
        ar.template fwd_tab<8>(v, 1 << (LOGR - 1 - 6), w6, [&](int e) { return e >> (8 - 6); });
        stages(0, 7, 8);
    }
    else
    {
        stages(B_A, 0, 3);
        transpose(B_A, B_B);
        stages(B_B, 3, 6);
        transpose(B_B, 0);
        stages(0, 6, 8);
    }
    // back to the coalesced layout for the epilogue; a brev View (hoist.h) stores at position p the
    // value of position brev8(p)
    wave_lds_fence();
#pragma unroll
    for (int e = 0; e < 8; e++) x[swz(lay(t, e, 0))] = v[e];
    wave_lds_fence();
#pragma unroll
    for (int e = 0; e < 8; e++)
    {
        u32 src = lay(t, e, B_A);
        if constexpr (BrevOf<VW>::value) src = brev8_ntt(src);
        v[e] = x[swz(src)];
    }
#pragma unroll
    for (int e = 0; e < 8; e++)
    {
        if constexpr (PRE)
            V.store(base + lay(t, e, B_A), ar.out(v[e]), pr[e]);
        else
            V.store(base + lay(t, e, B_A), ar.out(v[e]));
    }
}

// --------------------------------------------------------------------- inverse, row pass
template <int LOGR, int LOGT, class Job, bool FP>
__global__ __launch_bounds__(256) void k_inv_row(Job job, int log_n, long long twd)
{
    using SH = Shape<LOGR, LOGT>;
    using A = NttArith<FP>;
    using T = typename A::T;
    using RL = RowLds<LOGR, LOGT>;
    constexpr int E = SH::E, TPS = SH::TPS, LOGE = SH::LOGE, S = SH::S;
    __shared__ T lds[S * RL::LD];
    const int tid = threadIdx.x, t = tid % TPS, sl = tid / TPS;
    const u32 b = blockIdx.x * S + sl;
    const u32 base = b << LOGR;
    const u32 rb = (1u << (log_n - LOGR)) + b;
    const auto V = job.view(blockIdx.y);
    if (V.skip) return; // uniform per workgroup, before any barrier
    const A ar(V.p, V.tw, twd);
    T v[E];
    // the first stage's twiddles with the data (see k_fwd_row): entries (rb << s) + (E t >> 1) + j
    using TWT = typename A::TW;
    [[maybe_unused]] TWT p0[E / 2];
    if constexpr (MHE_ROW_TWPF)
    {
#pragma unroll
        for (int j = 0; j < E / 2; j++) p0[j] = ar.tw[(rb << (LOGR - 1)) + ((E * t) >> 1) + j];
    }
#pragma unroll
    for (int e = 0; e < E; e++) lds[RL::at(sl, t + TPS * e)] = ar.in(V.load(base + t + TPS * e));
    wave_lds_fence(); // a sub-transform is TPS <= 16 consecutive lanes of one wave
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = lds[RL::at(sl, E * t + e)];
#pragma unroll
    for (int s = LOGR - 1; s >= LOGE; s--)
    {
        if (MHE_ROW_TWPF && s == LOGR - 1)
            ar.template inv_tab<E>(v, 1 << (LOGR - 1 - s), p0, [&](int e) { return e >> 1; });
        else
            ar.template inv<E>(v, 1 << (LOGR - 1 - s), [&](int e) { return (rb << s) + ((E * t + e) >> (LOGR - s)); });
    }
#pragma unroll
    for (int e = 0; e < E; e++) lds[RL::at(sl, E * t + e)] = v[e];
    wave_lds_fence(); // a sub-transform is TPS <= 16 consecutive lanes of one wave
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = lds[RL::at(sl, t + TPS * e)];
#pragma unroll
    for (int s = LOGE - 1; s >= 0; s--)
        ar.template inv<E>(v, 1 << (LOGE - 1 - s), [&](int e) { return (rb << s) + (e >> (LOGE - s)); });
#pragma unroll
    for (int e = 0; e < E; e++) V.store(base + t + TPS * e, ar.out(v[e]));
}

// ------------------------------------------- inverse row pass, 2^8-point rows, three phases
// The mirror of k_fwd_row3: coalesced loads, a transpose to the 8t + e layout, stages 7-6, 5-3,
// 2-0 with two more wave-local transposes, coalesced stores.
template <class Job>
__global__ __launch_bounds__(256) void k_inv_row3(Job job, int log_n, long long twd)
{
    constexpr int LOGR = 8, R = 256, TPS = 32, S = 8, B_A = 5, B_B = 2;
    using A = NttArith<true>;
    using T = double;
    __shared__ T lds[S * R];
    const int tid = threadIdx.x, t = tid % TPS, sl = tid / TPS;
    const u32 b = blockIdx.x * S + sl;
    const u32 base = b << LOGR;
    const u32 rb = (1u << (log_n - LOGR)) + b;
    const auto V = job.view(blockIdx.y);
    if (V.skip) return; // uniform per workgroup
    const A ar(V.p, V.tw, twd);
    T *x = &lds[sl * R];
    T v[8];
#pragma unroll
    for (int e = 0; e < 8; e++) v[e] = ar.in(V.load(base + lay(t, e, B_A)));
    auto stages = [&](int b_lo, int s_hi, int s_lo) {
#pragma unroll
        for (int s = s_hi; s >= s_lo; s--)
            ar.template inv<8>(v, 1 << (LOGR - 1 - s - b_lo), [&](int e) { return (rb << s) + (lay(t, e, b_lo) >> (LOGR - s)); });
    };
    auto transpose = [&](int from, int to) {
        wave_lds_fence(); // the previous transpose's reads come first
#pragma unroll
        for (int e = 0; e < 8; e++) x[swz(lay(t, e, from))] = v[e];
        wave_lds_fence(); // a row is 32 lanes of one wave
#pragma unroll
        for (int e = 0; e < 8; e++) v[e] = x[swz(lay(t, e, to))];
    };
    if constexpr (MHE_ROW3_PF)
    {
        using TWT = typename A::TW;
        TWT w7[4], w6[4], w5[4], w2[4];
        row3_tw<7, 0>(ar, rb, t, w7);
        row3_tw<6, 0>(ar, rb, t, w6);
        transpose(B_A, 0); // loaded coalesced
        row3_tw<5, B_B>(ar, rb, t, w5);
        ar.template inv_tab<8>(v, 1 << (LOGR - 1 - 7), w7, [&](int e) { return e >> (8 - 7); });
        ar.template inv_tab<8>(v, 1 << (LOGR - 1 - 6), w6, [&](int e) { return e >> (8 - 6); });
        transpose(0, B_B);
        row3_tw<2, B_A>(ar, rb, t, w2);
        ar.template inv_tab<8>(v, 1 << (LOGR - 1 - 5 - B_B), w5, [&](int e) { return e >> (8 - 5 - B_B); });
        stages(B_B, 4, 3);
        transpose(B_B, B_A);
        ar.template inv_tab<8>(v, 1 << (LOGR - 1 - 2 - B_A), w2, [&](int e) { return e >> (8 - 2 - B_A); });
        stages(B_A, 1, 0);
    }
    else
    {
        transpose(B_A, 0); // loaded coalesced
        stages(0, 7, 6);
        transpose(0, B_B);
        stages(B_B, 5, 3);
        transpose(B_B, B_A);
        stages(B_A, 2, 0);
    }
#pragma unroll
    for (int e = 0; e < 8; e++) V.store(base + lay(t, e, B_A), ar.out(v[e]));
}

// ------------------------------------------------------------------ inverse, column pass
template <int LOGR, int LOGT, class Job, bool FP>
__global__ __launch_bounds__(256) void k_inv_col(Job job, int log_n, long long twd)
{
    using SH = Shape<LOGR, LOGT>;
    using A = NttArith<FP>;
    using T = typename A::T;
    constexpr int E = SH::E, TPS = SH::TPS, LOGE = SH::LOGE, S = SH::S, LD = SH::LD;
    __shared__ T lds[S * LD];
    const int tid = threadIdx.x, sl = tid % S, t = tid / S;
    const int logC = log_n - LOGR;
    const u32 c = blockIdx.x * S + sl;
    const auto V = job.view(blockIdx.y);
    if (V.skip) return; // uniform per workgroup, before any barrier
    const A ar(V.p, V.tw, twd);
    T v[E];
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = ar.in(V.load(c + ((u32)(E * t + e) << logC)));
#pragma unroll
    for (int s = LOGR - 1; s >= LOGE; s--)
        ar.template inv<E>(v, 1 << (LOGR - 1 - s), [&](int e) { return (1 << s) + ((E * t + e) >> (LOGR - s)); });
#pragma unroll
    for (int e = 0; e < E; e++) lds[sl * LD + E * t + e] = v[e];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = lds[sl * LD + t + TPS * e];
#pragma unroll
    for (int s = LOGE - 1; s >= 1; s--)
        ar.template inv<E>(v, 1 << (LOGE - 1 - s), [&](int e) { return (1 << s) + (e >> (LOGE - s)); });
    {
        constexpr int gap = E / 2;
#pragma unroll
        for (int e = 0; e < gap; e++) ar.inv_last(v[e], v[e + gap], V.p);
    }
#pragma unroll
    for (int e = 0; e < E; e++) V.store(c + ((u32)(t + TPS * e) << logC), ar.out(v[e]));
}

// ------------------------------------ inverse column pass fused with a lift + forward column pass
// ModDown (evaluator.cpp:2466-2524) and rescale (rns.cpp:737-808) both take one limb (the special
// prime's accumulator / the last limb) through an INTT, lift it into every other prime and
// forward-transform it.  After the inverse column stages a lane holds exactly the positions the
// forward column pass loads, so one workgroup per (column block, poly, group of output primes)
// finishes the INTT of its columns once (canonical), then for each output prime lifts (the job's
// View::lift) and runs the forward column stages: the separate inverse-column launch and its HBM
// round trip disappear, and the outputs are the same words.
// The first register phase of a forward column pass (stages 0 .. LOGE-1) uses twiddle entries
// 1 .. E-1, the same for every lane: read them as scalar loads of the prime's FP table (ftab), issued
// together, instead of per-stage LDS reads each waited for a few instructions later.
#ifndef MHE_COL_STW
#define MHE_COL_STW 0 // k_icol_lift / k_col_lift2 (FP): scalar first-phase twiddles (k_modup_col: MHE_MODUP_STW);
                      // measured equal (profiles/r06s), so off
#endif
template <int E, int LOGE, class AR>
__device__ __forceinline__ void fwd_first_phase_s(const AR &ar, typename AR::T (&v)[E], const void *ftab)
{
    const const_u64_p g = (const_u64_p)ftab;
    typename AR::TW w1[E];
#pragma unroll
    for (int k = 1; k < E; k++)
    {
        w1[k].x = __longlong_as_double((long long)g[2 * k]);
        w1[k].y = __longlong_as_double((long long)g[2 * k + 1]);
    }
#pragma unroll
    for (int s = 0; s < LOGE; s++)
        ar.template fwd_tab<E>(v, 1 << (LOGE - 1 - s), w1, [&](int e) { return (1 << s) + (e >> (LOGE - s)); });
}

// q < 2^47 (the lazy forward butterflies) as a scalar compare of the high word: the compiler folds any
// 64-bit form into v_cmp_lt_u64 against a 2^47 it keeps in a VGPR pair, which the column passes spilled
// and reloaded in every output prime's skip test (with a vmcnt(0) that also drained the stores)
__device__ __forceinline__ bool lazy_prime(u64 q)
{
    u32 hi = (u32)(q >> 32);
    asm volatile("" : "+s"(hi));
    return hi < (1u << 15);
}

struct ColSrc
{
    const u64 *src[MHE_MAXB]; // poly s of batch entry e at src[e] + s * stride, after the inverse row pass
    size_t stride;
    int per;                  // polys per batch entry
    const PrimeDev *primes;
    const Tw *itw;            // inverse twiddle rows
    int pi;                   // prime index of the source limb
    __device__ const u64 *poly(int y) const
    {
        const int e = y / per;
        return src[e] + (size_t)(y - e * per) * stride;
    }
};

#ifndef MHE_ICOL_G
#define MHE_ICOL_G 5 // at most this many output primes per lift-pass workgroup (icol_lift_a); 5 fills the LDS
                     // of 3 workgroups per CU: 8 rescales at 25 limbs -5 % against 3 (profiles/r06w)
#endif
template <int LOGR, int LOGT, class Job, bool FP>
__global__ __launch_bounds__(256, 3) void k_icol_lift(ColSrc cs, Job job, int cnt, int log_n, long long dinv,
                                                      long long dfwd)
{
    using SH = Shape<LOGR, LOGT>;
    using A = NttArith<FP>;
    using T = typename A::T;
    constexpr int E = SH::E, TPS = SH::TPS, LOGE = SH::LOGE, S = SH::S, LD = SH::LD, R = SH::R;
    __shared__ T lds[S * LD];
    // FP: the forward column twiddles of the group's primes (entries 1 .. R-1 of each table, the same
    // for every column), staged once.  Read from global memory in the prime loop, each twiddle load's
    // wait also waited for the previous prime's stores (one counter for loads and stores).
    __shared__ TwF twc[FP ? MHE_ICOL_G * R : 1];
    const int tid = threadIdx.x, sl = tid % S, t = tid / S;
    const int logC = log_n - LOGR;
    const u32 c = blockIdx.x * S + sl;
    const int s = blockIdx.y;
    const int IG = gridDim.z, g = blockIdx.z;
    const int i_lo = (cnt * g) / IG, i_hi = (cnt * (g + 1)) / IG; // i_hi - i_lo <= MHE_ICOL_G (host)
    if constexpr (FP)
    {
        for (int i = i_lo; i < i_hi; i++)
        {
            const auto V = job.view(s * cnt + i);
            const TwF *tf = reinterpret_cast<const TwF *>(reinterpret_cast<const char *>(V.tw) + dfwd);
            for (int k = tid; k < R; k += 256) twc[(i - i_lo) * R + k] = tf[k];
        }
    }
    u64 x[E];
    {
        // the inverse column pass of k_inv_col, canonical output
        const PrimeDev P = cs.primes[cs.pi];
        const A ai(P, cs.itw + ((size_t)cs.pi << log_n), dinv);
        const u64 *src = cs.poly(s);
        T v[E];
#pragma unroll
        for (int e = 0; e < E; e++) v[e] = ai.in(src[c + ((u32)(E * t + e) << logC)]);
#pragma unroll
        for (int st = LOGR - 1; st >= LOGE; st--)
            ai.template inv<E>(v, 1 << (LOGR - 1 - st), [&](int e) { return (1 << st) + ((E * t + e) >> (LOGR - st)); });
#pragma unroll
        for (int e = 0; e < E; e++) lds[sl * LD + E * t + e] = v[e];
        __syncthreads();
#pragma unroll
        for (int e = 0; e < E; e++) v[e] = lds[sl * LD + t + TPS * e];
#pragma unroll
        for (int st = LOGE - 1; st >= 1; st--)
            ai.template inv<E>(v, 1 << (LOGE - 1 - st), [&](int e) { return (1 << st) + (e >> (LOGE - st)); });
        {
            constexpr int gap = E / 2;
#pragma unroll
            for (int e = 0; e < gap; e++) ai.inv_last(v[e], v[e + gap], P);
        }
#pragma unroll
        for (int e = 0; e < E; e++) x[e] = ai.canon(v[e]);
    }
    // x[e] is the coefficient at c + ((t + TPS e) << logC): the forward column pass's load order
    if constexpr (FP)
    {
        // The lift as the centred integer c (|c| < 2^50, the same for every output prime) reduced
        // mod q_i in FP64: congruent to the integer lift's [0, 2q_i) value, so the same residues,
        // without its 64-bit Barrett reduction and u64 -> f64 conversion per prime.
        double cd[E];
        {
            const auto V0 = job.view(s * cnt + i_lo);
#pragma unroll
            for (int e = 0; e < E; e++) cd[e] = V0.lift_c(x[e]);
        }
        // two sweeps over the group's primes, the q < 2^47 ones with the lazy forward butterflies
        // first (the lift leaves |v| <= q/2 + 1, 8 stages grow it to <= 12.5q), so each loop body
        // has one arithmetic variant (one body with both needed ~100 more VGPRs)
        auto sweep = [&](auto lz) {
            constexpr bool LZ = decltype(lz)::value;
            for (int i = i_lo; i < i_hi; i++)
            {
                const auto V = job.view(s * cnt + i);
                if (lazy_prime(V.p.q) != LZ) continue; // uniform per workgroup
                const NttArithF<LZ> ar(V.p, V.tw, dfwd);
                const TwF *tl = &twc[(i - i_lo) * R];
                T v[E];
#pragma unroll
                for (int e = 0; e < E; e++) v[e] = fp_reduce(cd[e], ar.q, ar.qinv);
                if constexpr (MHE_COL_STW)
                    fwd_first_phase_s<E, LOGE>(ar, v, reinterpret_cast<const char *>(V.tw) + dfwd);
                else
                {
#pragma unroll
                    for (int st = 0; st < LOGE; st++)
                        ar.template fwd_tab<E>(v, 1 << (LOGE - 1 - st), tl, [&](int e) { return (1 << st) + (e >> (LOGE - st)); });
                }
                lds_barrier(); // lds still holds the previous prime's (or the inverse pass's) transpose
#pragma unroll
                for (int e = 0; e < E; e++) lds[sl * LD + t + TPS * e] = v[e];
                lds_barrier(); // LDS only: the previous prime's stores stay in flight
#pragma unroll
                for (int e = 0; e < E; e++) v[e] = lds[sl * LD + E * t + e];
#pragma unroll
                for (int st = LOGE; st < LOGR; st++)
                    ar.template fwd_tab<E>(v, 1 << (LOGR - 1 - st), tl,
                                           [&](int e) { return (1 << st) + ((E * t + e) >> (LOGR - st)); });
#pragma unroll
                for (int e = 0; e < E; e++) V.store(c + ((u32)(E * t + e) << logC), ar.out(v[e]));
            }
        };
        sweep(std::true_type{});
        sweep(std::false_type{});
    }
    else
    {
        for (int i = i_lo; i < i_hi; i++)
        {
            const auto V = job.view(s * cnt + i);
            const A ar(V.p, V.tw, dfwd);
            T v[E];
#pragma unroll
            for (int e = 0; e < E; e++) v[e] = ar.in(V.lift(x[e]));
#pragma unroll
            for (int st = 0; st < LOGE; st++)
                ar.template fwd<E>(v, 1 << (LOGE - 1 - st), [&](int e) { return (1 << st) + (e >> (LOGE - st)); });
            lds_barrier(); // lds still holds the previous prime's (or the inverse pass's) transpose
#pragma unroll
            for (int e = 0; e < E; e++) lds[sl * LD + t + TPS * e] = v[e];
            lds_barrier(); // LDS only: the previous prime's stores stay in flight
#pragma unroll
            for (int e = 0; e < E; e++) v[e] = lds[sl * LD + E * t + e];
#pragma unroll
            for (int st = LOGE; st < LOGR; st++)
                ar.template fwd<E>(v, 1 << (LOGR - 1 - st),
                                   [&](int e) { return (1 << st) + ((E * t + e) >> (LOGR - st)); });
#pragma unroll
            for (int e = 0; e < E; e++) V.store(c + ((u32)(E * t + e) << logC), ar.out(v[e]));
        }
    }
}

// ------------------------------------------------------------- FP64 lift column pass, two sources
// The fused HMult tail's column pass (JobMDRCol): every output prime's input is a function of two
// prime-independent source words (the special accumulator limb and the rescale's last limb).  One
// workgroup per (column block, source poly, group of <= MHE_ICOL_G output primes) reads them once,
// as centred doubles (View::src_c), and per prime forms the lift (View::lift_f), reduces it and runs
// the forward column stages with twiddles staged in LDS, the q < 2^47 primes with lazy butterflies
// -- k_fwd_col instead re-read both sources and redid the integer lift per prime.  FP contexts only.
template <int LOGR, int LOGT, class Job>
__global__ __launch_bounds__(256, 3) void k_col_lift2(Job job, int cnt, int log_n, long long dfwd)
{
    using SH = Shape<LOGR, LOGT>;
    using T = double;
    constexpr int E = SH::E, TPS = SH::TPS, LOGE = SH::LOGE, S = SH::S, LD = SH::LD, R = SH::R;
    __shared__ T lds[S * LD];
    __shared__ TwF twc[MHE_ICOL_G * R];
    const int tid = threadIdx.x, sl = tid % S, t = tid / S;
    const int logC = log_n - LOGR;
    const u32 c = blockIdx.x * S + sl;
    const int s = blockIdx.y;
    const int IG = gridDim.z, g = blockIdx.z;
    const int i_lo = (cnt * g) / IG, i_hi = (cnt * (g + 1)) / IG; // i_hi - i_lo <= MHE_ICOL_G (host)
    for (int i = i_lo; i < i_hi; i++)
    {
        const auto V = job.view(s * cnt + i);
        const TwF *tf = reinterpret_cast<const TwF *>(reinterpret_cast<const char *>(V.tw) + dfwd);
        for (int k = tid; k < R; k += 256) twc[(i - i_lo) * R + k] = tf[k];
    }
    double ca[E], cb[E];
    {
        const auto V0 = job.view(s * cnt + i_lo);
#pragma unroll
        for (int e = 0; e < E; e++) V0.src_c(c + ((u32)(t + TPS * e) << logC), ca[e], cb[e]);
    }
    lds_barrier(); // twiddles visible
    auto sweep = [&](auto lz) {
        constexpr bool LZ = decltype(lz)::value;
        for (int i = i_lo; i < i_hi; i++)
        {
            const auto V = job.view(s * cnt + i);
            if (lazy_prime(V.p.q) != LZ) continue; // uniform per workgroup
            const NttArithF<LZ> ar(V.p, V.tw, dfwd);
            const TwF *tl = &twc[(i - i_lo) * R];
            T v[E];
#pragma unroll
            for (int e = 0; e < E; e++) v[e] = fp_reduce(V.lift_f(ca[e], cb[e]), ar.q, ar.qinv);
            if constexpr (MHE_COL_STW)
                fwd_first_phase_s<E, LOGE>(ar, v, reinterpret_cast<const char *>(V.tw) + dfwd);
            else
            {
#pragma unroll
                for (int st = 0; st < LOGE; st++)
                    ar.template fwd_tab<E>(v, 1 << (LOGE - 1 - st), tl, [&](int e) { return (1 << st) + (e >> (LOGE - st)); });
            }
            lds_barrier(); // lds still holds the previous prime's transpose
#pragma unroll
            for (int e = 0; e < E; e++) lds[sl * LD + t + TPS * e] = v[e];
            lds_barrier(); // LDS only: the previous prime's stores stay in flight
#pragma unroll
            for (int e = 0; e < E; e++) v[e] = lds[sl * LD + E * t + e];
#pragma unroll
            for (int st = LOGE; st < LOGR; st++)
                ar.template fwd_tab<E>(v, 1 << (LOGR - 1 - st), tl,
                                       [&](int e) { return (1 << st) + ((E * t + e) >> (LOGR - st)); });
#pragma unroll
            for (int e = 0; e < E; e++) V.store(c + ((u32)(E * t + e) << logC), ar.out(v[e]));
        }
    };
    sweep(std::true_type{});
    sweep(std::false_type{});
}

// ------------------------------------------------- key-switch ModUp, digit-major column pass
// Column pass of the ModUp (evaluator.cpp:2386-2408) with one workgroup per (column block,
// digit J, group of output primes): the digit's columns are read once into registers and
// lifted + transformed for every output prime I of the group (I == J skipped: the MAC reads
// the input NTT form).  Reading each digit once instead of once per output prime removes
// L(L+1) - L limb reads (~1 GB at L=44) from the key switch.
// Per-entry buffers of a (batched) key switch: entry e is blockIdx.y of the ModUp column pass and
// blockIdx.z of the fused row pass + MAC.
struct KsPtrs
{
    const u64 *coeff[MHE_MAXB];  // INTT(target), canonical [L][n]
    u64 *inter[MHE_MAXB];        // ModUp column-pass output [Icnt][L][n]
    const u64 *target[MHE_MAXB]; // target, NTT form [L][n]
    const u64 *key[MHE_MAXB];    // [digits][2][key_limbs][n]
    u64 *acc[MHE_MAXB];          // key inner products [2][L+1][n]
    int key_limbs[MHE_MAXB];
    const int *run_if[MHE_MAXB]; // non-null: the entry's workgroups return unless *run_if != 0 (hoist.h fallback)
};

#ifndef MHE_MODUP_OCC
#define MHE_MODUP_OCC 3 // waves per SIMD the ModUp column pass is compiled for (168 VGPRs)
#endif
#ifndef MHE_MODUP_WAVE
#define MHE_MODUP_WAVE 0 // n = 2^16: a column's lanes in one wave, wave-local transposes (k_modup_col);
                         // with non-temporal stores 8x slower (16-byte store segments, profiles/r06f)
#endif
#ifndef MHE_MODUP_PING
#define MHE_MODUP_PING 1 // n = 2^16: alternate two LDS images per output prime, one barrier per prime (k_modup_col)
#endif
#ifndef MHE_MODUP_STW
#define MHE_MODUP_STW 1 // k_modup_col (FP): first-phase twiddles as scalar loads instead of LDS reads
#endif
#ifndef MHE_MODUP_TPF
#define MHE_MODUP_TPF 0 // k_modup_col: stage-4 (2: and stage-5) twiddles read before the transpose; at 168 VGPRs
                        // both spill (6 / 14 bytes per lane), so off
#endif
#ifndef MHE_MODUP_TWG
#define MHE_MODUP_TWG 5 // output primes per group whose twiddles the ModUp column pass stages in LDS
#endif
// MIX (with FP): output primes >= 2^51 (the GPT-2 chain's special prime) take the integer sweep.
// The integer and MIX variants get 2 waves/SIMD: at 3 (168 VGPRs) they spilled 116-124 bytes per
// lane, and each scratch reload waits for every store in flight (one vmcnt for loads and stores)
#ifndef MHE_MODUP_OCC_INT
#define MHE_MODUP_OCC_INT 2
#endif
template <int LOGR, int LOGT, bool FP, bool MIX = false>
__global__ __launch_bounds__(256, (FP && !MIX) ? MHE_MODUP_OCC : MHE_MODUP_OCC_INT) void k_modup_col(KsPtrs P, const PrimeDev *__restrict__ primes,
                                                   const Tw *__restrict__ tw_all, int L, int K, int log_n,
                                                   long long twd, int I0, int Icnt, int pack, int X, int IG, int xcd)
{
    if (P.run_if[blockIdx.y] && !*P.run_if[blockIdx.y]) return; // uniform, before any barrier
    const u64 *__restrict__ coeff = P.coeff[blockIdx.y];
    u64 *__restrict__ modup = P.inter[blockIdx.y];
    using SH = Shape<LOGR, LOGT>;
    using A = NttArith<FP>;
    using T = typename A::T;
    constexpr int E = SH::E, TPS = SH::TPS, LOGE = SH::LOGE, S = SH::S, LD = SH::LD;
    constexpr int R = SH::R;
    // MHE_MODUP_WAVE (n = 2^16, 16 lanes per column): a column's 16 lanes are consecutive lanes of
    // one wave (4 columns per wave) instead of one lane in each of 16 waves' worth of rows, so the
    // transpose between the two register phases stays inside the wave: no workgroup barrier per
    // output prime (round 5: two, a third of the kernel's wave time waiting).  The column's LDS image
    // is unpadded and XOR-skewed (wslot): conflict-free for the transpose's ds_write_b64 (one column's
    // 16 lanes) and ds_read_b64 (two columns' 32 lanes) under MI355X_MICROARCH.md §LDS's bank rules.
    constexpr bool WV = MHE_MODUP_WAVE && LOGR == 8 && TPS == 16;
    // MHE_MODUP_PING (n = 2^16): the transpose's LDS image alternates between two placements from
    // one output prime to the next.  Prime k writes row t + 16e of its column at the slot the same
    // lane read row 16t + e from in prime k - 1, and reads row 16t + e from the slot it wrote row
    // t + 16e to in prime k - 1: every slot a lane overwrites was last read by that lane itself, so
    // the barrier after each prime's reads (round 5: two barriers per prime) is not needed.  The
    // placements are the padded image (column sl at sl * LD) with the two roles of t and e swapped, so
    // both address patterns stay a lane base plus immediates and the LDS size (occupancy: 3 workgroups
    // per CU, one more element per column already drops it to 2, profiles/r06k) is unchanged.  Banks
    // (MI355X_MICROARCH.md §LDS): the writes are conflict-free either way (16 lanes, sl = 0..15); the
    // reads of rows 16t + e from the swapped placement (element sl * 257 + t + 16e) are 2-way
    // conflicted, on every second output prime.
    constexpr bool PG = !WV && MHE_MODUP_PING && LOGR == 8 && TPS == 16;
#ifndef MHE_MODUP_LDS_EXTRA
#define MHE_MODUP_LDS_EXTRA 0 // A/B only: extra elements in the LDS image (occupancy probe)
#endif
#ifndef MHE_MODUP_PING_BAR
#define MHE_MODUP_PING_BAR 0 // A/B only: keep the end-of-prime barrier with the ping-pong image
#endif
    __shared__ T lds[(WV ? S * R : S * LD) + MHE_MODUP_LDS_EXTRA];
    auto wslot = [](int col, int r) { return col * R + ((r ^ ((r >> 4) & 15)) ^ ((col & 1) << 4)); };
    // The column-pass twiddles of the group's output primes (entries 1 .. R-1 of each prime's table,
    // the same for every column), staged once per workgroup.  Read from global memory stage by stage
    // instead, each twiddle load's s_waitcnt also waited for the previous prime's stores (one
    // counter for loads and stores), so compute and stores of consecutive primes never overlapped.
    __shared__ Tw twc[MHE_MODUP_TWG > 0 ? MHE_MODUP_TWG * R : 1];
    const int tid = threadIdx.x, sl = WV ? tid / TPS : tid % S, t = WV ? tid % TPS : tid / S;
    const int logC = log_n - LOGR;
    // 1-D grid of X column blocks x L digits x IG output-prime groups.  xcd: the IG groups of one
    // (column block, digit) get ids i, i + 8, ..., i + 8 (IG - 1) -- workgroups are dealt to the 8
    // XCDs round robin, so they run on one XCD close in time and share its L2 copy of the digit
    u32 bj;
    int g;
    {
        const u32 id = blockIdx.x;
        if (xcd)
        {
            const u32 per = 8u * (u32)IG, r = id % per;
            g = (int)(r / 8);
            bj = (id / per) * 8 + r % 8;
        }
        else
        {
            const u32 XL = (u32)X * (u32)L;
            bj = id % XL;
            g = (int)(id / XL);
        }
    }
    const u32 c = (bj % (u32)X) * S + sl;
    const int J = (int)(bj / (u32)X);
    const int i_lo = I0 + (Icnt * g) / IG, i_hi = I0 + (Icnt * (g + 1)) / IG;
    const u64 *src = coeff + ((size_t)J << log_n);
    u64 x[E];
#pragma unroll
    for (int e = 0; e < E; e++) x[e] = src[c + ((u32)(t + TPS * e) << logC)];
    const u64 qJ = primes[J].q;
    // twiddles of the group's primes into LDS (16 B each: the FP table (w, w/q) or the integer one
    // (w, Shoup), whichever the prime's sweep uses); groups wider than MHE_MODUP_TWG read global
    const bool twl_on = MHE_MODUP_TWG > 0 && i_hi - i_lo <= MHE_MODUP_TWG; // uniform per workgroup
    if (twl_on)
    {
        const int ng = i_hi - i_lo;
        for (int k = tid; k < ng * R; k += 256)
        {
            const int g = k / R, idx = k % R;
            const int I = i_lo + g;
            const int pi = (I == L) ? K - 1 : I;
            const bool fpt = FP && primes[pi].q < (1ull << 51);
            const char *base = reinterpret_cast<const char *>(tw_all + ((size_t)pi << log_n)) + (fpt ? twd : 0);
            twc[k] = reinterpret_cast<const Tw *>(base)[idx];
        }
        lds_barrier(); // twiddles visible
    }
    // FP: the digit residues (< 2^51, exact in a double) are converted once, not once per output
    // prime (u64 -> f64 is several VALU instructions)
    double xd[E];
    if constexpr (FP)
    {
#pragma unroll
        for (int e = 0; e < E; e++) xd[e] = fp_from_u52(x[e]); // canonical INTT output
    }
    // PG: the two lane bases, pa + 16e and pb + e
    const u32 pa = (u32)(sl * LD + t), pb = (u32)(sl * LD + 16 * t);
    int ph = 0; // PG: placement of the next output prime (uniform), carried across the sweeps
    // two sweeps over the group's output primes when FP: first the q < 2^47 ones with the lazy
    // forward butterflies, then the rest, so each loop body has one arithmetic variant
    auto sweep = [&](auto mode) {
        constexpr int M = decltype(mode)::value; // 0 integer, 1 FP lazy, 2 FP full
        using AA = std::conditional_t<M == 0, NttArith<false>, std::conditional_t<M == 1, NttArithF<true>, NttArithF<false>>>;
        using VT = typename AA::T;
        VT *const lds_v = reinterpret_cast<VT *>(lds); // same 8-byte elements either way
        for (int I = i_lo; I < i_hi; I++)
        {
            if (I == J) continue; // uniform per workgroup
            const int pi = (I == L) ? K - 1 : I;
            const PrimeDev p = primes[pi];
            if (M == 1 && !(p.q < (1ull << 47))) continue;
            if (M == 2 && (p.q < (1ull << 47) || !(p.q < (1ull << 51)))) continue;
            if (M == 0 && FP && p.q < (1ull << 51)) continue; // mixed: the FP sweeps took it
            const AA ar(p, tw_all + ((size_t)pi << log_n), twd);
            using TWA = typename AA::TW;
            const TWA *tl = reinterpret_cast<const TWA *>(&twc[(I - i_lo) * R]);
            VT v[E];
            if constexpr (M != 0)
            {
#pragma unroll
                for (int e = 0; e < E; e++) v[e] = fp_reduce(xd[e], ar.q, ar.qinv);
            }
            else
            {
                const bool red = qJ > p.q; // key_modulus[J] <= key_modulus[I] -> plain copy
#pragma unroll
                for (int e = 0; e < E; e++)
                {
                    const u64 xe = FP ? (u64)xd[e] : x[e]; // FP: the digit held as an exact double
                    v[e] = red ? barrett64(xe, p) : xe;
                }
            }
            if constexpr (MHE_MODUP_STW && M != 0)
            {
                // the first phase's twiddles as scalar loads (fwd_first_phase_s), issued with the prime's
                // setup
                fwd_first_phase_s<E, LOGE>(ar, v, reinterpret_cast<const char *>(tw_all + ((size_t)pi << log_n)) + twd);
            }
            else if (twl_on)
            {
#pragma unroll
                for (int s = 0; s < LOGE; s++)
                    ar.template fwd_tab<E>(v, 1 << (LOGE - 1 - s), tl, [&](int e) { return (1 << s) + (e >> (LOGE - s)); });
            }
            else
            {
#pragma unroll
                for (int s = 0; s < LOGE; s++)
                    ar.template fwd<E>(v, 1 << (LOGE - 1 - s), [&](int e) { return (1 << s) + (e >> (LOGE - s)); });
            }
            // MHE_MODUP_TPF: the twiddles of the first two stages after the transpose (1 and 2 per lane)
            // read before it, so their LDS round trip overlaps the transpose's
            [[maybe_unused]] TWA q4[1], q5[2];
            if constexpr (MHE_MODUP_TPF && LOGE == 4 && LOGR == 8)
            {
                if (twl_on)
                {
                    q4[0] = tl[16 + t];
                    if constexpr (MHE_MODUP_TPF > 1)
                    {
                        q5[0] = tl[32 + 2 * t];
                        q5[1] = tl[32 + 2 * t + 1];
                    }
                }
            }
            if constexpr (WV)
            {
                // wslot is XOR-linear in e: row t + 16e sits at wslot(sl, t) ^ 17e, row 16t + e at
                // wslot(sl, 16t) ^ e; the two bases go through an empty asm each output prime so the
                // 32 slots are recomputed (one v_xor each) rather than hoisted into 32 VGPRs
                u32 wb = (u32)wslot(sl, t), rb = (u32)wslot(sl, 16 * t);
                asm volatile("" : "+v"(wb), "+v"(rb));
                wave_lds_fence(); // the previous output prime's reads of this column come first
#pragma unroll
                for (int e = 0; e < E; e++) lds_v[wb ^ (17u * e)] = v[e];
                wave_lds_fence();
#pragma unroll
                for (int e = 0; e < E; e++) v[e] = lds_v[rb ^ (u32)e];
            }
            else if constexpr (PG)
            {
                // the asm markers keep the two read sequences apart: merged, they took their offsets
                // from SGPRs, one v_add per read
                if (!ph)
                {
#pragma unroll
                    for (int e = 0; e < E; e++) lds_v[pa + 16 * e] = v[e];
                    lds_barrier(); // LDS only: the previous output prime's stores stay in flight
#pragma unroll
                    for (int e = 0; e < E; e++) v[e] = lds_v[pb + e];
                    asm volatile("; modup placement 0");
                }
                else
                {
#pragma unroll
                    for (int e = 0; e < E; e++) lds_v[pb + e] = v[e];
                    lds_barrier();
#pragma unroll
                    for (int e = 0; e < E; e++) v[e] = lds_v[pa + 16 * e];
                    asm volatile("; modup placement 1");
                }
                ph ^= 1;
            }
            else
            {
#pragma unroll
                for (int e = 0; e < E; e++) lds_v[sl * LD + t + TPS * e] = v[e];
                lds_barrier(); // LDS only: the previous output prime's stores stay in flight
#pragma unroll
                for (int e = 0; e < E; e++) v[e] = lds_v[sl * LD + E * t + e];
            }
            if (twl_on)
            {
                constexpr int S0 = (MHE_MODUP_TPF && LOGE == 4 && LOGR == 8) ? LOGE + (MHE_MODUP_TPF > 1 ? 2 : 1) : LOGE;
                // stage 4: entry 16 + t; stage 5: 32 + 2t + (e >> 3)
                if constexpr (S0 > LOGE) ar.template fwd_tab<E>(v, 1 << (LOGR - 1 - LOGE), q4, [&](int) { return 0; });
                if constexpr (S0 > LOGE + 1) ar.template fwd_tab<E>(v, 1 << (LOGR - 2 - LOGE), q5, [&](int e) { return e >> 3; });
#pragma unroll
                for (int s = S0; s < LOGR; s++)
                    ar.template fwd_tab<E>(v, 1 << (LOGR - 1 - s), tl,
                                           [&](int e) { return (1 << s) + ((E * t + e) >> (LOGR - s)); });
            }
            else
            {
#pragma unroll
                for (int s = LOGE; s < LOGR; s++)
                    ar.template fwd<E>(v, 1 << (LOGR - 1 - s),
                                       [&](int e) { return (1 << s) + ((E * t + e) >> (LOGR - s)); });
            }
            u64 *dst = modup + (((size_t)(I - I0) * L + J) << log_n);
            if (inter_packed(pack, p.q)) // uniform per workgroup
            {
                // n = 2^16 here, so logC = 16 - LOGR is a constant and the tile offsets fold into
                // one base per lane plus immediates
                constexpr int LC = 16 - LOGR;
                u32 *lo = reinterpret_cast<u32 *>(dst) + tile16(c + ((u32)(E * t) << LC));
                // word index of the lane's first row pair (E t is a multiple of 16: tile16h is even)
                u32 *hi = reinterpret_cast<u32 *>(dst) + 65536 + (tile16h(c + ((u32)(E * t) << LC)) >> 1);
#pragma unroll
                for (int e = 0; e < E; e += 2)
                {
                    // FP: the centred residue as 48-bit two's complement (fp_to_s48; k_ks_row_mac
                    // reads it back with fp_from_s48); integer: the canonical residue
                    u64 o0, o1;
                    if constexpr (M != 0)
                    {
                        o0 = fp_to_s48(v[e], ar.q, ar.qinv);
                        o1 = fp_to_s48(v[e + 1], ar.q, ar.qinv);
                    }
                    else
                    {
                        o0 = ar.out(v[e]);
                        o1 = ar.out(v[e + 1]);
                    }
                    // tile16(c + ((E t + e) << LC)) - tile16(c + ((E t) << LC)), E t a multiple of 16
                    const u32 k0 = ((u32)(e >> 4) << 12) | ((u32)(e & 15) << 4);
                    const u32 k1 = ((u32)((e + 1) >> 4) << 12) | ((u32)((e + 1) & 15) << 4);
                    st_nt<0>(&lo[k0], (u32)o0);
                    st_nt<0>(&lo[k1], (u32)o1);
                    // the same difference for tile16h in words: row pair (e & 15) / 2 of tile row e / 16
                    const u32 kw = ((u32)(e >> 4) << 11) | ((u32)((e & 15) >> 1) << 4);
                    st_nt<0>(&hi[kw], ((u32)(o0 >> 32) & 0xFFFFu) | ((u32)(o1 >> 32) << 16));
                }
            }
            else
            {
                // one base pointer per lane and a uniform stride: no per-element 64-bit offsets to
                // keep (they were spilled to scratch and reloaded with a vmcnt(0) wait per store)
                const size_t stride = (size_t)1 << logC;
                u64 *d0 = dst + c + ((size_t)(E * t) << logC);
#pragma unroll
                for (int e = 0; e < E; e++) st_nt<0>(d0 + (size_t)e * stride, ar.out(v[e]));
            }
            if constexpr (!WV && (!PG || MHE_MODUP_PING_BAR)) lds_barrier(); // lds is rewritten by the next output prime (its stores need not land)
        }
    };
    if constexpr (FP)
    {
        sweep(std::integral_constant<int, 1>{});
        sweep(std::integral_constant<int, 2>{});
        if constexpr (MIX) sweep(std::integral_constant<int, 0>{});
    }
    else
        sweep(std::integral_constant<int, 0>{});
}

template <int LOGR, bool FP, bool MIX = false>
static inline void modup_col_a(const KsPtrs &P, int B, const PrimeDev *primes, const Tw *tw, int L, int K,
                               int log_n, long long twd, int I0, int Icnt, int IG, int pack, hipStream_t st)
{
#ifndef MHE_MODUP_LOGT8
#define MHE_MODUP_LOGT8 4
#endif
    constexpr int LOGT = LOGR <= 7 ? 3 : MHE_MODUP_LOGT8;
    using SH = Shape<LOGR, LOGT>;
    const int subs = 1 << (log_n - LOGR);
    const int X = subs / SH::S;
    const int xcd = (X * L) % 8 == 0 ? 1 : 0; // XCD-grouped output-prime groups (profiles/r02k_modup_xcd_ab.txt)
    hipLaunchKernelGGL((k_modup_col<LOGR, LOGT, FP, MIX>), dim3((unsigned)(X * L * IG), (unsigned)B), dim3(256), 0, st,
                       P, primes, tw, L, K, log_n, twd, I0, Icnt, pack, X, IG, xcd);
}

// ModUp column pass for output primes I0 .. I0+Icnt-1 (each entry's inter holds exactly those), in
// IG groups of output primes per digit, over B batch entries.  pack (n = 2^16 only): limbs of
// primes below 2^48 are stored in the packed 48-bit form (tile16), which k_ks_row_mac must then be
// told as well.
static inline void modup_col(const KsPtrs &P, int B, const PrimeDev *primes, const Tw *tw, int L, int K,
                             int log_n, const NttMode &m, int I0, int Icnt, int IG, int pack, hipStream_t st)
{
    switch ((log_n + 1) / 2)
    {
    case 6:
        if (m.fp == 2) modup_col_a<6, true, true>(P, B, primes, tw, L, K, log_n, m.dfwd, I0, Icnt, IG, 0, st);
        else if (m.fp) modup_col_a<6, true>(P, B, primes, tw, L, K, log_n, m.dfwd, I0, Icnt, IG, 0, st);
        else modup_col_a<6, false>(P, B, primes, tw, L, K, log_n, 0, I0, Icnt, IG, 0, st);
        break;
    case 7:
        if (m.fp == 2) modup_col_a<7, true, true>(P, B, primes, tw, L, K, log_n, m.dfwd, I0, Icnt, IG, 0, st);
        else if (m.fp) modup_col_a<7, true>(P, B, primes, tw, L, K, log_n, m.dfwd, I0, Icnt, IG, 0, st);
        else modup_col_a<7, false>(P, B, primes, tw, L, K, log_n, 0, I0, Icnt, IG, 0, st);
        break;
    case 8:
        pack = (pack && log_n == 16) ? 1 : 0;
        if (m.fp == 2) modup_col_a<8, true, true>(P, B, primes, tw, L, K, log_n, m.dfwd, I0, Icnt, IG, pack, st);
        else if (m.fp) modup_col_a<8, true>(P, B, primes, tw, L, K, log_n, m.dfwd, I0, Icnt, IG, pack, st);
        else modup_col_a<8, false>(P, B, primes, tw, L, K, log_n, 0, I0, Icnt, IG, pack, st);
        break;
    }
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

// Launches of at most this many workgroups prefetch a row pass's epilogue operands (PreOf): with
// the operands in registers the kernel runs at 3 instead of 4 waves/SIMD, which pays for latency-bound
// launches of a few rounds (ResNet's rescales and ModDowns) but not for the HMult tail's ~11k
// workgroups.
// (r05t: with the grouped epilogue loads of the large launches applied everywhere instead, the
// ResNet-20 batch ran at 1.398 instead of 1.450 images/s; the ops at 25-31 limbs measured equal)
static inline long row_pre_max_wg()
{
    return 8192L;
}

template <int PASS, int LOGR, class Job, bool FP>
static inline void launch_pass_a(const Job &job, int log_n, int jobs, long long twd, hipStream_t st)
{
    constexpr int LOGT = LOGR <= 7 ? 3 : 4;
    using SH = Shape<LOGR, LOGT>;
    const int subs = 1 << (log_n - LOGR);
    dim3 grid(subs / SH::S, jobs);
    // if constexpr: only the pass asked for is instantiated for this Job (four kernels per Job
    // otherwise, most of them never launched)
    if constexpr (PASS == FWD_COL) hipLaunchKernelGGL((k_fwd_col<LOGR, LOGT, Job, FP>), grid, dim3(256), 0, st, job, log_n, twd);
    if constexpr (PASS == FWD_ROW)
    {
        if constexpr (MHE_ROW3 && FP && LOGR == 8)
        {
            if (log_n == 16)
            {
                hipLaunchKernelGGL((k_fwd_row3<Job>), dim3(subs / 8, jobs), dim3(256), 0, st, job, log_n, twd);
                return;
            }
        }
        if ((long)grid.x * grid.y <= row_pre_max_wg())
            hipLaunchKernelGGL((k_fwd_row<LOGR, LOGT, Job, FP, true>), grid, dim3(256), 0, st, job, log_n, twd);
        else
            hipLaunchKernelGGL((k_fwd_row<LOGR, LOGT, Job, FP, false>), grid, dim3(256), 0, st, job, log_n, twd);
    }
    if constexpr (PASS == INV_ROW)
    {
        if constexpr (MHE_ROW3 && FP && LOGR == 8)
        {
            if (log_n == 16)
            {
                hipLaunchKernelGGL((k_inv_row3<Job>), dim3(subs / 8, jobs), dim3(256), 0, st, job, log_n, twd);
                return;
            }
        }
        hipLaunchKernelGGL((k_inv_row<LOGR, LOGT, Job, FP>), grid, dim3(256), 0, st, job, log_n, twd);
    }
    if constexpr (PASS == INV_COL) hipLaunchKernelGGL((k_inv_col<LOGR, LOGT, Job, FP>), grid, dim3(256), 0, st, job, log_n, twd);
}

template <int PASS, int LOGR, class Job>
static inline void launch_pass(const Job &job, int log_n, int jobs, const NttMode &m, hipStream_t st)
{
    const long long d = (PASS == FWD_COL || PASS == FWD_ROW) ? m.dfwd : m.dinv;
    if (m.fp)
        launch_pass_a<PASS, LOGR, Job, true>(job, log_n, jobs, d, st);
    else
        launch_pass_a<PASS, LOGR, Job, false>(job, log_n, jobs, 0, st);
}

template <int PASS, class Job>
static inline void launch_col(const Job &job, int log_n, int jobs, const NttMode &m, hipStream_t st)
{
    switch ((log_n + 1) / 2)
    {
    case 6: launch_pass<PASS, 6>(job, log_n, jobs, m, st); break;
    case 7: launch_pass<PASS, 7>(job, log_n, jobs, m, st); break;
    case 8: launch_pass<PASS, 8>(job, log_n, jobs, m, st); break;
    }
}

template <int PASS, class Job>
static inline void launch_row(const Job &job, int log_n, int jobs, const NttMode &m, hipStream_t st)
{
    switch (log_n / 2)
    {
    case 6: launch_pass<PASS, 6>(job, log_n, jobs, m, st); break;
    case 7: launch_pass<PASS, 7>(job, log_n, jobs, m, st); break;
    case 8: launch_pass<PASS, 8>(job, log_n, jobs, m, st); break;
    }
}

// MHE_ICOL_PER=1..MHE_ICOL_G (A/B runs): output primes per lift workgroup, instead of the size rule
static inline int icol_per_override()
{
    static const int v = [] {
        const char *e = getenv("MHE_ICOL_PER");
        const int x = e ? atoi(e) : 0;
        return x >= 1 && x <= MHE_ICOL_G ? x : 0;
    }();
    return v;
}
// k_icol_lift over `polys` source polys (all batch entries: cs.per polys each) and `cnt` output
// primes each (job index s * cnt + i), the column-pass shape of launch_col; IG groups of output
// primes per (column block, poly)
template <int LOGR, class Job, bool FP>
static inline void icol_lift_a(const ColSrc &cs, const Job &job, int polys, int cnt, int log_n, long long dinv,
                               long long dfwd, hipStream_t st)
{
    constexpr int LOGT = LOGR <= 7 ? 3 : 4;
    using SH = Shape<LOGR, LOGT>;
    const int subs = 1 << (log_n - LOGR);
    // output primes per workgroup: each workgroup redoes the inverse column stages of its columns
    // (from L2) once per group, so small launches keep one prime per workgroup (the widest grid) and
    // batched ones share the inverse stages over 2 to MHE_ICOL_G primes (ubench at 31 / 20 limbs, profiles/r03v:
    // 4 rescales 207 -> 185 us)
    const int jobs = polys * cnt;
    int per = jobs >= 128 ? MHE_ICOL_G : jobs >= 56 ? 2 : 1;
    if (const int po = icol_per_override()) per = po;
    const int IG = (cnt + per - 1) / per;
    hipLaunchKernelGGL((k_icol_lift<LOGR, LOGT, Job, FP>), dim3(subs / SH::S, polys, IG), dim3(256), 0, st, cs, job,
                       cnt, log_n, dinv, dfwd);
}
template <class Job>
static inline void icol_lift(const ColSrc &cs, const Job &job, int polys, int cnt, int log_n, const NttMode &m,
                             hipStream_t st)
{
    if (cnt <= 0 || polys <= 0) return;
    switch ((log_n + 1) / 2)
    {
    case 6:
        if (m.fp) icol_lift_a<6, Job, true>(cs, job, polys, cnt, log_n, m.dinv, m.dfwd, st);
        else icol_lift_a<6, Job, false>(cs, job, polys, cnt, log_n, 0, 0, st);
        break;
    case 7:
        if (m.fp) icol_lift_a<7, Job, true>(cs, job, polys, cnt, log_n, m.dinv, m.dfwd, st);
        else icol_lift_a<7, Job, false>(cs, job, polys, cnt, log_n, 0, 0, st);
        break;
    case 8:
        if (m.fp) icol_lift_a<8, Job, true>(cs, job, polys, cnt, log_n, m.dinv, m.dfwd, st);
        else icol_lift_a<8, Job, false>(cs, job, polys, cnt, log_n, 0, 0, st);
        break;
    }
}
// k_col_lift2 over `polys` source polys and `cnt` output primes each (job s * cnt + i), FP contexts
template <int LOGR, class Job>
static inline void col_lift2_a(const Job &job, int polys, int cnt, int log_n, long long dfwd, hipStream_t st)
{
    constexpr int LOGT = LOGR <= 7 ? 3 : 4;
    using SH = Shape<LOGR, LOGT>;
    const int subs = 1 << (log_n - LOGR);
    const int jobs = polys * cnt;
    int per = jobs >= 128 ? MHE_ICOL_G : jobs >= 56 ? 2 : 1; // as icol_lift_a
    if (const int po = icol_per_override()) per = po;
    const int IG = (cnt + per - 1) / per;
    hipLaunchKernelGGL((k_col_lift2<LOGR, LOGT, Job>), dim3(subs / SH::S, polys, IG), dim3(256), 0, st, job, cnt, log_n,
                       dfwd);
}
template <class Job>
static inline void col_lift2(const Job &job, int polys, int cnt, int log_n, const NttMode &m, hipStream_t st)
{
    if (cnt <= 0 || polys <= 0 || m.fp != 1) return;
    switch ((log_n + 1) / 2)
    {
    case 6: col_lift2_a<6>(job, polys, cnt, log_n, m.dfwd, st); break;
    case 7: col_lift2_a<7>(job, polys, cnt, log_n, m.dfwd, st); break;
    case 8: col_lift2_a<8>(job, polys, cnt, log_n, m.dfwd, st); break;
    }
}
template <class Job> static inline void fwd_col(const Job &j, int log_n, int jobs, const NttMode &m, hipStream_t st) { launch_col<FWD_COL>(j, log_n, jobs, m, st); }
template <class Job> static inline void fwd_row(const Job &j, int log_n, int jobs, const NttMode &m, hipStream_t st) { launch_row<FWD_ROW>(j, log_n, jobs, m, st); }
template <class Job> static inline void inv_row(const Job &j, int log_n, int jobs, const NttMode &m, hipStream_t st) { launch_row<INV_ROW>(j, log_n, jobs, m, st); }
template <class Job> static inline void inv_col(const Job &j, int log_n, int jobs, const NttMode &m, hipStream_t st) { launch_col<INV_COL>(j, log_n, jobs, m, st); }

// ============================================================================
// Fused key-switching ModUp row pass + key inner product (evaluator.cpp:2386-2463).
//
// One workgroup owns output prime I (blockIdx.y; I == L is the special prime) and S blocks of
// R = 2^LOGR coefficients; blockIdx.z is the batch entry (KsPtrs).  For every digit J it takes
// the column-pass output of (I, J) (or, for I == J, the input target limb, already in NTT
// form), finishes the forward NTT in registers, and multiply-accumulates with key[J][0][I] and
// key[J][1][I] into 128-bit accumulators.  NTT'd digits never touch HBM; each key residue is
// read once.
//   * 8 residues per lane keep the 2 x 8 x 128-bit accumulators at 64 VGPRs; the 2^LOGR-point
//     row transform runs as radix-8 register phases with swizzled (conflict-free) LDS
//     transposes.
//   * The row-pass twiddles depend on (I, block) but not on J, so they are staged in LDS
//     once per workgroup; no global load is left inside the digit loop except the digit and
//     key streams, which are issued one digit (digits) / one NTT (key) ahead.
//   * Barriers wait on LDS only (s_waitcnt lgkmcnt(0) + s_barrier): __syncthreads() would
//     also drain vmcnt and serialise the prefetch (cdna_hip_programming.md §8).
template <int LOGR>
struct RowMacShape
{
    static constexpr int R = 1 << LOGR;
    static constexpr int E = 8;
    static constexpr int TPS = R / E;     // lanes per block
    static_assert(TPS <= 64, "a block's transposes must stay inside one wave");
    static constexpr int S = 256 / TPS;   // blocks per workgroup
};



// Slot of twiddle entry k in a block's LDS row.  The last stages read entries 4 apart across the
// lanes (16-byte entries: a 64-byte stride), a 4-way conflict for ds_read_b128's 16-lane groups;
// XOR-ing bits 4-5 into bits 0-1 with an unpadded row makes every stage's reads conflict-free
// (bank model of MI355X_MICROARCH.md §LDS; SQ_LDS_BANK_CONFLICT was 0.55x the LDS busy cycles).
__device__ __forceinline__ u32 twz(u32 k)
{
    return k ^ ((k >> 4) & 3);
}

// Forward stages [s0, s1) of the local 2^LOGR transform, twiddles from the block's LDS row
// (entry (1 << s) + g, at slot twz(.), holds tw[((2^k1 + b) << s) + g]).
template <int LOGR, class A>
__device__ __forceinline__ void row_stages(typename A::T (&v)[8], u32 t, int b_lo, int s0, int s1,
                                           const typename A::TW *twl, const A &ar, int /*deduce*/ = 0)
{
#pragma unroll
    for (int s = s0; s < s1; s++)
        ar.template fwd_tab<8>(v, 1 << (LOGR - 1 - s - b_lo), twl, // gap in slot units
                               [&](int e) { return twz((1u << s) + (lay(t, e, b_lo) >> (LOGR - s))); });
}

template <int LOGR, bool FP, bool MIX = false>
#ifndef MHE_KS_OCC
#define MHE_KS_OCC 3 // waves per SIMD the FP64 fused MAC at n = 2^16 is compiled for: 168 VGPRs, one LDS
                     // transpose buffer (48 KB).  With the loads at the top of each digit (MHE_KS_SB)
                     // C2's k_ks_row_mac 2743 -> 2698 us, ResNet-level ops equal (profiles/r06n); without
                     // them 3 waves were equal on C2 and 2 % slower on single key switches (r06c)
#endif
#ifndef MHE_KS_PP
#define MHE_KS_PP 0 // digit loop unrolled twice, prefetched digit in alternating registers
#endif
#ifndef MHE_KS_KPF
#define MHE_KS_KPF 0 // key limbs loaded one digit ahead too (32 VGPRs more)
#endif
#ifndef MHE_KS_SB
#define MHE_KS_SB 1 // digit loop: key and next-digit loads issued at the top of the step (sched_barrier)
#endif
#ifndef MHE_KS_FL
#define MHE_KS_FL 1 // keys and accumulators in the row transform's last layout (no transpose back per digit)
#endif
__global__ __launch_bounds__(256, (FP && !MIX && LOGR == 8) ? MHE_KS_OCC : 2) void k_ks_row_mac(KsPtrs P, const PrimeDev *__restrict__ primes,
                                                       const Tw *__restrict__ tw_all, int L, int K, int log_n,
                                                       long long twd, int I0, int pack, int kpack, int share,
                                                       const Tw *__restrict__ itw_all, long long tinv, int inv_special)
{
    // tile (bx = column block group, by = output prime) and batch entry bz.  With `share` (every
    // entry reads the same key, gridDim.x * gridDim.y a multiple of 8) the linear workgroup ids are
    // dealt so that the gridDim.z entries of one tile are ids 8 apart and adjacent in dispatch
    // order: workgroups go to the 8 XCDs round robin, so all entries of a tile run on one XCD at
    // the same time and the key stream is fetched from HBM once and hit in that XCD's L2 by the
    // others.
    u32 bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    if (share)
    {
        const u32 X = gridDim.x, Y = gridDim.y, Bn = gridDim.z;
        const u32 id = blockIdx.x + X * (blockIdx.y + Y * blockIdx.z);
        const u32 r = id % (8 * Bn), tile = (id / (8 * Bn)) * 8 + r % 8;
        bz = r / 8;
        bx = tile % X;
        by = tile / X;
    }
    if (P.run_if[bz] && !*P.run_if[bz]) return; // uniform, before any barrier
    // batch entry bz: inter [cnt][L][n] column-pass output, target [L][n] NTT form,
    // key [digits][2][key_limbs][n], acc [2][L+1][n]
    const u64 *__restrict__ inter = P.inter[bz];
    const u64 *__restrict__ target = P.target[bz];
    const u64 *__restrict__ key = P.key[bz];
    u64 *__restrict__ acc = P.acc[bz];
    const int key_limbs = P.key_limbs[bz];
    using SH = RowMacShape<LOGR>;
    using A = NttArith<FP>;
    using T = typename A::T;
    using TW = typename A::TW;
    constexpr int R = SH::R, TPS = SH::TPS, S = SH::S;
    constexpr int B_A = LOGR - 3, B_B = LOGR - 6;
    static_assert(LOGR >= 6, "the row transform ends in layout lay(t, e, 0)");
    // layout of the key limbs, the input limb and the accumulators: the row transform's last
    // (lay(t, e, 0): 8 consecutive residues per lane) with MHE_KS_FL, so a digit needs no transpose
    // back to the coalesced layout lay(t, e, B_A) -- the accumulators take it once, at the end
    constexpr int BK = MHE_KS_FL ? 0 : B_A;
    // one transpose buffer is enough (every transpose stays inside one wave and a wave's LDS
    // operations complete in order; the fences only stop the compiler from reordering them):
    // 48 KB per workgroup fits 3 workgroups per CU, two buffers (64 KB) only 2
    constexpr int XCH = (FP && !MIX && LOGR == 8 && MHE_KS_OCC >= 3) ? 1 : 2;
    __shared__ T xch[XCH][S * R];
    __shared__ TW twl[S * R];
    const int j0 = 0, j1 = L;
    const u32 tid = threadIdx.x, t = tid % TPS, sl = tid / TPS;
    const u32 b = bx * S + sl;
    const u32 base = b << LOGR;
    const u32 R1 = 1u << (log_n - LOGR);
    const int I = I0 + (int)by; // inter holds output primes I0 .. I0 + gridDim.y - 1
    const int pi = (I == L) ? K - 1 : I;
    const int ki = (I == L) ? key_limbs - 1 : I;
    const PrimeDev p = primes[pi];
    const size_t n = (size_t)1 << log_n;
    const size_t kstride = (size_t)key_limbs * n;
    const A ar0(p, tw_all + ((size_t)pi << log_n), twd);

    auto run = [&](const auto &ar) {
        // the arithmetic of this workgroup's prime: FP64, or (MIX, a prime >= 2^51) integer, with the
        // LDS buffers reinterpreted (8-byte residues, 16-byte twiddles either way)
        using AR = typename std::decay<decltype(ar)>::type;
        using T = typename AR::T;
        using TW = typename AR::TW;
        constexpr bool FPA = !std::is_same<T, u64>::value;
        TW *const twl_a = reinterpret_cast<TW *>(twl);
        // stage this workgroup's row-pass twiddles (all digits share them)
        {
            const TW *tw = ar.tw;
            for (u32 idx = tid; idx < (u32)(S * R); idx += 256)
            {
                const u32 blk = idx / R, k = idx % R;
                if (k == 0) continue;
                const int s = 31 - __builtin_clz(k);
                twl_a[blk * R + twz(k)] = tw[(((R1 + bx * S + blk) << s)) + (k - (1u << s))];
            }
        }
        const TW *mytw = &twl_a[sl * R];
        T *x0 = reinterpret_cast<T *>(&xch[0][sl * R]), *x1 = reinterpret_cast<T *>(&xch[XCH - 1][sl * R]);
        // FP: the key inner products run in FP64 as well (fp_mulmod_gen); with q < 2^47 and
        // 1.25 (j1 - j0) q < 2^53 (LZ, chosen below) the digits stay unreduced and the products
        // (|.| < 1.25q each) sum exactly, otherwise digits are reduced and the sums every second
        // digit.  Integer: 128-bit
        // accumulation, one Barrett reduction at the end (evaluator.cpp:2412-2462).
        constexpr bool LZ = std::is_same<AR, NttArithF<true>>::value;
        using AccT = typename std::conditional<FPA, double, Acc128>::type;
        AccT a0[8], a1[8];
#pragma unroll
        for (int e = 0; e < 8; e++)
        {
            if constexpr (FPA)
                a0[e] = a1[e] = 0.0;
            else
                a0[e] = a1[e] = Acc128{ 0, 0 };
        }

        // Digit J of this output prime is the input limb itself (J == I, already NTT form) or the
        // column-pass output, packed (tile16) when the column pass packed it.  The input limb is
        // taken first, on its own; the loop then runs over the other digits in order (I skipped),
        // so every iteration issues the same load instructions from the same per-lane offsets
        // (only the uniform base moves) -- with the input limb inside the loop, the compiler
        // selected between two offset sets and rebuilt 16 64-bit addresses per digit.  The loop is
        // unrolled twice with the prefetched digit in alternating registers (no copies), and
        // instantiated per (packed intermediate, prepared key) pair, uniform per workgroup.  The
        // last digit's prefetch is repeated past the end: with a data-dependent load count the
        // compiler drained every load in flight (vmcnt(0)) at the top of each digit.
        const bool pk = inter_packed(pack, p.q); // uniform per workgroup
        // a prepared slot (mhe_key_prepare): the residues as doubles (no unpacking) or as 48-bit planes
        const int kfmt = kpack ? key_slot_format(key[(size_t)ki * n + n - 1]) : 0; // uniform
        const bool has_self = I < L;                                                 // uniform
        const int nd = has_self ? L - 1 : L; // digits other than I
        auto loop = [&](auto pk_c, auto kf_c) {
            constexpr bool PK = decltype(pk_c)::value;
            constexpr int KF = decltype(kf_c)::value; // key slot format (key_slot_format)
            auto digit_of = [&](int u) { return u + ((has_self && u >= I) ? 1 : 0); };
            // packed digit slots at n = 2^16: byte offsets of this lane's residue 0 in the 32-bit
            // plane and in the 16-bit plane (which starts at 4n)
            const u32 off_lo = 4u * tile16(base + lay(t, 0, B_A));
            const u32 off_hi = 4u * (u32)n + 2u * tile16h(base + lay(t, 0, B_A));
            auto load_inter = [&](int J, u64 (&v)[8]) {
                if constexpr (PK && LOGR == 8)
                {
                    // buffer loads: the digit's slot as a descriptor built from uniform values and
                    // loop-invariant 32-bit lane offsets (global loads rebuilt a 64-bit address per
                    // load and digit).  At n = 2^16 a lane's residues e = 0..7 are one column block
                    // apart in both planes: tile16 / tile16h of base + lay(t, e, 5) grow by 512 e.
                    const u64 *slot = inter + ((size_t)(I - I0) * L + J) * n;
                    const __amdgpu_buffer_rsrc_t rs =
                        __builtin_amdgcn_make_buffer_rsrc(const_cast<u64 *>(slot), 0, (int)(8 * n), 0x00020000);
                    constexpr int AUX = ((MHE_NT >> 2) & 1) ? 2 : 0; // nt
#pragma unroll
                    for (int e = 0; e < 8; e++)
                    {
                        // the per-residue step as the scalar offset: two lane offsets in VGPRs
                        const u32 l = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)off_lo, 2048 * e, AUX);
                        const u32 h = __builtin_amdgcn_raw_buffer_load_b16(rs, (int)off_hi, 1024 * e, AUX);
                        v[e] = (u64)l | ((u64)h << 32);
                    }
                }
                else if constexpr (PK)
                {
                    const u32 *lo = reinterpret_cast<const u32 *>(inter + ((size_t)(I - I0) * L + J) * n);
                    const unsigned short *hi = reinterpret_cast<const unsigned short *>(lo + n);
#pragma unroll
                    for (int e = 0; e < 8; e++)
                    {
                        const u32 idx = base + lay(t, e, B_A);
                        v[e] = (u64)ld_nt<2>(&lo[tile16(idx)]) | ((u64)ld_nt<2>(&hi[tile16h(idx)]) << 32);
                    }
                }
                else
                {
                    const u64 *src = inter + ((size_t)(I - I0) * L + J) * n + base;
#pragma unroll
                    for (int e = 0; e < 8; e++) v[e] = ld_nt<2>(&src[lay(t, e, B_A)]);
                }
            };
            // key limbs of a digit: issued at the top of the digit, consumed after the digit's NTT
            // (a one-digit-ahead key prefetch measured equal and costs 32 VGPRs)
            auto load_key = [&](int J, u64 (&ka)[8], u64 (&kb)[8]) {
                const u64 *k0 = key + (size_t)(2 * J) * kstride + (size_t)ki * n;
                const u64 *k1 = k0 + kstride;
                if constexpr (KF == 2)
                {
                    const u32 *l0 = reinterpret_cast<const u32 *>(k0) + base;
                    const u32 *l1 = reinterpret_cast<const u32 *>(k1) + base;
                    const unsigned short *h0 = reinterpret_cast<const unsigned short *>(reinterpret_cast<const u32 *>(k0) + n) + base;
                    const unsigned short *h1 = reinterpret_cast<const unsigned short *>(reinterpret_cast<const u32 *>(k1) + n) + base;
#pragma unroll
                    for (int e = 0; e < 8; e++)
                    {
                        const u32 r = lay(t, e, BK);
                        ka[e] = (u64)ld_nt<1>(&l0[r]) | ((u64)ld_nt<1>(&h0[r]) << 32);
                        kb[e] = (u64)ld_nt<1>(&l1[r]) | ((u64)ld_nt<1>(&h1[r]) << 32);
                    }
                }
                else
                {
#pragma unroll
                    for (int e = 0; e < 8; e++)
                    {
                        ka[e] = ld_nt<1>(&k0[base + lay(t, e, BK)]);
                        kb[e] = ld_nt<1>(&k1[base + lay(t, e, BK)]);
                    }
                }
            };
            // d (the digit in the coalesced layout, NTT form) times both key limbs; `odd` is the
            // parity of the digits taken so far (the non-lazy FP sums are reduced every second one)
            auto mac = [&](const T (&d)[8], const u64 (&ka)[8], const u64 (&kb)[8], bool odd) {
                if constexpr (FPA)
                {
#pragma unroll
                    for (int e = 0; e < 8; e++)
                    {
                        const double dv = LZ ? d[e] : fp_reduce(d[e], ar.q, ar.qinv);
                        // canonical key residues
                        const double k0v = KF == 1 ? key_word_f(ka[e]) : fp_from_u52(ka[e]);
                        const double k1v = KF == 1 ? key_word_f(kb[e]) : fp_from_u52(kb[e]);
                        a0[e] += fp_mulmod_gen(dv, k0v, ar.q, ar.qinv);
                        a1[e] += fp_mulmod_gen(dv, k1v, ar.q, ar.qinv);
                        if (!LZ && odd)
                        {
                            a0[e] = fp_reduce(a0[e], ar.q, ar.qinv);
                            a1[e] = fp_reduce(a1[e], ar.q, ar.qinv);
                        }
                    }
                }
                else
                {
#pragma unroll
                    for (int e = 0; e < 8; e++)
                    {
                        mac128(a0[e], d[e], KF == 1 ? key_word_u(ka[e]) : ka[e]);
                        mac128(a1[e], d[e], KF == 1 ? key_word_u(kb[e]) : kb[e]);
                    }
                }
            };
            // the row stages of a column-pass output (J != I)
            auto ntt_digit = [&](const u64 (&vin)[8], T (&d)[8]) {
                T w[8];
#pragma unroll
                for (int e = 0; e < 8; e++)
                {
                    // the column-pass output: FP and packed, a centred 48-bit residue (fp_to_s48);
                    // otherwise canonical
                    if constexpr (FPA)
                        w[e] = PK ? fp_from_s48(vin[e]) : ar.in52(vin[e]);
                    else
                        w[e] = ar.in52(vin[e]);
                }
                // LDS slots of the transposes: swz is linear over GF(2) and lay(t, e, b) is the
                // disjoint OR of a lane part and e << b, so slot = swz(lane part) ^ swz(e << b).  The
                // non-lazy sweep (more live values) recomputes the XORs from three per-lane bases
                // each digit (asm barrier: not hoisted) instead of keeping 24 slots in VGPRs, which
                // at 3 waves/SIMD were spilled and reloaded behind vmcnt(0) every digit.
                u32 sa = swz(lay(t, 0, B_A)), sb = swz(lay(t, 0, B_B)), s0 = swz(lay(t, 0, 0));
                if constexpr (!LZ) asm volatile("" : "+v"(sa), "+v"(sb), "+v"(s0));
                auto slot = [&](u32 lane_part, int e, int b) { return lane_part ^ swz((u32)e << b); };
                row_stages<LOGR>(w, t, B_A, 0, 3, mytw, ar);
                wave_lds_fence(); // the previous digit's reads of x0 come first
#pragma unroll
                for (int e = 0; e < 8; e++) x0[slot(sa, e, B_A)] = w[e];
                wave_lds_fence();
#pragma unroll
                for (int e = 0; e < 8; e++) w[e] = x0[slot(sb, e, B_B)];
                row_stages<LOGR>(w, t, B_B, 3, 6, mytw, ar);
                T *xl = x1;
                int bl = B_B;
                if (LOGR > 6)
                {
                    wave_lds_fence();
#pragma unroll
                    for (int e = 0; e < 8; e++) x1[slot(sb, e, B_B)] = w[e];
                    wave_lds_fence();
#pragma unroll
                    for (int e = 0; e < 8; e++) w[e] = x1[slot(s0, e, 0)];
                    row_stages<LOGR>(w, t, 0, 6, LOGR, mytw, ar);
                    xl = x0;
                    bl = 0;
                }
                if constexpr (MHE_KS_FL)
                {
                    // already the keys' layout (integer: canonical digits keep the 128-bit sums
                    // exact for any digit count below 2^8)
#pragma unroll
                    for (int e = 0; e < 8; e++)
                    {
                        if constexpr (FPA)
                            d[e] = w[e];
                        else
                            d[e] = ar.canon(w[e]);
                    }
                    return;
                }
                // back to the coalesced layout of the key stream (integer: canonical digits keep
                // the 128-bit sums exact for any digit count below 2^8)
                wave_lds_fence();
#pragma unroll
                for (int e = 0; e < 8; e++)
                {
                    if constexpr (FPA)
                        xl[swz(lay(t, e, bl))] = w[e];
                    else
                        xl[swz(lay(t, e, bl))] = ar.canon(w[e]);
                }
                wave_lds_fence();
#pragma unroll
                for (int e = 0; e < 8; e++) d[e] = xl[swz(lay(t, e, B_A))];
            };
            u64 ka[8], kb[8], va[8], vb[8];
            if (nd > 0) load_inter(digit_of(0), va); // nd == 0: one data limb, output prime 0
            lds_barrier();                             // twiddles visible
            if (has_self)
            {
                // the input limb of digit I: a canonical ciphertext limb, already NTT form
                const u64 *src = target + (size_t)I * n + base;
#pragma unroll
                for (int e = 0; e < 8; e++) vb[e] = ld_nt<2>(&src[lay(t, e, BK)]);
                load_key(I, ka, kb);
                T d[8];
#pragma unroll
                for (int e = 0; e < 8; e++) d[e] = ar.in52(vb[e]);
                mac(d, ka, kb, false);
            }
            const int c0 = has_self ? 1 : 0; // digits taken before the loop
#if MHE_KS_KPF
            // keys one digit ahead as well: digit u's key limbs are in ka / kb when its step starts
            if (nd > 0) load_key(digit_of(0), ka, kb);
            auto step = [&](int u, const u64 (&cur)[8], u64 (&nxt)[8]) {
                const int un = u + 1 < nd ? u + 1 : u;
                u64 na[8], nb[8];
                load_key(digit_of(un), na, nb);
                load_inter(digit_of(un), nxt); // one digit ahead
                T d[8];
                ntt_digit(cur, d);
                mac(d, ka, kb, ((u + c0) & 1) != 0);
#pragma unroll
                for (int e = 0; e < 8; e++)
                {
                    ka[e] = na[e];
                    kb[e] = nb[e];
                }
            };
#else
            auto step = [&](int u, const u64 (&cur)[8], u64 (&nxt)[8]) {
                load_key(digit_of(u), ka, kb);
                load_inter(digit_of(u + 1 < nd ? u + 1 : u), nxt); // one digit ahead
                // issue both streams before the digit's transform: left to the scheduler, they went
                // out a quarter into it and the copy of the prefetched digit at the end of the step
                // waited for them (vmcnt(0)).  FP64 without MIX only: the integer and MIX variants
                // spill already and spilled more
                if constexpr (MHE_KS_SB && FP && !MIX) __builtin_amdgcn_sched_barrier(0);
                T d[8];
                ntt_digit(cur, d);
                mac(d, ka, kb, ((u + c0) & 1) != 0);
            };
#endif
#if MHE_KS_PP
            int u = 0;
            for (; u + 1 < nd; u += 2)
            {
                step(u, va, vb);
                step(u + 1, vb, va);
            }
            if (u < nd) step(u, va, vb);
#else
            for (int u = 0; u < nd; u++)
            {
                step(u, va, vb);
#pragma unroll
                for (int e = 0; e < 8; e++) va[e] = vb[e];
            }
#endif
        };
        using F0 = std::integral_constant<int, 0>;
        using F1 = std::integral_constant<int, 1>;
        using F2 = std::integral_constant<int, 2>;
        if (pk)
        {
            if (kfmt == 1) loop(std::true_type{}, F1{});
            else if (kfmt == 2) loop(std::true_type{}, F2{});
            else loop(std::true_type{}, F0{});
        }
        else
        {
            if (kfmt == 1) loop(std::false_type{}, F1{});
            else if (kfmt == 2) loop(std::false_type{}, F2{});
            else loop(std::false_type{}, F0{});
        }
        u64 *o0 = acc + (size_t)I * n + base;
        u64 *o1 = o0 + (size_t)(L + 1) * n;
        if (inv_special && I == L) // uniform per workgroup
        {
            // The ModDown's first step, the inverse row pass of the special limbs (k_inv_row with
            // JobStrided, evaluator.cpp:2466-2475), on this workgroup's rows: its accumulators are
            // whole 2^LOGR-blocks, so the Gentleman-Sande stages LOGR-1 .. 0 run here -- in-lane
            // position bits 0-2, then 3-5, then the rest, with the same swizzled in-wave transposes
            // -- and the separate launch (and its HBM round trip) disappears.  Canonical output.
            using AI = NttArith<FPA>;
            const AI ai(p, itw_all + ((size_t)pi << log_n), tinv);
            const u32 rbi = R1 + b;
            auto tr = [&](T (&w)[8], int from, int to) {
                wave_lds_fence();
#pragma unroll
                for (int e = 0; e < 8; e++) x0[swz(lay(t, e, from))] = w[e];
                wave_lds_fence();
#pragma unroll
                for (int e = 0; e < 8; e++) w[e] = x0[swz(lay(t, e, to))];
            };
            auto stages = [&](T (&w)[8], int b_lo, int s_hi, int s_lo) {
#pragma unroll
                for (int s = s_hi; s >= s_lo; s--)
                    ai.template inv<8>(w, 1 << (LOGR - 1 - s - b_lo),
                                       [&](int e) { return (rbi << s) + (lay(t, e, b_lo) >> (LOGR - s)); });
            };
            auto inv_rows = [&](T (&w)[8]) {
                if constexpr (BK != 0) tr(w, BK, 0);
                stages(w, 0, LOGR - 1, LOGR - 3);
                tr(w, 0, 3);
                stages(w, 3, LOGR - 4, LOGR > 6 ? LOGR - 6 : 0);
                if (LOGR > 6)
                {
                    tr(w, 3, B_A);
                    stages(w, B_A, LOGR - 7, 0);
                }
            };
            T w0[8], w1[8];
#pragma unroll
            for (int e = 0; e < 8; e++)
            {
                if constexpr (FPA)
                {
                    w0[e] = fp_reduce(a0[e], ar.q, ar.qinv);
                    w1[e] = fp_reduce(a1[e], ar.q, ar.qinv);
                }
                else
                {
                    w0[e] = barrett128(a0[e].lo, a0[e].hi, p);
                    w1[e] = barrett128(a1[e].lo, a1[e].hi, p);
                }
            }
            inv_rows(w0);
            inv_rows(w1);
#pragma unroll
            for (int e = 0; e < 8; e++)
            {
                const u32 r = lay(t, e, B_A);
                o0[r] = ai.canon(w0[e]);
                o1[r] = ai.canon(w1[e]);
            }
            return;
        }
        u64 c0v[8], c1v[8]; // canonical key products, layout BK
#pragma unroll
        for (int e = 0; e < 8; e++)
        {
            if constexpr (FPA)
            {
                c0v[e] = fp_canon(a0[e], ar.q, ar.qinv);
                c1v[e] = fp_canon(a1[e], ar.q, ar.qinv);
            }
            else
            {
                c0v[e] = barrett128(a0[e].lo, a0[e].hi, p);
                c1v[e] = barrett128(a1[e].lo, a1[e].hi, p);
            }
        }
        if constexpr (BK != B_A)
        {
            // one transpose per workgroup to the coalesced layout for the stores
            u64 *xu = reinterpret_cast<u64 *>(x0);
            auto back = [&](u64 (&v)[8]) {
                wave_lds_fence();
#pragma unroll
                for (int e = 0; e < 8; e++) xu[swz(lay(t, e, BK))] = v[e];
                wave_lds_fence();
#pragma unroll
                for (int e = 0; e < 8; e++) v[e] = xu[swz(lay(t, e, B_A))];
            };
            back(c0v);
            back(c1v);
        }
#pragma unroll
        for (int e = 0; e < 8; e++)
        {
            const u32 r = lay(t, e, B_A);
            o0[r] = c0v[e];
            o1[r] = c1v[e];
        }
    };
    if constexpr (FP)
    {
        // lazy digits and sums only while this group's j1 - j0 products (|.| < 1.25q each) sum
        // exactly: 1.25 (j1 - j0) q < 2^53 (q < 2^47 allows up to 51 digits per group)
        if (MIX && !(p.q < (1ull << 51)))
            run(NttArith<false>(p, tw_all + ((size_t)pi << log_n), 0));
        else if (p.q < (1ull << 47) && (double)(j1 - j0) * 1.25 * (double)p.q < 9007199254740992.0)
            run(NttArithF<true>(p, tw_all + ((size_t)pi << log_n), twd));
        else
            run(ar0);
    }
    else
        run(ar0);
}

// measured at L=44: G=1 763, 2 738, 4 700 HMult/s (digit groups with a partial-sum reduction, since
// removed); ResNet-20 (L <= 31): G=1 0.865-0.873 images/s vs 0.832-0.839 with G=2
template <int LOGR, bool FP, bool MIX = false>
static inline int ks_row_mac_a(const KsPtrs &P, int B, const PrimeDev *primes, const Tw *tw, int L, int K, int log_n,
                               long long twd, int I0, int cnt, int pack, int kpack, int share, const Tw *itw,
                               long long tinv, int inv_special, hipStream_t st)
{
    const int blocks = 1 << (log_n - LOGR);
    if constexpr (MIX)
    {
        const dim3 g(blocks / RowMacShape<LOGR>::S, cnt, B);
        share = (share && B > 1 && (g.x * g.y) % 8 == 0) ? 1 : 0;
        hipLaunchKernelGGL((k_ks_row_mac<LOGR, true, true>), g, dim3(256), 0, st, P, primes, tw, L, K, log_n, twd,
                           I0, pack, kpack, share, itw, tinv, inv_special);
        return inv_special;
    }
    const dim3 grid(blocks / RowMacShape<LOGR>::S, cnt, B);
    share = (share && B > 1 && (grid.x * grid.y) % 8 == 0) ? 1 : 0;
    hipLaunchKernelGGL((k_ks_row_mac<LOGR, FP>), grid, dim3(256), 0, st, P, primes, tw, L, K, log_n, twd, I0,
                       pack, kpack, share, itw, tinv, inv_special);
    return inv_special;
}

template <int LOGR>
static inline int ks_row_mac_m(const KsPtrs &P, int B, const PrimeDev *primes, const Tw *tw, int L, int K, int log_n,
                               const NttMode &m, int I0, int cnt, int pack, int kpack, int share, const Tw *itw,
                               int inv_special, hipStream_t st)
{
    if (m.fp == 2)
        return ks_row_mac_a<LOGR, true, true>(P, B, primes, tw, L, K, log_n, m.dfwd, I0, cnt, pack, kpack, share, itw,
                                              m.dinv, inv_special, st);
    if (m.fp)
        return ks_row_mac_a<LOGR, true>(P, B, primes, tw, L, K, log_n, m.dfwd, I0, cnt, pack, kpack, share, itw, m.dinv,
                                        inv_special, st);
    return ks_row_mac_a<LOGR, false>(P, B, primes, tw, L, K, log_n, 0, I0, cnt, pack, kpack, share, itw, 0, inv_special,
                                     st);
}

// Fused row pass + MAC for output primes I0 .. I0+cnt-1 (each entry's inter holds exactly those),
// over B batch entries; share: every entry's key pointer is the same (XCD-grouped entries)
// inv_special: the launch covers the special prime (I = L) and may finish the special limbs' inverse
// row pass itself (itw: inverse twiddles); returns 1 when it did, 0 when k_inv_row must still run.
static inline int ks_row_mac_chunk(const KsPtrs &P, int B, const PrimeDev *primes, const Tw *tw, int L, int K,
                                   int log_n, const NttMode &m, int I0, int cnt, int pack, int kpack, int share,
                                   const Tw *itw, int inv_special, hipStream_t st)
{
    switch (log_n / 2)
    {
    case 6: return ks_row_mac_m<6>(P, B, primes, tw, L, K, log_n, m, I0, cnt, 0, kpack, share, itw, inv_special, st);
    case 7: return ks_row_mac_m<7>(P, B, primes, tw, L, K, log_n, m, I0, cnt, 0, kpack, share, itw, inv_special, st);
    case 8:
        return ks_row_mac_m<8>(P, B, primes, tw, L, K, log_n, m, I0, cnt, (pack && log_n == 16) ? 1 : 0, kpack, share,
                               itw, inv_special, st);
    }
    return 0;
}
