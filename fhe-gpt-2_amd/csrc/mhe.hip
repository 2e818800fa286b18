// libmhe: MI355X-native RNS-CKKS evaluator kernels behind the C ABI of include/mhe.h.
//
// Data layout in HBM: [poly][limb][n] u64, identical to SEAL's
// Ciphertext::data() so host<->device moves are single memcpys.  Per-context tables:
//   primes[K]        PrimeDev constants
//   tw[K][n]         (psi^rev(j), Shoup quotient)       -- NTTTables::root_powers_
//   itw[K][n]        (psi^-rev(j), Shoup quotient)      -- same transform as SEAL's scrambled
//                                                          inv_root_powers_, bit-reversed index
//   invq[K][K]       (q_j^-1 mod q_i, Shoup)            -- RNSTool::inv_q_last_mod_q for every j
// Scratch workspaces are per stream (see Workspace).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <atomic>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/mhe.h"
#include "arith.h"
#include "ntt.h"
#include "hoist.h"

#define MHE_EXPORT extern "C" __attribute__((visibility("default")))

typedef unsigned __int128 u128;

// ============================================================================ errors
static thread_local std::string g_err;

static int fail(int code, const std::string &msg)
{
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do                                                                                         \
    {                                                                                          \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) return fail(MHE_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

#define HIP_LAUNCH_CHECK()                                                                     \
    do                                                                                         \
    {                                                                                          \
        hipError_t e_ = hipGetLastError();                                                     \
        if (e_ != hipSuccess) return fail(MHE_ERR_DEVICE, std::string("kernel launch: ") + hipGetErrorString(e_)); \
    } while (0)

// ===================================================================== host number theory
// (product code: the engine builds its own tables; it never calls the test oracle)
namespace host
{
static u64 mulmod(u64 a, u64 b, u64 q)
{
    return (u64)((u128)a * b % q);
}

static u64 powmod(u64 b, u64 e, u64 q)
{
    u64 r = 1 % q;
    b %= q;
    while (e)
    {
        if (e & 1) r = mulmod(r, b, q);
        b = mulmod(b, b, q);
        e >>= 1;
    }
    return r;
}

// try_invert_uint_mod (util/numth.h:145)
static bool invmod(u64 a, u64 q, u64 &out)
{
    __int128 r0 = q, r1 = a % q, s0 = 0, s1 = 1;
    if (r1 == 0) return false;
    while (r1)
    {
        __int128 qt = r0 / r1, r2 = r0 - qt * r1, s2 = s0 - qt * s1;
        r0 = r1;
        r1 = r2;
        s0 = s1;
        s1 = s2;
    }
    if (r0 != 1) return false;
    __int128 v = s0 % (__int128)q;
    if (v < 0) v += q;
    out = (u64)v;
    return true;
}

// is_prime (util/numth.cpp:179-277): deterministic Miller-Rabin bases for 64-bit inputs.
static bool is_prime(u64 v)
{
    if (v < 2) return false;
    static const u64 sm[] = { 2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37 };
    for (u64 p : sm)
    {
        if (v == p) return true;
        if (v % p == 0) return false;
    }
    u64 d = v - 1;
    int r = 0;
    while (!(d & 1))
    {
        d >>= 1;
        r++;
    }
    for (u64 a : sm)
    {
        u64 x = powmod(a, d, v);
        if (x == 1 || x == v - 1) continue;
        bool ok = false;
        for (int i = 0; i < r - 1; i++)
        {
            x = mulmod(x, x, v);
            if (x == v - 1)
            {
                ok = true;
                break;
            }
        }
        if (!ok) return false;
    }
    return true;
}

// try_minimal_primitive_root (util/numth.cpp:398-424): smallest primitive degree-th root.
static u64 minimal_primitive_root(u64 degree, u64 q)
{
    u64 quo = (q - 1) / degree;
    if (quo * degree != q - 1) return 0;
    u64 root = 0;
    for (u64 c = 2; c < q && !root; c++)
    {
        u64 g = powmod(c, quo, q);
        if (g && powmod(g, degree >> 1, q) == q - 1) root = g;
    }
    if (!root) return 0;
    u64 gsq = mulmod(root, root, q), cur = root, best = root;
    for (u64 i = 0; i < degree; i++)
    {
        if (cur < best) best = cur;
        cur = mulmod(cur, gsq, q);
    }
    return best;
}

static u64 shoup(u64 w, u64 q)
{
    return (u64)(((u128)w << 64) / q);
}

static u32 rev_bits(u32 x, int bits)
{
    return bits ? (__builtin_bitreverse32(x) >> (32 - bits)) : 0;
}
} // namespace host

// ============================================================================= context
// Per batch entry (a key switch / rescale of one ciphertext inside a batched launch).
struct WsEntry
{
    u64 *coeff = nullptr; // [L][n]        INTT(target); the rescale's / ModDown's INTT'd last limbs
    u64 *modup = nullptr; // [L+1][L][n]   lifted + NTT'd digits; reused by mod-down/rescale
    u64 *acc = nullptr;   // [2][L+1][n]   key inner products
    u64 *ct3 = nullptr;   // [3][L][n]     tensor output of a batched HMult
};

struct Workspace
{
    int max_limbs = 0;
    int entries = 0;      // batch entries the scratch is sized for (<= MHE_MAXB)
    u64 *base = nullptr;
    WsEntry e[MHE_MAXB];
    u64 *coeff = nullptr; // entry 0's buffers under their old names
    u64 *modup = nullptr;
    u64 *acc = nullptr;
    u64 *tmp = nullptr;   // [L][n]        permuted c1 for Galois
    u64 *ct3 = nullptr;   // [3][L][n]     tensor output for hmult
    // hoisted rotations (hoist.h): the ModUp of up to MHE_MAXB inputs, [K][K-1][n] each, and one
    // zero-coefficient flag per input
    u64 *hoist_base = nullptr;
    int hoist_entries = 0;
    u64 *hoist[MHE_MAXB] = {};
    u64 *hacc[MHE_MAXB * MHE_HOIST_R] = {}; // [2][K][n] key products of each hoisted rotation
    int *flags = nullptr;
    // kernel timing (mhe_ctx_set_timing): event pairs recorded around the two dominant
    // key-switch kernels on this stream, read back by mhe_kernel_time
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[2];
    size_t ev_used[2] = { 0, 0 };
    // device bytes of base / hoist_base: written under mu, read by mhe_scratch_bytes without it
    std::atomic<size_t> bytes{ 0 }, hoist_bytes{ 0 };
    int hoist_limbs = 0;                // the hoisting buffers' level (per-input ModUp of up to this many limbs)
    std::mutex mu;                      // growth of this stream's buffers
};

enum TimedKernel
{
    TK_KS_ROW_MAC = 0, // k_ks_row_mac: fused ModUp row pass + key inner products
    TK_MODUP_COL = 1   // k_modup_col / ModUp column pass
};

// Per-level operation counts (mhe_op_counts, include/mhe.h MHE_OPK_*): what a workload asked of the
// engine, by kind and level -- the op mix a CPU cost model multiplies by per-op CPU timings.
#define MHE_OPK_KINDS 8
#define MHE_OPK_LEVELS 64

struct mhe_ctx
{
    std::atomic<unsigned long long> opc[MHE_OPK_KINDS][MHE_OPK_LEVELS] = {};
    std::atomic<unsigned long long> key_bytes{ 0 }; // key-switching key bytes read since reset (mhe_key_traffic)
    std::atomic<unsigned long long> key_bytes_prep{ 0 }; // the same slices' bytes in the prepared key format
    int device = 0;
    int log_n = 0;
    size_t n = 0;
    int K = 0;
    std::vector<u64> q;
    std::vector<PrimeDev> primes_h;
    PrimeDev *primes = nullptr;
    Tw *tw = nullptr;
    Tw *itw = nullptr;
    Tw *invq = nullptr;
    TwF *twf = nullptr; // FP64 twiddles (w, w/q), [K][n] forward then [K][n] inverse
    NttMode nm;         // FP64 butterflies when every prime is < 2^51 (MHE_FP=0 forces integer)
    // the two ModUp key-switch kernels when only the special prime is >= 2^51 (the GPT-2 chain's
    // 60-bit P): FP64 per output prime below 2^51, integer for P (fp = 2: mixed; MHE_KS_MIX=0: off)
    NttMode nm_ks;
    int ks_fused = 1; // fused row-pass + key-MAC kernel (MHE_KS_FUSED=0: separate row pass + MAC)
    int timing = 0;      // record HIP events around the key-switch kernels (mhe_ctx_set_timing)
    int hmult_fused = 1; // HMult: ModDown fused with the rescale (MHE_HMULT_FUSED=0: separate)
    int ks_share = 1;    // batched key switches sharing one key: XCD-grouped entries (MHE_KS_SHARE=0: off)
    int ks_colgroups = 9; // ModUp column pass: output-prime groups per digit (MHE_KS_COLGROUPS; 0 = one job per (I, J))
    int ks_inv_fused = 1; // the fused MAC runs the special limbs' inverse row pass (MHE_KS_INV_FUSED)
    int ks_pack = 1; // n = 2^16: ModUp intermediate of primes < 2^48 stored in 48 bits (MHE_KS_PACK=0: 64 bits)
    int icol_fused = 1; // ModDown / rescale: inverse column pass fused into the lift column pass (MHE_ICOL_FUSED=0: separate)
    int galois_fused = 1; // apply_galois: one permutation launch, c1 written by the ModDown (MHE_GALOIS_FUSED=0: SEAL's order with a zero fill)
    // read by every thread's rotations, written by mhe_ctx_set_hoist at any time: atomic
    std::atomic<int> ks_hoist{ 1 }; // batched rotations of one input share their ModUp (hoist.h); mhe_ctx_set_hoist / MHE_KS_HOIST=0 turn it off
    std::atomic<int> hoist_check{ 0 }; // recompute every hoisted rotation by the classic path and compare (mhe_ctx_set_hoist)
    std::atomic<int> fail_switch{ 0 }; // mhe_debug_fail_switch: the n-th next batched key switch fails (0: off)
    std::atomic<unsigned long long> hoist_rot{ 0 }, hoist_mac{ 0 }, hoist_bad{ 0 }; // mhe_hoist_stats
    std::atomic<int> fail_alloc{ 0 }; // mhe_debug_fail_alloc: the n-th next allocation fails (0: off)
    TwF *cmodf = nullptr; // [K][K]: (q_j mod q_i, (q_j mod q_i) / q_i) as doubles, j major (hoist.h)
    std::mutex mask_mu;
    std::map<u32, u64 *> masks; // Galois element -> NTT of its negation mask, [K][n] (hoist.h)
    std::mutex mu;
    std::map<hipStream_t, Workspace> ws;
};

// Key limbs a prepared key converts: format 1 (doubles) every prime below 2^51, the FP64 path's;
// format 2 (48-bit planes) every prime below 2^48 (ntt.h KEY_PREP_MIN, KEY_PACK_TAG).
static bool key_limb_packed(const mhe_ctx *c, int limb, int key_limbs, int fmt)
{
    const int pi = (limb == key_limbs - 1) ? c->K - 1 : limb;
    return c->q[pi] < (fmt == 2 ? (1ull << 48) : (1ull << 51));
}

// The prepared format of `key` (0: SEAL's layout, 1 doubles, 2 48-bit planes), from the last word of
// its first slot that either format converts (host sync: only prepare / unprepare and the
// separate-MAC debugging path ask).
static int key_tagged(mhe_ctx *c, const u64 *key, int key_limbs, hipStream_t st, int *tagged)
{
    *tagged = 0;
    for (int fmt = 2; fmt >= 1; fmt--)
        for (int l = 0; l < key_limbs; l++)
            if (key_limb_packed(c, l, key_limbs, fmt))
            {
                u64 w = 0;
                HIP_TRY(hipMemcpyAsync(&w, key + (size_t)l * c->n + c->n - 1, 8, hipMemcpyDeviceToHost, st));
                HIP_TRY(hipStreamSynchronize(st));
                const int f = key_slot_format(w);
                if (f == fmt)
                {
                    *tagged = f;
                    return MHE_OK;
                }
                break; // this format's first slot is not in it
            }
    return MHE_OK;
}

// Events around a launch of kernel kind k on stream st when timing is on.
static hipEvent_t *timing_slot(mhe_ctx *c, Workspace *w, int k, hipStream_t st)
{
    if (!c->timing) return nullptr;
    auto &v = w->ev[k];
    if (w->ev_used[k] == v.size())
    {
        std::pair<hipEvent_t, hipEvent_t> e{};
        if (hipEventCreate(&e.first) != hipSuccess || hipEventCreate(&e.second) != hipSuccess) return nullptr;
        v.push_back(e);
    }
    hipEvent_t *pair = &v[w->ev_used[k]++].first;
    (void)hipEventRecord(pair[0], st);
    return pair;
}

static void timing_end(hipEvent_t *pair, hipStream_t st)
{
    if (pair) (void)hipEventRecord(pair[1], st);
}

// Scratch allocation (hipMalloc) that, when the device reports out of memory, first gives the
// blocks the engine's caching allocator holds back to the device (mhe_internal_release_cached:
// synchronises the device) and retries once.  Freed ciphertext / key buffers stay cached for reuse at
// their own sizes; a plain hipMalloc cannot use them.
static void release_cached_blocks();
// process-wide counts for mhe_alloc_stats: allocations that succeeded only after the cache was
// released, and allocations that failed (including injected ones)
static std::atomic<unsigned long long> g_alloc_retries{ 0 }, g_alloc_failures{ 0 };
static hipError_t scratch_alloc(void **p, size_t bytes)
{
    hipError_t e = hipMalloc(p, bytes);
    if (e == hipSuccess) return e;
    (void)hipGetLastError();
    release_cached_blocks();
    e = hipMalloc(p, bytes);
    if (e != hipSuccess)
    {
        (void)hipGetLastError();
        g_alloc_failures.fetch_add(1);
    }
    else
        g_alloc_retries.fetch_add(1);
    return e;
}

// mhe_debug_fail_alloc's countdown: true for the allocation it designates
static bool injected_alloc_failure(mhe_ctx *c)
{
    int v = c->fail_alloc.load();
    while (v > 0)
        if (c->fail_alloc.compare_exchange_weak(v, v - 1))
        {
            if (v == 1) g_alloc_failures.fetch_add(1);
            return v == 1;
        }
    return false;
}

// The scratch of stream st, for ciphertexts of up to `limbs` limbs and `entries` batch entries.
// The context lock only guards the map; growing one stream's scratch (which drains that stream
// first: its queued kernels may still use the old buffers) holds that workspace's own lock, so
// other threads' streams are not held up by the drain.
static Workspace &ws_of(mhe_ctx *c, hipStream_t st)
{
    std::lock_guard<std::mutex> g(c->mu);
    return c->ws[st];
}

static int get_ws(mhe_ctx *c, hipStream_t st, int limbs, Workspace **out, int entries = 1)
{
    Workspace &w = ws_of(c, st);
    std::lock_guard<std::mutex> g(w.mu);
    if (w.max_limbs < limbs || w.entries < entries)
    {
        if (w.base)
        {
            HIP_TRY(hipStreamSynchronize(st));
            HIP_TRY(hipFree(w.base));
        }
        w.base = nullptr;
        w.bytes = 0;
        const int E = std::max(entries, w.entries);
        const size_t n = c->n, L = std::max(limbs, w.max_limbs);
        const size_t Lc = L < 3 ? 3 : L;
        const size_t per = Lc * n + (L + 1) * L * n + 2 * (L + 1) * n + 3 * L * n;
        size_t words = (size_t)E * per + L * n;
        HIP_TRY(hipSetDevice(c->device));
        if (injected_alloc_failure(c) || scratch_alloc((void **)&w.base, words * sizeof(u64)) != hipSuccess)
        {
            w.base = nullptr;
            w.max_limbs = 0;
            w.entries = 0;
            return fail(MHE_ERR_MEMORY, "workspace allocation failed");
        }
        w.bytes = words * sizeof(u64);
        for (int i = 0; i < E; i++)
        {
            w.e[i].coeff = w.base + (size_t)i * per;
            w.e[i].modup = w.e[i].coeff + Lc * n;
            w.e[i].acc = w.e[i].modup + (L + 1) * L * n;
            w.e[i].ct3 = w.e[i].acc + 2 * (L + 1) * n;
        }
        w.coeff = w.e[0].coeff;
        w.modup = w.e[0].modup;
        w.acc = w.e[0].acc;
        w.tmp = w.base + (size_t)E * per;
        w.ct3 = w.e[0].ct3;
        w.max_limbs = (int)L;
        w.entries = E;
    }
    *out = &w;
    return MHE_OK;
}

// ================================================================================ jobs
// A batch of jobs of one kind: entry e owns job indices [e * per, (e + 1) * per) of the launch and
// its own buffers (pointers inside j[e]); the shared geometry (level, primes) is the same for all.
template <class Job>
struct JobB
{
    Job j[MHE_MAXB];
    int per = 1; // jobs per entry
    __device__ auto view(int y) const
    {
        const int e = y / per;
        return j[e].view(y - e * per);
    }
};
// Plain transform over [poly][limb][n] with limb l on prime l (optionally src != dst).
struct JobPlain
{
    const u64 *src;
    u64 *dst;
    const PrimeDev *primes;
    const Tw *tw;
    int limbs;
    int log_n;
    int mode; // forward row store: 0 = lazy [0,4q), 1 = full; inverse col store: 0 lazy [0,2q), 1 full
    struct View
    {
        const u64 *src;
        u64 *dst;
        PrimeDev p;
        const Tw *tw;
        int mode;
        bool skip;
        __device__ u64 load(u32 x) const { return src[x]; }
        __device__ void store_fwd(u32 x, u64 v) const
        {
            if (mode) v = csub(csub(v, p.two_q), p.q);
            dst[x] = v;
        }
    };
    __device__ View view(int y) const
    {
        const int l = y % limbs;
        const size_t off = (size_t)y << log_n;
        return View{ src + off, dst + off, primes[l], tw + ((size_t)l << log_n), mode, false };
    }
};

// Views must expose store(); wrappers pick the forward / inverse reduction.
struct JobFwdPlain : JobPlain
{
    struct V2 : View
    {
        __device__ void store(u32 x, u64 v) const { store_fwd(x, v); }
    };
    __device__ V2 view(int y) const { return V2{ JobPlain::view(y) }; }
};

struct JobInvPlain : JobPlain
{
    struct V2 : View
    {
        __device__ void store(u32 x, u64 v) const
        {
            if (mode) v = csub(v, p.q);
            dst[x] = v;
        }
    };
    __device__ V2 view(int y) const { return V2{ JobPlain::view(y) }; }
};

// Key-switching ModUp, column pass (evaluator.cpp:2386-2408): job y = I*L + J lifts digit J
// (canonical mod q_J, from INTT(target)) to prime I and starts its NTT; I == L is the special
// prime.  I == J is skipped: the MAC reads the input NTT form (evaluator.cpp:2380-2384).
struct JobModUpCol
{
    const u64 *coeff; // [L][n]
    u64 *modup;       // [chunk][L][n] for output primes I0 .. I0+chunk-1
    const PrimeDev *primes;
    const Tw *tw;
    int L, K, log_n, I0;
    struct View
    {
        const u64 *src;
        u64 *dst;
        PrimeDev p;
        const Tw *tw;
        bool reduce;
        bool skip;
        __device__ u64 load(u32 x) const
        {
            u64 v = src[x];
            return reduce ? barrett64(v, p) : v;
        }
        __device__ void store(u32 x, u64 v) const { dst[x] = v; }
    };
    __device__ View view(int y) const
    {
        const int I = I0 + y / L, J = y % L;
        const int pi = (I == L) ? K - 1 : I;
        View v;
        v.src = coeff + ((size_t)J << log_n);
        v.dst = modup + ((size_t)y << log_n);
        v.p = prime_at(primes, pi);
        v.tw = tw + ((size_t)pi << log_n);
        v.reduce = prime_at(primes, J).q > v.p.q; // key_modulus[J] <= key_modulus[key_index] -> copy
        v.skip = (I == J);
        return v;
    }
};

struct JobModUpRow
{
    u64 *modup;
    const PrimeDev *primes;
    const Tw *tw;
    int L, K, log_n, I0;
    struct View
    {
        u64 *buf;
        PrimeDev p;
        const Tw *tw;
        bool skip;
        __device__ u64 load(u32 x) const { return buf[x]; }
        // canonical output keeps the 128-bit MAC safe for any digit count (< 2^8 terms)
        __device__ void store(u32 x, u64 v) const { buf[x] = csub(csub(v, p.two_q), p.q); }
    };
    __device__ View view(int y) const
    {
        const int I = I0 + y / L, J = y % L;
        const int pi = (I == L) ? K - 1 : I;
        return View{ modup + ((size_t)y << log_n), prime_at(primes, pi), tw + ((size_t)pi << log_n), I == J };
    }
};

// The hoisted ModUp's row pass (hoist.h): src [I][J][n] column-pass output -> dst the same layout,
// canonical, each 256-slot block stored in bit-reversed order.  BREV (n = 2^16, 256-slot rows): the
// row pass reads its LDS row bit-reversed and stores contiguously; otherwise the store scatters
// inside the block (out of place: at n < 2^16 a block spans rows of several workgroups).
template <bool BREV>
struct JobModUpRowH
{
    const u64 *src;
    u64 *dst;
    const PrimeDev *primes;
    const Tw *tw;
    int L, K, log_n;
    struct View
    {
        const u64 *src;
        u64 *dst;
        PrimeDev p;
        const Tw *tw;
        bool skip;
        static constexpr bool brev = BREV;
        __device__ u64 load(u32 x) const { return src[x]; }
        __device__ void store(u32 x, u64 v) const
        {
            dst[BREV ? x : ((x & ~255u) | brev8(x & 255u))] = csub(csub(v, p.two_q), p.q);
        }
    };
    __device__ View view(int y) const
    {
        const int I = y / L, J = y % L;
        const int pi = (I == L) ? K - 1 : I;
        const size_t off = (size_t)y << log_n;
        return View{ src + off, dst + off, prime_at(primes, pi), tw + ((size_t)pi << log_n), I == J };
    }
};

// Key-switching ModDown (evaluator.cpp:2466-2524).  t_last = INTT_lazy(acc[k][L]) in [0,2P);
// column pass job y = k*L + i computes ((barrett(t_last + P/2) mod q_i) + fix_i) and starts
// the NTT mod q_i; the row pass epilogue does ct[k][i] += (acc[k][i] + 4q_i - t) * P^-1.
struct JobModDownCol
{
    const u64 *acc; // [2][L+1][n]
    u64 *scratch;   // [2][L][n]
    const PrimeDev *primes;
    const Tw *tw;
    int L, K, log_n;
    int fixed_i = -1; // >= 0: one job per poly, all on limb fixed_i
    struct View
    {
        const u64 *src;
        u64 *dst;
        PrimeDev p;
        PrimeDev P;
        const Tw *tw;
        u64 half, fix;
        bool reduce;
        bool skip;
        __device__ u64 lift(u64 s) const
        {
            u64 t = barrett64(s + half, P);
            if (reduce) t = barrett64(t, p);
            return t + fix;
        }
        // the integer lift() stands for, from s canonical mod P: s - P when s > P/2, else s
        __device__ double lift_c(u64 s) const { return fp_from_u52(s) - (s > half ? (double)P.q : 0.0); }
        __device__ u64 load(u32 x) const { return lift(src[x]); }
        __device__ void store(u32 x, u64 v) const { dst[x] = v; }
    };
    __device__ View view(int y) const
    {
        const int k = fixed_i >= 0 ? y : y / L, i = fixed_i >= 0 ? fixed_i : y % L;
        View v;
        v.src = acc + ((size_t)(k * (L + 1) + L) << log_n);
        v.dst = scratch + ((size_t)y << log_n);
        v.p = prime_at(primes, i);
        v.P = prime_at(primes, K - 1);
        v.tw = tw + ((size_t)i << log_n);
        v.half = v.P.q >> 1;
        v.fix = v.p.q - barrett64(v.half, v.p);
        v.reduce = v.P.q > v.p.q;
        v.skip = false;
        return v;
    }
};

struct JobModDownRow
{
    u64 *scratch;
    const u64 *acc;
    u64 *ct; // [2][L][n]
    const PrimeDev *primes;
    const Tw *tw;
    const Tw *invq; // [K][K]
    int L, K, log_n;
    int fixed_i = -1; // >= 0: one job per poly, all on limb fixed_i
    int c1_write = 0; // 1: ct[1] = ModDown(acc[1]) instead of += (apply_galois: ct[1] was 0)
    int fp = 0;       // every prime < 2^51: the epilogue in exact FP64 (fparith.h)
    struct View
    {
        u64 *buf;
        const u64 *accp;
        u64 *ctp;
        PrimeDev p;
        const Tw *tw;
        Tw inv;
        bool skip;
        bool replace;
        bool fp;
        double pd, pi, invd;
        __device__ u64 load(u32 x) const { return buf[x]; }
        struct Pre
        {
            u64 a, c;
        };
        __device__ Pre pre(u32 x) const { return Pre{ accp[x], replace ? 0 : ctp[x] }; }
        __device__ void store(u32 x, u64 t, Pre o) const
        {
            if (fp)
            {
                // acc and t canonical: (acc - t) P^-1 in (-1.25p, 1.25p), plus c < p, one
                // canonicalisation (|.| < 2^53): the residue of the integer form
                const double v = fp_mulmod_gen(fp_from_u52(o.a) - fp_from_u52(t), invd, pd, pi);
                ctp[x] = fp_canon(replace ? v : v + fp_from_u52(o.c), pd, pi);
                return;
            }
            u64 v = mul_shoup(o.a + p.four_q - t, inv.x, inv.y, p.q);
            ctp[x] = replace ? v : addmod(v, o.c, p.q); // 0 + v = v: the same word
        }
        __device__ void store(u32 x, u64 t) const { store(x, t, pre(x)); }
    };
    __device__ View view(int y) const
    {
        const int k = fixed_i >= 0 ? y : y / L, i = fixed_i >= 0 ? fixed_i : y % L;
        View v;
        v.buf = scratch + ((size_t)y << log_n);
        v.accp = acc + ((size_t)(k * (L + 1) + i) << log_n);
        v.ctp = ct + ((size_t)(k * L + i) << log_n);
        v.p = prime_at(primes, i);
        v.tw = tw + ((size_t)i << log_n);
        v.inv = tw_at(invq, (size_t)(K - 1) * K + i);
        v.skip = false;
        v.replace = c1_write && k == 1;
        v.fp = fp != 0;
        v.pd = (double)v.p.q;
        v.pi = 1.0 / v.pd;
        v.invd = (double)v.inv.x;
        return v;
    }
};

// Rescale (util/rns.cpp:737-808): last[s] = INTT(in[s][L-1]) canonical; column pass job
// y = s*(L-1) + i: ((last + half mod q_last) mod q_i) + (q_i - half mod q_i); row pass
// epilogue out[s][i] = (in[s][i] + 4q_i - t) * q_last^-1 mod q_i.
struct JobRescaleCol
{
    const u64 *last; // [size][n]
    u64 *scratch;    // [size][L-1][n]
    const PrimeDev *primes;
    const Tw *tw;
    int L, log_n;
    struct View
    {
        const u64 *src;
        u64 *dst;
        PrimeDev p;
        u64 ql, half, neg_half;
        const Tw *tw;
        bool reduce;
        bool skip;
        __device__ u64 lift(u64 s) const // s canonical mod q_last
        {
            u64 v = csub(s + half, ql);
            if (reduce) v = barrett64(v, p);
            return v + neg_half;
        }
        // the integer lift() stands for: s - q_last when s > q_last/2, else s
        __device__ double lift_c(u64 s) const { return fp_from_u52(s) - (s > half ? (double)ql : 0.0); }
        __device__ u64 load(u32 x) const { return lift(src[x]); }
        __device__ void store(u32 x, u64 v) const { dst[x] = v; }
    };
    __device__ View view(int y) const
    {
        const int s = y / (L - 1), i = y % (L - 1);
        View v;
        v.src = last + ((size_t)s << log_n);
        v.dst = scratch + ((size_t)y << log_n);
        v.p = prime_at(primes, i);
        v.ql = prime_at(primes, L - 1).q;
        v.half = v.ql >> 1;
        v.neg_half = v.p.q - barrett64(v.half, v.p);
        v.tw = tw + ((size_t)i << log_n);
        v.reduce = v.p.q < v.ql;
        v.skip = false;
        return v;
    }
};

struct JobRescaleRow
{
    u64 *scratch;
    const u64 *in; // [size][L][n]
    u64 *out;      // [size][L-1][n]
    const PrimeDev *primes;
    const Tw *tw;
    const Tw *invq;
    int L, K, log_n;
    int fp = 0; // every prime < 2^51: the epilogue in exact FP64 (fparith.h)
    struct View
    {
        u64 *buf;
        const u64 *inp;
        u64 *outp;
        PrimeDev p;
        const Tw *tw;
        Tw inv;
        bool skip, fp;
        double pd, pi, invd;
        __device__ u64 load(u32 x) const { return buf[x]; }
        using Pre = u64;
        __device__ Pre pre(u32 x) const { return inp[x]; }
        __device__ void store(u32 x, u64 t, u64 in) const
        {
            if (fp) // in and t canonical: (in - t) q_last^-1 in (-1.25p, 1.25p), canonicalised
                outp[x] = fp_canon(fp_mulmod_gen(fp_from_u52(in) - fp_from_u52(t), invd, pd, pi), pd, pi);
            else
                outp[x] = mul_shoup(in + p.four_q - t, inv.x, inv.y, p.q);
        }
        __device__ void store(u32 x, u64 t) const { store(x, t, pre(x)); }
    };
    __device__ View view(int y) const
    {
        const int s = y / (L - 1), i = y % (L - 1);
        View v;
        v.buf = scratch + ((size_t)y << log_n);
        v.inp = in + ((size_t)(s * L + i) << log_n);
        v.outp = out + ((size_t)(s * (L - 1) + i) << log_n);
        v.p = prime_at(primes, i);
        v.tw = tw + ((size_t)i << log_n);
        v.inv = tw_at(invq, (size_t)(L - 1) * K + i);
        v.skip = false;
        v.fp = fp != 0;
        v.pd = (double)v.p.q;
        v.pi = 1.0 / v.pd;
        v.invd = (double)v.inv.x;
        return v;
    }
};

// ModDown fused with the following rescale (one HMult = multiply + relinearize + rescale).
// With t_i the ModDown lift of INTT(acc_P) and r_i the rescale lift of last = INTT(ct'_{L-1})
// (ct' = ct after ModDown), SEAL computes
//     out_i = ((c_i + (acc_i + 4q - NTT(t_i)) P^-1) + 4q - NTT(r_i)) q_{L-1}^-1   (mod q_i),
// and NTT is linear mod q_i, so the same residues come from ONE forward NTT per limb:
//     out_i = (c_i + acc_i P^-1 - NTT(t_i P^-1 + r_i)) q_{L-1}^-1.
// Column pass job y = k*(L-1) + i builds u_i = t_i P^-1 + r_i (evaluator.cpp:2466-2524 and
// util/rns.cpp:737-808 lifts), the row pass epilogue forms out_i.
struct JobMDRCol
{
    const u64 *acc;  // [2][L+1][n], limb L = INTT_lazy(acc_P) in [0, 2P)
    const u64 *last; // [2][n] = INTT(ct'[k][L-1]), canonical
    u64 *scratch;    // [2][L-1][n]
    const PrimeDev *primes;
    const Tw *tw;
    const Tw *invq; // [K][K]
    int L, K, log_n;
    int fp = 0; // every prime < 2^51 (NttMode::fp): the lift in exact FP64 (fparith.h)
    struct View
    {
        const u64 *accP, *lastp;
        u64 *dst;
        PrimeDev p, P;
        const Tw *tw;
        Tw pinv;
        u64 halfP, fixP, ql, halfL, neg_halfL;
        bool redP, redL, skip, fp;
        double pd, pi, pinvd;
        __device__ u64 load(u32 x) const
        {
            if (fp)
            {
                // accP in [0, 2P) -> a mod P canonical by two conditional subtractions; t + fixP
                // and the rescale lift r + neg_halfL are exact doubles (< 2^52), the product by
                // P^-1 is in (-2p, 2p), the sum below 2^53: one canonicalisation, the same residue
                const u64 t = csub(csub(accP[x] + halfP, 2 * P.q), P.q);
                const u64 r = csub(lastp[x] + halfL, ql);
                const double u = fp_mulmod_gen(fp_from_u52(t + fixP), pinvd, pd, pi) + fp_from_u52(r + neg_halfL);
                return fp_canon(u, pd, pi);
            }
            u64 t = barrett64(accP[x] + halfP, P);
            if (redP) t = barrett64(t, p);
            t += fixP;                                  // ModDown lift, [0, 2q)
            u64 r = csub(lastp[x] + halfL, ql);
            if (redL) r = barrett64(r, p);
            r += neg_halfL;                             // rescale lift, [0, 2q)
            const u64 u = mul_shoup(t, pinv.x, pinv.y, p.q) + r; // [0, 3q)
            return csub(csub(u, p.two_q), p.q);
        }
        __device__ void store(u32 x, u64 v) const { dst[x] = v; }
        // k_col_lift2 (FP): the two lifts' centred integers, the same for every output prime -- the
        // special accumulator limb (in [0, 2P)) and the rescale's last limb (canonical mod q_last)
        __device__ void src_c(u32 x, double &ct, double &cr) const
        {
            const u64 a = csub(accP[x], P.q), l = lastp[x];
            ct = fp_from_u52(a) - (a > halfP ? (double)P.q : 0.0);
            cr = fp_from_u52(l) - (l > halfL ? (double)ql : 0.0);
        }
        // t P^-1 + r mod p from them: |.| < 1.25p + 2^50, congruent to load()'s value
        __device__ double lift_f(double ct, double cr) const { return fp_mulmod_gen(ct, pinvd, pd, pi) + cr; }
    };
    __device__ View view(int y) const
    {
        const int k = y / (L - 1), i = y % (L - 1);
        View v;
        v.accP = acc + ((size_t)(k * (L + 1) + L) << log_n);
        v.lastp = last + ((size_t)k << log_n);
        v.dst = scratch + ((size_t)y << log_n);
        v.p = prime_at(primes, i);
        v.P = prime_at(primes, K - 1);
        v.tw = tw + ((size_t)i << log_n);
        v.pinv = tw_at(invq, (size_t)(K - 1) * K + i);
        v.halfP = v.P.q >> 1;
        v.fixP = v.p.q - barrett64(v.halfP, v.p);
        v.redP = v.P.q > v.p.q;
        v.ql = prime_at(primes, L - 1).q;
        v.halfL = v.ql >> 1;
        v.neg_halfL = v.p.q - barrett64(v.halfL, v.p);
        v.redL = v.p.q < v.ql;
        v.skip = false;
        v.fp = fp != 0;
        v.pd = (double)v.p.q;
        v.pi = 1.0 / v.pd;
        v.pinvd = (double)v.pinv.x;
        return v;
    }
};

struct JobMDRRow
{
    u64 *scratch;
    const u64 *acc; // [2][L+1][n]
    const u64 *ct;  // [2][L][n], limbs < L-1 before ModDown
    u64 *out;       // [2][L-1][n]
    const PrimeDev *primes;
    const Tw *tw;
    const Tw *invq;
    int L, K, log_n;
    int fp = 0; // every prime < 2^51: the epilogue in exact FP64 (fparith.h)
    struct View
    {
        u64 *buf;
        const u64 *accp, *ctp;
        u64 *outp;
        PrimeDev p;
        const Tw *tw;
        Tw pinv, qlinv;
        bool skip, fp;
        double pd, pi, pinvd, qlinvd;
        __device__ u64 load(u32 x) const { return buf[x]; }
        struct Pre
        {
            u64 a, c;
        };
        __device__ Pre pre(u32 x) const { return Pre{ accp[x], ctp[x] }; }
        __device__ void store(u32 x, u64 U, Pre o) const
        {
            if (fp)
            {
                // acc_i P^-1 in (-1.25p, 1.25p); c + a - U is an exact integer below 2^53; its
                // centered residue times q_{L-1}^-1, canonicalised: the residue of the integer form
                const double a = fp_mulmod_gen(fp_from_u52(o.a), pinvd, pd, pi);
                const double v = fp_reduce(fp_from_u52(o.c) + a - fp_from_u52(U), pd, pi);
                outp[x] = fp_canon(fp_mulmod_gen(v, qlinvd, pd, pi), pd, pi);
                return;
            }
            const u64 a = mul_shoup(o.a, pinv.x, pinv.y, p.q); // acc_i P^-1
            const u64 v = o.c + a + p.four_q - U;              // < 6q
            outp[x] = mul_shoup(v, qlinv.x, qlinv.y, p.q);
        }
        __device__ void store(u32 x, u64 U) const { store(x, U, pre(x)); }
    };
    __device__ View view(int y) const
    {
        const int k = y / (L - 1), i = y % (L - 1);
        View v;
        v.buf = scratch + ((size_t)y << log_n);
        v.accp = acc + ((size_t)(k * (L + 1) + i) << log_n);
        v.ctp = ct + ((size_t)(k * L + i) << log_n);
        v.outp = out + ((size_t)(k * (L - 1) + i) << log_n);
        v.p = prime_at(primes, i);
        v.tw = tw + ((size_t)i << log_n);
        v.pinv = tw_at(invq, (size_t)(K - 1) * K + i);
        v.qlinv = tw_at(invq, (size_t)(L - 1) * K + i);
        v.skip = false;
        v.fp = fp != 0;
        v.pd = (double)v.p.q;
        v.pi = 1.0 / v.pd;
        v.pinvd = (double)v.pinv.x;
        v.qlinvd = (double)v.qlinv.x;
        return v;
    }
};

// Rescale INTT of the last limb: src limb (L-1) of poly s -> last[s], canonical.
struct JobLastInv
{
    const u64 *in;
    u64 *last;
    const PrimeDev *primes;
    const Tw *itw;
    int L, log_n;
    int lazy;
    struct View
    {
        const u64 *src;
        u64 *dst;
        PrimeDev p;
        const Tw *tw;
        int lazy;
        bool skip;
        __device__ u64 load(u32 x) const { return src[x]; }
        __device__ void store(u32 x, u64 v) const { dst[x] = lazy ? v : csub(v, p.q); }
    };
    __device__ View view(int y) const
    {
        View v;
        v.src = in + ((size_t)(y * L + (L - 1)) << log_n);
        v.dst = last + ((size_t)y << log_n);
        v.p = prime_at(primes, L - 1);
        v.tw = itw + ((size_t)(L - 1) << log_n);
        v.lazy = lazy;
        v.skip = false;
        return v;
    }
};

// Generic job on explicit (src, dst, prime) with a per-job stride: used for the key-switch
// INTT of the target (limb J on prime J) and of the special accumulator limbs.
struct JobStrided
{
    const u64 *src;
    u64 *dst;
    size_t src_stride, dst_stride; // in words, per job
    int prime0;                    // prime index of job 0
    int prime_step;                // 0: all jobs on prime0; 1: job y on prime0 + y
    const PrimeDev *primes;
    const Tw *tw;
    int log_n;
    int mode; // inverse store: 0 lazy, 1 full
    const int *run_if = nullptr; // non-null: every job returns unless *run_if != 0 (hoist.h fallback)
    struct View
    {
        const u64 *src;
        u64 *dst;
        PrimeDev p;
        const Tw *tw;
        int mode;
        bool skip;
        __device__ u64 load(u32 x) const { return src[x]; }
        __device__ void store(u32 x, u64 v) const { dst[x] = mode ? csub(v, p.q) : v; }
    };
    __device__ View view(int y) const
    {
        const int pi = prime0 + prime_step * y;
        return View{ src + y * src_stride, dst + y * dst_stride, primes[pi], tw + ((size_t)pi << log_n), mode,
                     run_if && !*run_if };
    }
};

// ============================================================================ kernels
// Elementwise kernels process 2 residues per lane (16-B loads); n is a multiple of 512.
#define ELEM_GRID(total2) dim3((unsigned)(((total2) + 255) / 256))

// Elementwise products in FP64 (csrc/fparith.h) for primes below 2^51, where the integer path's
// 64 x 64 -> 128-bit product and Barrett reduction cost several half- and quarter-rate instructions:
// canonical residues are exact doubles, fp_mulmod_gen leaves a*b mod q in (-1.25q, 1.25q) and
// fp_canon returns the canonical residue, so the words are the integer path's.  fp: the context's
// FP64 mode (MHE_FP=0 keeps every product on the integer path).
__device__ __forceinline__ bool elem_fp(int fp, const PrimeDev &p)
{
    return fp && p.q < (1ull << 51);
}
__device__ __forceinline__ double mulmod_fd(u64 a, u64 b, const PrimeDev &p) // (-1.25q, 1.25q)
{
    return fp_mulmod_gen(fp_from_u52(a), fp_from_u52(b), p.qd, p.qi);
}
__device__ __forceinline__ u64 mulmod_e(u64 a, u64 b, const PrimeDev &p, bool f)
{
    return f ? fp_canon(mulmod_fd(a, b, p), p.qd, p.qi) : mulmod(a, b, p);
}

__device__ __forceinline__ void addsub_at(const u64 *a, const u64 *b, u64 *out, const PrimeDev *primes, int limbs,
                                          int log_n, size_t i2, int op)
{
    const size_t i = i2 * 2;
    const int l = (int)((i >> log_n) % limbs);
    const u64 q = primes[l].q;
    ulonglong2 x = *(const ulonglong2 *)(a + i);
    ulonglong2 r;
    if (op == 0)
    {
        ulonglong2 y = *(const ulonglong2 *)(b + i);
        r.x = addmod(x.x, y.x, q);
        r.y = addmod(x.y, y.y, q);
    }
    else if (op == 1)
    {
        ulonglong2 y = *(const ulonglong2 *)(b + i);
        r.x = submod(x.x, y.x, q);
        r.y = submod(x.y, y.y, q);
    }
    else
    {
        r.x = x.x ? q - x.x : 0;
        r.y = x.y ? q - x.y : 0;
    }
    *(ulonglong2 *)(out + i) = r;
}

__global__ void k_addsub(const u64 *a, const u64 *b, u64 *out, const PrimeDev *primes, int limbs, int log_n,
                         size_t total2, int op)
{
    size_t i2 = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i2 < total2) addsub_at(a, b, out, primes, limbs, log_n, i2, op);
}

// dyadic product with b broadcast over polys (multiply_plain_ntt)
__device__ __forceinline__ void mulplain_at(const u64 *a, const u64 *b, u64 *out, const PrimeDev *primes, int limbs,
                                            int log_n, size_t i2, int fp)
{
    const size_t i = i2 * 2;
    const size_t limb_words = (size_t)limbs << log_n;
    const int l = (int)((i >> log_n) % limbs);
    const PrimeDev p = primes[l];
    const bool f = elem_fp(fp, p); // uniform: a wave's residues are of one limb
    ulonglong2 x = *(const ulonglong2 *)(a + i);
    ulonglong2 y = *(const ulonglong2 *)(b + i % limb_words);
    ulonglong2 r;
    r.x = mulmod_e(x.x, y.x, p, f);
    r.y = mulmod_e(x.y, y.y, p, f);
    *(ulonglong2 *)(out + i) = r;
}

__global__ void k_mulplain(const u64 *a, const u64 *b, u64 *out, const PrimeDev *primes, int limbs, int log_n,
                           size_t total2, int fp)
{
    size_t i2 = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i2 < total2) mulplain_at(a, b, out, primes, limbs, log_n, i2, fp);
}

// acc += a * b, b broadcast over polys (multiply_plain_ntt then add_inplace, one pass)
__device__ __forceinline__ void mulplain_add_at(const u64 *a, const u64 *b, u64 *acc, const PrimeDev *primes,
                                                int limbs, int log_n, size_t i2, int fp)
{
    const size_t i = i2 * 2;
    const size_t limb_words = (size_t)limbs << log_n;
    const int l = (int)((i >> log_n) % limbs);
    const PrimeDev p = primes[l];
    ulonglong2 x = *(const ulonglong2 *)(a + i);
    ulonglong2 y = *(const ulonglong2 *)(b + i % limb_words);
    ulonglong2 z = *(const ulonglong2 *)(acc + i);
    ulonglong2 r;
    if (elem_fp(fp, p))
    {
        // canonical acc (< q) + a product in (-1.25q, 1.25q): |.| < 2.25q, exact
        r.x = fp_canon(fp_from_u52(z.x) + mulmod_fd(x.x, y.x, p), p.qd, p.qi);
        r.y = fp_canon(fp_from_u52(z.y) + mulmod_fd(x.y, y.y, p), p.qd, p.qi);
    }
    else
    {
        r.x = addmod(z.x, mulmod(x.x, y.x, p), p.q);
        r.y = addmod(z.y, mulmod(x.y, y.y, p), p.q);
    }
    *(ulonglong2 *)(acc + i) = r;
}

__global__ void k_mulplain_add(const u64 *a, const u64 *b, u64 *acc, const PrimeDev *primes, int limbs, int log_n,
                               size_t total2, int fp)
{
    size_t i2 = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i2 < total2) mulplain_add_at(a, b, acc, primes, limbs, log_n, i2, fp);
}

// acc = (accumulate ? acc : 0) + sum_k a_k * b_k, up to 16 terms per launch (pointers in the kernel
// arguments); each thread's 2 * cnt loads are independent, so they are all in flight together
#define MHE_SUM_TERMS 16
struct SumPtrs
{
    const u64 *a[MHE_SUM_TERMS];
    const u64 *b[MHE_SUM_TERMS];
};
__global__ void k_mulplain_sum(SumPtrs P, int cnt, u64 *acc, int accumulate, const PrimeDev *primes, int limbs,
                               int log_n, size_t total2, int fp)
{
    size_t i2 = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i2 >= total2) return;
    const size_t i = i2 * 2;
    const size_t limb_words = (size_t)limbs << log_n;
    const int l = (int)((i >> log_n) % limbs);
    const PrimeDev p = primes[l];
    ulonglong2 z = accumulate ? *(const ulonglong2 *)(acc + i) : ulonglong2{ 0, 0 };
    if (elem_fp(fp, p))
    {
        // FP64 sums: products in (-1.25q, 1.25q), centred by fp_reduce after every second one, so
        // |sum| < q/2 + 1 + 2.5q < 2^53 throughout; one fp_canon at the end
        double sx = fp_from_u52(z.x), sy = fp_from_u52(z.y);
        for (int k = 0; k < cnt; k++)
        {
            const ulonglong2 x = *(const ulonglong2 *)(P.a[k] + i);
            const ulonglong2 y = *(const ulonglong2 *)(P.b[k] + i % limb_words);
            sx += mulmod_fd(x.x, y.x, p);
            sy += mulmod_fd(x.y, y.y, p);
            if (k & 1)
            {
                sx = fp_reduce(sx, p.qd, p.qi);
                sy = fp_reduce(sy, p.qd, p.qi);
            }
        }
        z.x = fp_canon(sx, p.qd, p.qi);
        z.y = fp_canon(sy, p.qd, p.qi);
    }
    else
    {
        for (int k = 0; k < cnt; k++)
        {
            const ulonglong2 x = *(const ulonglong2 *)(P.a[k] + i);
            const ulonglong2 y = *(const ulonglong2 *)(P.b[k] + i % limb_words);
            z.x = addmod(z.x, mulmod(x.x, y.x, p), p.q);
            z.y = addmod(z.y, mulmod(x.y, y.y, p), p.q);
        }
    }
    *(ulonglong2 *)(acc + i) = z;
}

struct ScalarTab
{
    u64 v[64];
    u64 vq[64];
};

__device__ __forceinline__ void scalar_at(const u64 *a, u64 *out, const PrimeDev *primes, const ScalarTab &s, int limbs,
                                          int log_n, size_t i2, int op)
{
    const size_t i = i2 * 2;
    const int l = (int)((i >> log_n) % limbs);
    const u64 q = primes[l].q;
    ulonglong2 r;
    if (op == 2)
    {
        r.x = r.y = s.v[l];
        *(ulonglong2 *)(out + i) = r;
        return;
    }
    ulonglong2 x = *(const ulonglong2 *)(a + i);
    if (op == 0)
    {
        r.x = mul_shoup(x.x, s.v[l], s.vq[l], q);
        r.y = mul_shoup(x.y, s.v[l], s.vq[l], q);
    }
    else
    {
        r.x = addmod(x.x, s.v[l], q);
        r.y = addmod(x.y, s.v[l], q);
    }
    *(ulonglong2 *)(out + i) = r;
}

__global__ void k_scalar(const u64 *a, u64 *out, const PrimeDev *primes, ScalarTab s, int limbs, int log_n,
                         size_t total2, int op)
{
    size_t i2 = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i2 < total2) scalar_at(a, out, primes, s, limbs, log_n, i2, op);
}

// ckks_multiply tile loop (evaluator.cpp:714-773) / ckks_square (:1000-1059), fused.
__device__ __forceinline__ void tensor_at(const u64 *a, const u64 *b, u64 *out, const PrimeDev *primes, int limbs,
                                          int log_n, size_t i2, int square, int fp)
{
    const size_t i = i2 * 2;
    const size_t ps = (size_t)limbs << log_n;
    const int l = (int)(i >> log_n);
    const PrimeDev p = primes[l];
    ulonglong2 x0 = *(const ulonglong2 *)(a + i), x1 = *(const ulonglong2 *)(a + ps + i);
    ulonglong2 r0, r1, r2;
    if (elem_fp(fp, p))
    {
        // FP64: each product in (-1.25q, 1.25q), the cross term's two in (-2.5q, 2.5q), exact
        const ulonglong2 y0 = square ? x0 : *(const ulonglong2 *)(b + i), y1 = square ? x1 : *(const ulonglong2 *)(b + ps + i);
        const double qd = p.qd, qi = p.qi;
        r0.x = fp_canon(mulmod_fd(x0.x, y0.x, p), qd, qi);
        r0.y = fp_canon(mulmod_fd(x0.y, y0.y, p), qd, qi);
        r1.x = fp_canon(mulmod_fd(x0.x, y1.x, p) + mulmod_fd(x1.x, y0.x, p), qd, qi);
        r1.y = fp_canon(mulmod_fd(x0.y, y1.y, p) + mulmod_fd(x1.y, y0.y, p), qd, qi);
        r2.x = fp_canon(mulmod_fd(x1.x, y1.x, p), qd, qi);
        r2.y = fp_canon(mulmod_fd(x1.y, y1.y, p), qd, qi);
    }
    else if (square)
    {
        r0.x = mulmod(x0.x, x0.x, p);
        r0.y = mulmod(x0.y, x0.y, p);
        u64 t = mulmod(x0.x, x1.x, p), u = mulmod(x0.y, x1.y, p);
        r1.x = addmod(t, t, p.q);
        r1.y = addmod(u, u, p.q);
        r2.x = mulmod(x1.x, x1.x, p);
        r2.y = mulmod(x1.y, x1.y, p);
    }
    else
    {
        ulonglong2 y0 = *(const ulonglong2 *)(b + i), y1 = *(const ulonglong2 *)(b + ps + i);
        r0.x = mulmod(x0.x, y0.x, p);
        r0.y = mulmod(x0.y, y0.y, p);
        r1.x = addmod(mulmod(x0.x, y1.x, p), mulmod(x1.x, y0.x, p), p.q);
        r1.y = addmod(mulmod(x0.y, y1.y, p), mulmod(x1.y, y0.y, p), p.q);
        r2.x = mulmod(x1.x, y1.x, p);
        r2.y = mulmod(x1.y, y1.y, p);
    }
    *(ulonglong2 *)(out + i) = r0;
    *(ulonglong2 *)(out + ps + i) = r1;
    *(ulonglong2 *)(out + 2 * ps + i) = r2;
}

__global__ void k_tensor(const u64 *a, const u64 *b, u64 *out, const PrimeDev *primes, int limbs, int log_n,
                         size_t total2, int square, int fp)
{
    size_t i2 = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i2 < total2) tensor_at(a, b, out, primes, limbs, log_n, i2, square, fp);
}

// The same elementwise kernels over up to MHE_MAXB entries of one shape (entry = blockIdx.y): the
// launches that mhe_launch_run coalesces, e.g. the same-numbered adds of the images of a
// seal::FiberBatch
struct ElemPtrs
{
    const u64 *a[MHE_MAXB];
    const u64 *b[MHE_MAXB];
    u64 *out[MHE_MAXB];
};

__global__ void k_elem_b(ElemPtrs P, const PrimeDev *primes, ScalarTab st, int limbs, int log_n, size_t total2,
                         int kind, int op, int fp)
{
    const size_t i2 = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i2 >= total2) return;
    const int e = blockIdx.y;
    switch (kind)
    {
    case MHE_LK_ADDSUB: addsub_at(P.a[e], P.b[e], P.out[e], primes, limbs, log_n, i2, op); break;
    case MHE_LK_MULPLAIN: mulplain_at(P.a[e], P.b[e], P.out[e], primes, limbs, log_n, i2, fp); break;
    case MHE_LK_MULPLAIN_ADD: mulplain_add_at(P.a[e], P.b[e], P.out[e], primes, limbs, log_n, i2, fp); break;
    case MHE_LK_SCALAR: scalar_at(P.a[e], P.out[e], primes, st, limbs, log_n, i2, op); break;
    case MHE_LK_TENSOR: tensor_at(P.a[e], P.b[e], P.out[e], primes, limbs, log_n, i2, op, fp); break;
    }
}

__global__ void k_copy16_b(ElemPtrs P, size_t count)
{
    const int e = blockIdx.y;
    uint4 *dst = reinterpret_cast<uint4 *>(P.out[e]);
    const uint4 *src = reinterpret_cast<const uint4 *>(P.a[e]);
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < count; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}

// Key-switching inner product (evaluator.cpp:2410-2463): for output prime I (I == L -> P),
// acc[k][I] = sum_J d_J[I] * key[J][k][I] mod q_I, where d_J[I] is the lifted NTT digit
// (modup[I][J]) or, for I == J, the input target limb itself.  128-bit accumulation with a
// single final Barrett reduction (digits are canonical so < 2^8 terms never overflow).
__global__ __launch_bounds__(256) void k_ks_mac(const u64 *modup, const u64 *target, const u64 *key, u64 *acc,
                                                const PrimeDev *primes, int L, int K, int key_limbs, int log_n, int I0)
{
    const u32 i = (blockIdx.x * 256 + threadIdx.x) * 2;
    const int I = I0 + blockIdx.y;
    const int pi = (I == L) ? K - 1 : I;
    const int ki = (I == L) ? key_limbs - 1 : I;
    const size_t n = (size_t)1 << log_n;
    const PrimeDev p = primes[pi];
    Acc128 a0x{ 0, 0 }, a0y{ 0, 0 }, a1x{ 0, 0 }, a1y{ 0, 0 };
    const size_t kstride = (size_t)key_limbs * n;
    for (int J = 0; J < L; J++)
    {
        const u64 *d = (I == J) ? target + (size_t)J * n : modup + ((size_t)(I - I0) * L + J) * n;
        ulonglong2 x = *(const ulonglong2 *)(d + i);
        const u64 *k0 = key + (size_t)(2 * J) * kstride + (size_t)ki * n;
        ulonglong2 y0 = *(const ulonglong2 *)(k0 + i);
        ulonglong2 y1 = *(const ulonglong2 *)(k0 + kstride + i);
        mac128(a0x, x.x, y0.x);
        mac128(a0y, x.y, y0.y);
        mac128(a1x, x.x, y1.x);
        mac128(a1y, x.y, y1.y);
    }
    ulonglong2 r0, r1;
    r0.x = barrett128(a0x.lo, a0x.hi, p);
    r0.y = barrett128(a0y.lo, a0y.hi, p);
    r1.x = barrett128(a1x.lo, a1x.hi, p);
    r1.y = barrett128(a1y.lo, a1y.hi, p);
    *(ulonglong2 *)(acc + (size_t)I * n + i) = r0;
    *(ulonglong2 *)(acc + (size_t)(L + 1 + I) * n + i) = r1;
}

// GaloisTool::apply_galois_ntt (util/galois.cpp:192-218) with the permutation of
// generate_table_ntt (util/galois.cpp:18-51) computed on the fly: out[i] = in[tab(i)].
__global__ void k_galois(const u64 *in, u64 *out, u32 elt, int log_n, size_t total)
{
    size_t g = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= total) return;
    const u32 n = 1u << log_n;
    const u32 i = (u32)(g & (n - 1));
    const size_t base = g - i;
    const u32 reversed = __builtin_bitreverse32(n + i) >> (31 - log_n); // rev over log_n+1 bits
    const u32 idx = (u32)(((u64)elt * reversed) >> 1) & (n - 1);
    const u32 src = __builtin_bitreverse32(idx) >> (32 - log_n);
    out[g] = in[base + src];
}

// The same for up to MHE_MAXB independent (in, out, element) entries, entry = blockIdx.y.
struct GalPtrs
{
    const u64 *in[MHE_MAXB];
    u64 *out[MHE_MAXB];
    u32 elt[MHE_MAXB];
};

__global__ void k_galois_b(GalPtrs P, int log_n, size_t total)
{
    size_t g = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= total) return;
    const u64 *in = P.in[blockIdx.y];
    u64 *out = P.out[blockIdx.y];
    const u32 elt = P.elt[blockIdx.y];
    const u32 n = 1u << log_n;
    const u32 i = (u32)(g & (n - 1));
    const size_t base = g - i;
    const u32 reversed = __builtin_bitreverse32(n + i) >> (31 - log_n);
    const u32 idx = (u32)(((u64)elt * reversed) >> 1) & (n - 1);
    const u32 src = __builtin_bitreverse32(idx) >> (32 - log_n);
    out[g] = in[base + src];
}

// Bootstrapper::modraise_inplace (ckks_bootstrapping/Bootstrapper.cpp:2894-2948): the single-limb
// coefficient-form polynomial x (mod q_0, canonical) is lifted centered, v = x - q_0 if
// x > q_0/2, and reduced mod every prime of the target level.
__global__ void k_modraise(const u64 *in, u64 *out, const PrimeDev *primes, int limbs, int log_n, size_t total)
{
    size_t g = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= total) return;
    const size_t n = (size_t)1 << log_n;
    const size_t per_poly = (size_t)limbs << log_n;
    const size_t p = g / per_poly, r = g - p * per_poly;
    const int j = (int)(r >> log_n);
    const size_t i = r & (n - 1);
    const u64 x = in[p * n + i];
    const u64 q0 = primes[0].q, q = primes[j].q;
    u64 v = x % q;
    if (x > (q0 >> 1))
    {
        const u64 mq0 = q - q0 % q; // -q_0 mod q (q for j = 0 reduces to 0 below)
        v += mq0;
        v -= (v >= q) ? q : 0;
    }
    out[g] = v;
}

// ============================================================== caching device allocator
// Stream-ordered allocation for the engine's transient buffers (every Ciphertext temporary of the
// SEAL surface).  The runtime's stream-ordered pool (hipMallocAsync/hipFreeAsync) was observed on
// this image to hand out memory that was still live: bootstrapping's cached plaintexts and guard
// regions were overwritten even with kernels serialised, and disappeared with plain hipMalloc.
// So the engine keeps its own cache: a freed block records an event on the freeing stream and goes
// to a free list by size; an allocation reuses a block of the same rounded size (waiting on its
// event when it comes from another stream) or calls hipMalloc.  Memory is returned to the device
// only when hipMalloc fails (then every cached block is released and the call retried).
namespace
{
struct CachedBlock
{
    void *p;
    size_t size;
    hipStream_t st;
    hipEvent_t ev;
};
struct DevAlloc
{
    std::mutex mu;
    std::map<void *, size_t> live;
    std::multimap<size_t, CachedBlock> free_blocks;
    std::vector<hipEvent_t> ev_pool;
    size_t cached = 0, in_use = 0;
    int contexts = 0; // live engine contexts on this device: the cache is returned when the last goes
};
DevAlloc &dev_alloc()
{
    static DevAlloc a[64];
    int d = 0;
    (void)hipGetDevice(&d);
    return a[d & 63];
}
size_t round_size(size_t b)
{
    if (b == 0) b = 1;
    if (b < ((size_t)1 << 20)) return (b + 4095) & ~(size_t)4095;
    return (b + ((size_t)1 << 20) - 1) & ~(((size_t)1 << 20) - 1);
}
void release_cached(DevAlloc &a)
{
    // caller holds a.mu
    (void)hipDeviceSynchronize();
    for (auto &kv : a.free_blocks)
    {
        (void)hipFree(kv.second.p);
        a.ev_pool.push_back(kv.second.ev);
    }
    a.free_blocks.clear();
    a.cached = 0;
}
} // namespace

static void release_cached_blocks()
{
    DevAlloc &a = dev_alloc();
    std::lock_guard<std::mutex> g(a.mu);
    release_cached(a);
}

// context lifetime on the current device (mhe_ctx_create / mhe_ctx_destroy): when the last context
// of a device goes, its cached blocks go back to the device, so another process (or a later
// engine) on the same GPU gets that memory
extern "C" __attribute__((visibility("hidden"))) void mhe_internal_ctx_count(int delta)
{
    DevAlloc &a = dev_alloc();
    std::lock_guard<std::mutex> g(a.mu);
    a.contexts += delta;
    if (a.contexts <= 0)
    {
        a.contexts = 0;
        release_cached(a);
    }
}

extern "C" __attribute__((visibility("hidden"))) hipError_t mhe_internal_alloc(void **p, size_t bytes, hipStream_t st)
{
    DevAlloc &a = dev_alloc();
    const size_t sz = round_size(bytes);
    std::lock_guard<std::mutex> g(a.mu);
    auto it = a.free_blocks.lower_bound(sz);
    auto best = a.free_blocks.end();
    for (auto j = it; j != a.free_blocks.end() && j->first <= sz + sz / 4; ++j)
        if (best == a.free_blocks.end() || j->second.st == st)
        {
            best = j;
            if (j->second.st == st) break;
        }
    if (best != a.free_blocks.end())
    {
        CachedBlock b = best->second;
        a.free_blocks.erase(best);
        a.cached -= b.size;
        if (b.st != st)
        {
            hipError_t e = hipStreamWaitEvent(st, b.ev, 0);
            if (e != hipSuccess) return e;
        }
        a.ev_pool.push_back(b.ev);
        a.live[b.p] = b.size;
        a.in_use += b.size;
        *p = b.p;
        return hipSuccess;
    }
    hipError_t e = hipMalloc(p, sz);
    if (e != hipSuccess)
    {
        (void)hipGetLastError();
        release_cached(a);
        e = hipMalloc(p, sz);
        if (e != hipSuccess)
        {
            g_alloc_failures.fetch_add(1);
            return e;
        }
        g_alloc_retries.fetch_add(1);
    }
    a.live[*p] = sz;
    a.in_use += sz;
    return hipSuccess;
}

extern "C" __attribute__((visibility("hidden"))) hipError_t mhe_internal_free(void *p, hipStream_t st)
{
    if (!p) return hipSuccess;
    DevAlloc &a = dev_alloc();
    std::lock_guard<std::mutex> g(a.mu);
    auto it = a.live.find(p);
    if (it == a.live.end()) return hipErrorInvalidValue;
    const size_t sz = it->second;
    a.live.erase(it);
    a.in_use -= sz;
    hipEvent_t ev = nullptr;
    if (!a.ev_pool.empty())
    {
        ev = a.ev_pool.back();
        a.ev_pool.pop_back();
    }
    else
    {
        hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    hipError_t e = hipEventRecord(ev, st);
    if (e != hipSuccess) return e;
    a.free_blocks.emplace(sz, CachedBlock{ p, sz, st, ev });
    a.cached += sz;
    return hipSuccess;
}

// Device-to-device copies run as a kernel on the caller's stream (ordered with the stream's other
// kernels by construction, at HBM speed) rather than hipMemcpyAsync's copy engines.
__global__ void k_copy16(uint4 *__restrict__ dst, const uint4 *__restrict__ src, size_t count)
{
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < count; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}

__global__ void k_copy8(u64 *__restrict__ dst, const u64 *__restrict__ src, size_t count)
{
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < count; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}

extern "C" __attribute__((visibility("hidden"))) hipError_t mhe_internal_copy_d2d(void *dst, const void *src,
                                                                                  size_t bytes, hipStream_t st)
{
    if (!bytes || dst == src) return hipSuccess;
    const uintptr_t a = (uintptr_t)dst | (uintptr_t)src;
    if ((a & 15) == 0 && (bytes & 15) == 0)
    {
        const size_t cnt = bytes / 16;
        const unsigned grid = (unsigned)std::min<size_t>((cnt + 255) / 256, 4096);
        hipLaunchKernelGGL(k_copy16, dim3(grid), dim3(256), 0, st, (uint4 *)dst, (const uint4 *)src, cnt);
        return hipGetLastError();
    }
    if ((a & 7) == 0 && (bytes & 7) == 0)
    {
        const size_t cnt = bytes / 8;
        const unsigned grid = (unsigned)std::min<size_t>((cnt + 255) / 256, 4096);
        hipLaunchKernelGGL(k_copy8, dim3(grid), dim3(256), 0, st, (u64 *)dst, (const u64 *)src, cnt);
        return hipGetLastError();
    }
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st);
}

// ======================================================================= dispatch helpers
static bool valid_ctx(mhe_ctx *c)
{
    return c && c->primes;
}

static hipStream_t S(void *s)
{
    return (hipStream_t)s;
}

static int check_limbs(mhe_ctx *c, int limbs, int lo)
{
    if (!valid_ctx(c)) return fail(MHE_ERR_ARG, "context is not valid");
    if (limbs < lo || limbs > c->K - 1) return fail(MHE_ERR_ARG, "encrypted is not valid for encryption parameters");
    return MHE_OK;
}

// Do the word ranges [a, a + aw) and [b, b + bw) share a word?  The batched entry points run every
// entry inside the same kernels, so an output that overlaps another entry's operand would be read
// and written by one launch in an order that depends on the grid (not the order of count calls).
static bool ranges_overlap(const u64 *a, size_t aw, const u64 *b, size_t bw)
{
    return a < b + bw && b < a + aw;
}

static void count_op(mhe_ctx *c, int kind, int L, unsigned long long k)
{
    if (kind >= 0 && kind < MHE_OPK_KINDS && L >= 0 && L < MHE_OPK_LEVELS) c->opc[kind][L].fetch_add(k, std::memory_order_relaxed);
}

// launch coalescing (mhe_set_launch_hook): the calling thread's hook, off inside mhe_launch_run
static thread_local mhe_launch_hook tl_hook = nullptr;
static thread_local void *tl_hook_user = nullptr;
static thread_local int tl_hook_off = 0;

// true when the launch was handed to the hook (which ran it and set l.rc)
static bool hooked(mhe_ctx *c, mhe_launch &l)
{
    if (!tl_hook || tl_hook_off) return false;
    l.rc = -1;
    tl_hook(c, &l, tl_hook_user);
    return true;
}

// Forward NTT of [polys][limbs] (limb l on prime l).
static int run_ntt_fwd(mhe_ctx *c, const u64 *src, u64 *dst, int polys, int limbs, int full, hipStream_t st)
{
    count_op(c, MHE_OPK_NTT, limbs, (unsigned long long)polys);
    JobFwdPlain j;
    j.src = src;
    j.dst = dst;
    j.primes = c->primes;
    j.tw = c->tw;
    j.limbs = limbs;
    j.log_n = c->log_n;
    j.mode = 0;
    fwd_col(j, c->log_n, polys * limbs, c->nm, st);
    j.src = dst;
    j.mode = full;
    fwd_row(j, c->log_n, polys * limbs, c->nm, st);
    HIP_LAUNCH_CHECK();
    return MHE_OK;
}

static int run_ntt_inv(mhe_ctx *c, const u64 *src, u64 *dst, int polys, int limbs, int full, hipStream_t st)
{
    count_op(c, MHE_OPK_NTT, limbs, (unsigned long long)polys);
    JobInvPlain j;
    j.src = src;
    j.dst = dst;
    j.primes = c->primes;
    j.tw = c->itw;
    j.limbs = limbs;
    j.log_n = c->log_n;
    j.mode = 0;
    inv_row(j, c->log_n, polys * limbs, c->nm, st);
    j.src = dst;
    j.mode = full;
    inv_col(j, c->log_n, polys * limbs, c->nm, st);
    HIP_LAUNCH_CHECK();
    return MHE_OK;
}

// One entry of a (batched) key switch.
struct KsJob
{
    u64 *ct;               // [2][L][n]
    const u64 *target;     // [L][n], NTT form
    const u64 *key;        // [digits][2][key_limbs][n]
    int key_limbs;
    u64 *rescale_out;      // HMult: [2][L-1][n] (see run_switch_key_batch), else nullptr
};

static int ks_check_key(mhe_ctx *c, const KsJob &j, int L, hipStream_t st, int *kpack)
{
    if (j.key_limbs < L + 1 || j.key_limbs > c->K) return fail(MHE_ERR_ARG, "kswitch_keys is not valid for encryption parameters");
    // a prepared key (mhe_key_prepare) is recognised by the fused MAC itself (key_word_prepared
    // on a word of each slot); the separate-MAC debugging path reads SEAL's layout only
    *kpack = 1;
    if (!c->ks_fused)
    {
        int tagged = 0;
        int r0 = key_tagged(c, j.key, j.key_limbs, st, &tagged);
        if (r0) return r0;
        if (tagged) return fail(MHE_ERR_ARG, "key switch: prepared keys need the fused key MAC");
        *kpack = 0;
    }
    // the key slice one switch streams: L digits x 2 polys x (L + 1) primes
    c->key_bytes += 2ull * (unsigned long long)L * (unsigned long long)(L + 1) * c->n * 8ull;
    // prepared: doubles stream the same 8 B per residue, the 48-bit planes 6 B for primes below 2^48
    // (the format of a prepared key is not known here without a host sync: counted as doubles)
    c->key_bytes_prep += 2ull * (unsigned long long)L * (unsigned long long)(L + 1) * c->n * 8ull;
    return MHE_OK;
}

// Step 4 of a (batched) key switch, the ModDown (evaluator.cpp:2466-2524), over the key inner
// products in w->e[e].acc (or accs[e]): ct_e += ModDown(acc_e), or with rescale_out the fused HMult tail (see
// run_switch_key_batch).  special_inv_done: the key MAC already ran the special limbs' inverse
// row pass.
static void run_moddown(mhe_ctx *c, const KsJob *jobs, int B, int L, Workspace *w, int special_inv_done, int c1_write,
                        hipStream_t st, u64 *const *accs = nullptr)
{
    // key products of entry e: accs[e] when given (hoisted rotations), else the entry's scratch
    auto A = [&](int e) { return accs ? accs[e] : w->e[e].acc; };
    const bool hm = jobs[0].rescale_out != nullptr;
    const int log_n = c->log_n;
    const size_t n = c->n;
    // ModDown (evaluator.cpp:2466-2524): INTT_lazy of the special limbs, then fused
    //    lift + NTT + (c + 4q - t) * P^-1 + add.
    {
        JobB<JobStrided> j;
        j.per = 2;
        for (int e = 0; e < B; e++)
            j.j[e] = JobStrided{ A(e) + (size_t)L * n, A(e) + (size_t)L * n, (size_t)(L + 1) * n,
                                 (size_t)(L + 1) * n, c->K - 1, 0, c->primes, c->itw, log_n, 0 };
        if (!special_inv_done) inv_row(j, log_n, 2 * B, c->nm, st);
        // the special limbs' inverse column pass runs inside the lift column pass (k_icol_lift)
        // (not in the HMult tail: JobMDRCol reads the fully inverse-transformed special limbs)
        ColSrc cs{};
        cs.stride = (size_t)(L + 1) * n;
        cs.per = 2;
        cs.primes = c->primes;
        cs.itw = c->itw;
        cs.pi = c->K - 1;
        for (int e = 0; e < B; e++) cs.src[e] = A(e) + (size_t)L * n;
        const bool fuse = c->icol_fused && (!hm || L < 2);
        if (!fuse) inv_col(j, log_n, 2 * B, c->nm, st);
        if (!hm || L < 2)
        {
            JobB<JobModDownCol> dc;
            dc.per = 2 * L;
            JobB<JobModDownRow> dr;
            dr.per = 2 * L;
            for (int e = 0; e < B; e++)
            {
                dc.j[e] = JobModDownCol{ A(e), w->e[e].modup, c->primes, c->tw, L, c->K, log_n };
                dr.j[e] = JobModDownRow{ w->e[e].modup, A(e), jobs[e].ct, c->primes, c->tw, c->invq, L, c->K, log_n };
                dr.j[e].fp = c->nm.fp ? 1 : 0;
                dr.j[e].c1_write = c1_write;
            }
            if (fuse)
                icol_lift(cs, dc, 2 * B, L, log_n, c->nm, st);
            else
                fwd_col(dc, log_n, 2 * L * B, c->nm, st);
            fwd_row(dr, log_n, 2 * L * B, c->nm, st);
        }
        else
        {
            // ModDown of limb L-1 only, its INTT (the rescale's "last"), then ModDown and
            // rescale of the other limbs through one forward NTT each
            JobB<JobModDownCol> dc;
            dc.per = 2;
            JobB<JobModDownRow> dr;
            dr.per = 2;
            JobB<JobLastInv> li;
            li.per = 2;
            JobB<JobStrided> j2;
            j2.per = 2;
            JobB<JobMDRCol> mc;
            mc.per = 2 * (L - 1);
            JobB<JobMDRRow> mr;
            mr.per = 2 * (L - 1);
            for (int e = 0; e < B; e++)
            {
                dc.j[e] = JobModDownCol{ A(e), w->e[e].modup, c->primes, c->tw, L, c->K, log_n, L - 1 };
                dr.j[e] = JobModDownRow{ w->e[e].modup, A(e), jobs[e].ct, c->primes, c->tw, c->invq, L, c->K, log_n, L - 1 };
                dr.j[e].fp = c->nm.fp ? 1 : 0;
                li.j[e] = JobLastInv{ jobs[e].ct, w->e[e].coeff, c->primes, c->itw, L, log_n, 1 };
                j2.j[e] = JobStrided{ w->e[e].coeff, w->e[e].coeff, n, n, L - 1, 0, c->primes, c->itw, log_n, 1 };
                mc.j[e] = JobMDRCol{ A(e), w->e[e].coeff, w->e[e].modup, c->primes, c->tw, c->invq, L, c->K, log_n,
                                     c->nm.fp ? 1 : 0 };
                mr.j[e] = JobMDRRow{ w->e[e].modup, A(e), jobs[e].ct, jobs[e].rescale_out, c->primes, c->tw, c->invq,
                                     L, c->K, log_n, c->nm.fp ? 1 : 0 };
            }
            fwd_col(dc, log_n, 2 * B, c->nm, st);
            fwd_row(dr, log_n, 2 * B, c->nm, st);
            inv_row(li, log_n, 2 * B, c->nm, st);
            inv_col(j2, log_n, 2 * B, c->nm, st);
            if (c->nm.fp == 1)
                col_lift2(mc, 2 * B, L - 1, log_n, c->nm, st);
            else
                fwd_col(mc, log_n, 2 * (L - 1) * B, c->nm, st);
            fwd_row(mr, log_n, 2 * (L - 1) * B, c->nm, st);
        }
    }
}

// switch_key_inplace (evaluator.cpp:2281-2525) for B <= MHE_MAXB independent entries of one
// level L, every kernel launched once for all of them: ct_e[2][L][n] += KS(target_e[L][n]).
// rescale_out != nullptr (HMult; all entries or none): ct_e is the first two polys of a product,
// and instead of ct += KS(target) the result of rescale_to_next(ct + KS(target)) goes to
// rescale_out [2][L-1][n] (JobMDRCol / JobMDRRow); ct limb L-1 is overwritten on the way.
// c1_write: ct[1] is taken as zero and written, not read (target may then alias ct[1]: it is last
// read by the key MAC, before the ModDown writes ct).
static int run_switch_key_batch(mhe_ctx *c, const KsJob *jobs, int B, int L, hipStream_t st, int c1_write = 0)
{
    if (B < 1 || B > MHE_MAXB) return fail(MHE_ERR_ARG, "key switch: batch size out of range");
    // mhe_debug_fail_switch's countdown (tests): this launch sequence fails before its first launch
    for (int v = c->fail_switch.load(); v > 0;)
        if (c->fail_switch.compare_exchange_weak(v, v - 1))
        {
            if (v == 1) return fail(MHE_ERR_MEMORY, "device allocation failed (injected)");
            break;
        }
    const bool hm = jobs[0].rescale_out != nullptr;
    for (int e = 0; e < B; e++)
        if ((jobs[e].rescale_out != nullptr) != hm) return fail(MHE_ERR_ARG, "key switch: mixed fused-rescale batch");
    if (c1_write && hm) return fail(MHE_ERR_ARG, "key switch: c1_write with a fused rescale");
    if (!c->ks_fused && B > 1)
    {
        // the separate-MAC debugging path runs one entry at a time
        for (int e = 0; e < B; e++)
        {
            int r = run_switch_key_batch(c, jobs + e, 1, L, st, c1_write);
            if (r) return r;
        }
        return MHE_OK;
    }
    int kpack = 1;
    for (int e = 0; e < B; e++)
    {
        int r = ks_check_key(c, jobs[e], L, st, &kpack);
        if (r) return r;
    }
    count_op(c, MHE_OPK_KEYSWITCH, L, (unsigned long long)B);
    if (hm) count_op(c, MHE_OPK_RESCALE, L, 2ull * B); // the fused HMult tail rescales both polys
    Workspace *w;
    int r = get_ws(c, st, c->K - 1, &w, B);
    if (r) return r;
    const int log_n = c->log_n;
    const size_t n = c->n;
    int special_inv_done = 0; // the fused MAC ran the special limbs' inverse row pass
    // 1. t_target = INTT(target), canonical (evaluator.cpp:2351-2354)
    {
        JobB<JobStrided> j;
        j.per = L;
        for (int e = 0; e < B; e++) j.j[e] = JobStrided{ jobs[e].target, w->e[e].coeff, n, n, 0, 1, c->primes, c->itw, log_n, 0 };
        inv_row(j, log_n, B * L, c->nm, st);
        for (int e = 0; e < B; e++)
        {
            j.j[e].src = w->e[e].coeff;
            j.j[e].mode = 1;
        }
        inv_col(j, log_n, B * L, c->nm, st);
    }
    if (c->ks_fused)
    {
        // 2+3. ModUp column pass, then its row pass fused with the key MAC so NTT'd digits
        //      never leave registers (chunks of output primes sized for the Infinity Cache
        //      measured slower at every size).
        const int P = L + 1;
        // 48-bit intermediate (ntt.h tile16): only k_modup_col writes it, so only with column groups
        const int pack = (c->ks_pack && c->ks_colgroups > 0) ? 1 : 0;
        KsPtrs kp{};
        int share = B > 1 ? 1 : 0; // one key for every entry: XCD-grouped entries (k_ks_row_mac)
        for (int e = 0; e < B; e++)
            if (jobs[e].key != jobs[0].key || jobs[e].key_limbs != jobs[0].key_limbs) share = 0;
        if (!c->ks_share) share = 0;
        for (int e = 0; e < B; e++)
        {
            kp.coeff[e] = w->e[e].coeff;
            kp.inter[e] = w->e[e].modup;
            kp.target[e] = jobs[e].target;
            kp.key[e] = jobs[e].key;
            kp.acc[e] = w->e[e].acc;
            kp.key_limbs[e] = jobs[e].key_limbs;
        }
        for (int I0 = 0; I0 <= L; I0 += P)
        {
            const int cnt = (I0 + P <= L + 1) ? P : L + 1 - I0;
            hipEvent_t *tc = timing_slot(c, w, TK_MODUP_COL, st);
            if (c->ks_colgroups > 0)
            {
                const int IG = c->ks_colgroups < cnt ? c->ks_colgroups : cnt;
                modup_col(kp, B, c->primes, c->tw, L, c->K, log_n, c->nm_ks, I0, cnt, IG, pack, st);
            }
            else
            {
                JobB<JobModUpCol> j;
                j.per = cnt * L;
                for (int e = 0; e < B; e++) j.j[e] = JobModUpCol{ w->e[e].coeff, w->e[e].modup, c->primes, c->tw, L, c->K, log_n, I0 };
                fwd_col(j, log_n, B * cnt * L, c->nm, st);
            }
            timing_end(tc, st);
            hipEvent_t *tm = timing_slot(c, w, TK_KS_ROW_MAC, st);
            const int has_special = (I0 <= L && L < I0 + cnt && c->ks_inv_fused) ? 1 : 0;
            special_inv_done |= ks_row_mac_chunk(kp, B, c->primes, c->tw, L, c->K, log_n, c->nm_ks, I0, cnt, pack, kpack,
                                                 share, c->itw, has_special, st);
            timing_end(tm, st);
        }
    }
    else
    {
        // 2+3. (MHE_KS_FUSED=0, the independent debugging path) ModUp + key inner products in
        //      three kernels: lift digit J to prime I and NTT it (evaluator.cpp:2386-2408; I == J
        //      skipped), then acc[k][I] = sum_J digit * key[J][k][I] (evaluator.cpp:2410-2463).
        //      (One entry: B == 1 here.)
        const int P = L + 1;
        for (int I0 = 0; I0 <= L; I0 += P)
        {
            const int cnt = (I0 + P <= L + 1) ? P : L + 1 - I0;
            JobModUpCol j{ w->coeff, w->modup, c->primes, c->tw, L, c->K, log_n, I0 };
            fwd_col(j, log_n, cnt * L, c->nm, st);
            JobModUpRow r2{ w->modup, c->primes, c->tw, L, c->K, log_n, I0 };
            fwd_row(r2, log_n, cnt * L, c->nm, st);
            dim3 grid((unsigned)(n / 512), cnt);
            hipLaunchKernelGGL(k_ks_mac, grid, dim3(256), 0, st, w->modup, jobs[0].target, jobs[0].key, w->acc, c->primes, L,
                               c->K, jobs[0].key_limbs, log_n, I0);
        }
    }
    run_moddown(c, jobs, B, L, w, special_inv_done, c1_write, st);
    HIP_LAUNCH_CHECK();
    return MHE_OK;
}

static int run_switch_key(mhe_ctx *c, u64 *ct, const u64 *target, const u64 *key, int key_limbs, int L,
                          hipStream_t st, u64 *rescale_out = nullptr, int c1_write = 0)
{
    const KsJob j{ ct, target, key, key_limbs, rescale_out };
    return run_switch_key_batch(c, &j, 1, L, st, c1_write);
}

// rescale_to_next (util/rns.cpp:737-808) of B <= MHE_MAXB independent ciphertexts of `size` polys
// at L limbs, in[e] -> out[e] ([size][L-1][n]), every kernel launched once for all of them.
static int run_rescale_batch(mhe_ctx *c, const u64 *const *in, u64 *const *out, int B, int size, int L, hipStream_t st)
{
    if (B < 1 || B > MHE_MAXB) return fail(MHE_ERR_ARG, "rescale: batch size out of range");
    Workspace *w;
    int r = get_ws(c, st, c->K - 1, &w, B);
    if (r) return r;
    count_op(c, MHE_OPK_RESCALE, L, (unsigned long long)B * size);
    const int log_n = c->log_n;
    // last[s] = INTT(in[s][L-1]) canonical -> the entry's coeff (size <= 3 polys)
    JobB<JobLastInv> li;
    li.per = size;
    JobB<JobRescaleCol> rc;
    rc.per = size * (L - 1);
    JobB<JobRescaleRow> rr;
    rr.per = size * (L - 1);
    ColSrc cs{};
    cs.stride = c->n;
    cs.per = size;
    cs.primes = c->primes;
    cs.itw = c->itw;
    cs.pi = L - 1;
    for (int e = 0; e < B; e++)
    {
        li.j[e] = JobLastInv{ in[e], w->e[e].coeff, c->primes, c->itw, L, log_n, 1 };
        rc.j[e] = JobRescaleCol{ w->e[e].coeff, w->e[e].modup, c->primes, c->tw, L, log_n };
        rr.j[e] = JobRescaleRow{ w->e[e].modup, in[e], out[e], c->primes, c->tw, c->invq, L, c->K, log_n };
        rr.j[e].fp = c->nm.fp ? 1 : 0;
        cs.src[e] = w->e[e].coeff;
    }
    inv_row(li, log_n, size * B, c->nm, st);
    if (c->icol_fused)
    {
        // the last limb's inverse column pass runs inside the lift column pass (k_icol_lift)
        icol_lift(cs, rc, size * B, L - 1, log_n, c->nm, st);
    }
    else
    {
        JobB<JobStrided> j2;
        j2.per = size;
        for (int e = 0; e < B; e++) j2.j[e] = JobStrided{ w->e[e].coeff, w->e[e].coeff, c->n, c->n, L - 1, 0, c->primes, c->itw, log_n, 1 };
        inv_col(j2, log_n, size * B, c->nm, st);
        fwd_col(rc, log_n, size * (L - 1) * B, c->nm, st);
    }
    fwd_row(rr, log_n, size * (L - 1) * B, c->nm, st);
    HIP_LAUNCH_CHECK();
    return MHE_OK;
}

static int run_rescale(mhe_ctx *c, const u64 *in, u64 *out, int size, int L, hipStream_t st)
{
    return run_rescale_batch(c, &in, &out, 1, size, L, st);
}

// ================================================================ internal (encode.hip)
int mhe_internal_fail(int code, const char *msg)
{
    return fail(code, msg);
}

int mhe_internal_ntt_forward(mhe_ctx *c, uint64_t *data, int polys, int limbs, int full, hipStream_t st)
{
    return run_ntt_fwd(c, data, data, polys, limbs, full, st);
}

int mhe_internal_primes(mhe_ctx *c, const PrimeDev **dev, const uint64_t **host, int *count, int *log_n)
{
    if (!valid_ctx(c)) return MHE_ERR_ARG;
    *dev = c->primes;
    *host = c->q.data();
    *count = c->K;
    *log_n = c->log_n;
    return MHE_OK;
}

// ================================================================================ C ABI
MHE_EXPORT const char *mhe_last_error(void)
{
    return g_err.c_str();
}

MHE_EXPORT int mhe_version(void)
{
    return 1;
}

MHE_EXPORT int mhe_coeff_modulus_create(uint64_t n, const int *bit_sizes, int count, uint64_t *out)
{
    if (!bit_sizes || !out || count <= 0 || count > 64 || (n & (n - 1)) || n < 2)
        return fail(MHE_ERR_ARG, "bit_sizes is invalid");
    std::map<int, std::vector<u64>> table;
    std::map<int, int> cnt;
    for (int i = 0; i < count; i++)
    {
        if (bit_sizes[i] < 2 || bit_sizes[i] > 60) return fail(MHE_ERR_ARG, "bit_sizes is invalid");
        cnt[bit_sizes[i]]++;
    }
    for (auto &kv : cnt)
    {
        const int bits = kv.first;
        const u64 factor = 2 * n;
        u64 value = ((u64)1 << bits) - factor + 1, lower = (u64)1 << (bits - 1);
        std::vector<u64> &v = table[bits];
        while ((int)v.size() < kv.second && value > lower)
        {
            if (host::is_prime(value)) v.push_back(value);
            value -= factor;
        }
        if ((int)v.size() < kv.second) return fail(MHE_ERR_ARG, "failed to find enough qualifying primes");
    }
    for (int i = 0; i < count; i++)
    {
        auto &v = table[bit_sizes[i]];
        out[i] = v.back();
        v.pop_back();
    }
    return MHE_OK;
}

MHE_EXPORT uint32_t mhe_galois_elt_from_step(int log_n, int step)
{
    const u64 n = (u64)1 << log_n, m = 2 * n;
    if (step == 0) return (uint32_t)(m - 1);
    u64 pos = (u64)(step < 0 ? -(long long)step : step);
    if (pos >= (n >> 1)) return 0;
    u64 s = step < 0 ? (n >> 1) - pos : pos;
    u64 elt = 1;
    while (s--) elt = (elt * 5) & (m - 1); // generator_ = 5 (util/galois.h:169)
    return (uint32_t)elt;
}

MHE_EXPORT int mhe_ctx_create(mhe_ctx **out, int log_n, const uint64_t *moduli, int count, int device)
{
    if (!out) return fail(MHE_ERR_ARG, "ctx is null");
    *out = nullptr;
    if (log_n < 12 || log_n > 16) return fail(MHE_ERR_ARG, "poly_modulus_degree is invalid");
    if (!moduli || count < 2 || count > 64) return fail(MHE_ERR_ARG, "coeff_modulus is invalid");
    const size_t n = (size_t)1 << log_n;
    for (int i = 0; i < count; i++)
    {
        u64 q = moduli[i];
        if (q < 2 || q >= ((u64)1 << 61) || (q - 1) % (2 * n) != 0 || !host::is_prime(q))
            return fail(MHE_ERR_ARG, "coeff_modulus is not NTT-friendly prime");
    }
    mhe_ctx *c = new (std::nothrow) mhe_ctx;
    if (!c) return fail(MHE_ERR_MEMORY, "out of memory");
    c->device = device;
    c->log_n = log_n;
    c->n = n;
    c->K = count;
    c->q.assign(moduli, moduli + count);
    if (const char *f = getenv("MHE_KS_FUSED")) c->ks_fused = atoi(f);
    if (const char *f = getenv("MHE_HMULT_FUSED")) c->hmult_fused = atoi(f);
    if (const char *f = getenv("MHE_KS_SHARE")) c->ks_share = atoi(f);
    if (const char *f = getenv("MHE_KS_COLGROUPS")) c->ks_colgroups = atoi(f);
    if (const char *f = getenv("MHE_KS_INV_FUSED")) c->ks_inv_fused = atoi(f);
    if (const char *f = getenv("MHE_KS_PACK")) c->ks_pack = atoi(f);
    if (const char *f = getenv("MHE_GALOIS_FUSED")) c->galois_fused = atoi(f);
    if (const char *f = getenv("MHE_ICOL_FUSED")) c->icol_fused = atoi(f);
    if (const char *f = getenv("MHE_KS_HOIST")) c->ks_hoist = atoi(f);
    std::vector<Tw> tw((size_t)count * n), itw((size_t)count * n), invq((size_t)count * count);
    c->primes_h.resize(count);
    for (int k = 0; k < count; k++)
    {
        const u64 q = moduli[k];
        PrimeDev &p = c->primes_h[k];
        p.q = q;
        p.two_q = 2 * q;
        p.four_q = 4 * q;
        p.qd = (double)q;
        p.qi = 1.0 / (double)q;
        u128 ratio = (~(u128)0) / q;
        p.r0 = (u64)ratio;
        p.r1 = (u64)(ratio >> 64);
        // NTTTables::initialize (util/ntt.cpp:30-89)
        u64 psi = host::minimal_primitive_root(2 * n, q), ipsi = 0, ninv = 0;
        if (!psi || !host::invmod(psi, q, ipsi) || !host::invmod(n % q, q, ninv))
        {
            delete c;
            return fail(MHE_ERR_ARG, "invalid modulus");
        }
        Tw *t = &tw[(size_t)k * n], *it = &itw[(size_t)k * n];
        u64 pw = 1, ipw = 1;
        for (size_t i = 0; i < n; i++)
        {
            const u32 r = host::rev_bits((u32)i, log_n);
            t[r].x = pw;
            t[r].y = host::shoup(pw, q);
            it[r].x = ipw;
            it[r].y = host::shoup(ipw, q);
            pw = host::mulmod(pw, psi, q);
            ipw = host::mulmod(ipw, ipsi, q);
        }
        p.ninv = ninv;
        p.ninv_q = host::shoup(ninv, q);
        p.last_w = host::mulmod(it[1].x, ninv, q);
        p.last_wq = host::shoup(p.last_w, q);
    }
    for (int j = 0; j < count; j++)
        for (int i = 0; i < count; i++)
        {
            u64 inv = 0;
            if (i != j) host::invmod(moduli[j] % moduli[i], moduli[i], inv);
            invq[(size_t)j * count + i].x = inv;
            invq[(size_t)j * count + i].y = host::shoup(inv, moduli[i]);
        }
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess)
    {
        hipMemPool_t pool;
        if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess)
        {
            uint64_t threshold = UINT64_MAX;
            (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &threshold);
        }
    }
    if (e == hipSuccess) e = hipMalloc(&c->primes, sizeof(PrimeDev) * count);
    if (e == hipSuccess) e = hipMalloc(&c->tw, sizeof(Tw) * tw.size());
    if (e == hipSuccess) e = hipMalloc(&c->itw, sizeof(Tw) * itw.size());
    if (e == hipSuccess) e = hipMalloc(&c->invq, sizeof(Tw) * invq.size());
    if (e == hipSuccess) e = hipMemcpy(c->primes, c->primes_h.data(), sizeof(PrimeDev) * count, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(c->tw, tw.data(), sizeof(Tw) * tw.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(c->itw, itw.data(), sizeof(Tw) * itw.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(c->invq, invq.data(), sizeof(Tw) * invq.size(), hipMemcpyHostToDevice);
    // FP64 arithmetic (fparith.h) needs q < 2^51 for every prime of the chain; with only the last
    // (special) prime above, the ModUp kernels still run FP64 for every other output prime
    bool fp = true, fp_data = true;
    for (int k = 0; k < count; k++) fp = fp && moduli[k] < ((u64)1 << 51);
    for (int k = 0; k + 1 < count; k++) fp_data = fp_data && moduli[k] < ((u64)1 << 51);
    if (const char *f = getenv("MHE_FP"))
        if (atoi(f) == 0) fp = fp_data = false;
    bool mix = !fp && fp_data && count > 1;
    if (const char *f = getenv("MHE_KS_MIX")) mix = mix && atoi(f) != 0;
    if (e == hipSuccess && fp)
    {
        // hoisted rotations (hoist.h): q_j mod q_i and its quotient by q_i
        std::vector<TwF> cm((size_t)count * count);
        for (int j = 0; j < count; j++)
            for (int i = 0; i < count; i++)
            {
                const u64 r = moduli[j] % moduli[i];
                cm[(size_t)j * count + i] = make_double2((double)r, (double)r / (double)moduli[i]);
            }
        e = hipMalloc(&c->cmodf, sizeof(TwF) * cm.size());
        if (e == hipSuccess) e = hipMemcpy(c->cmodf, cm.data(), sizeof(TwF) * cm.size(), hipMemcpyHostToDevice);
    }
    if (e == hipSuccess && (fp || mix))
    {
        std::vector<TwF> twf((size_t)2 * count * n);
        for (int k = 0; k < count; k++)
        {
            const double qd = (double)moduli[k];
            for (size_t i = 0; i < n; i++)
            {
                const size_t o = (size_t)k * n + i;
                twf[o] = make_double2((double)tw[o].x, (double)tw[o].x / qd);
                twf[(size_t)count * n + o] = make_double2((double)itw[o].x, (double)itw[o].x / qd);
            }
        }
        e = hipMalloc(&c->twf, sizeof(TwF) * twf.size());
        if (e == hipSuccess) e = hipMemcpy(c->twf, twf.data(), sizeof(TwF) * twf.size(), hipMemcpyHostToDevice);
        if (e == hipSuccess)
        {
            NttMode m;
            m.fp = fp ? 1 : 2;
            m.dfwd = (long long)((const char *)c->twf - (const char *)c->tw);
            m.dinv = (long long)((const char *)(c->twf + (size_t)count * n) - (const char *)c->itw);
            if (fp) c->nm = m;
            c->nm_ks = m;
        }
    }
    if (e != hipSuccess)
    {
        (void)hipFree(c->cmodf);
        (void)hipFree(c->twf);
        (void)hipFree(c->primes);
        (void)hipFree(c->tw);
        (void)hipFree(c->itw);
        (void)hipFree(c->invq);
        c->primes = nullptr;
        delete c;
        return fail(MHE_ERR_DEVICE, std::string("mhe_ctx_create: ") + hipGetErrorString(e));
    }
    mhe_internal_ctx_count(+1);
    *out = c;
    return MHE_OK;
}

MHE_EXPORT int mhe_ctx_destroy(mhe_ctx *c)
{
    if (!c) return MHE_OK;
    (void)hipSetDevice(c->device);
    for (auto &kv : c->masks) (void)hipFree(kv.second);
    for (auto &kv : c->ws)
    {
        if (kv.second.base) (void)hipFree(kv.second.base);
        if (kv.second.hoist_base) (void)hipFree(kv.second.hoist_base);
        if (kv.second.flags) (void)hipFree(kv.second.flags);
        for (auto &v : kv.second.ev)
            for (auto &e : v)
            {
                (void)hipEventDestroy(e.first);
                (void)hipEventDestroy(e.second);
            }
    }
    (void)hipFree(c->primes);
    (void)hipFree(c->tw);
    (void)hipFree(c->itw);
    (void)hipFree(c->invq);
    (void)hipFree(c->twf);
    (void)hipFree(c->cmodf);
    delete c;
    mhe_internal_ctx_count(-1);
    return MHE_OK;
}

MHE_EXPORT int mhe_ctx_reserve(mhe_ctx *c, int max_limbs, void *stream)
{
    if (!valid_ctx(c)) return fail(MHE_ERR_ARG, "context is not valid");
    Workspace *w;
    return get_ws(c, S(stream), max_limbs < c->K - 1 ? c->K - 1 : max_limbs, &w);
}

MHE_EXPORT int mhe_malloc(mhe_ctx *c, void **dptr, size_t bytes)
{
    if (!valid_ctx(c) || !dptr) return fail(MHE_ERR_ARG, "invalid argument");
    HIP_TRY(hipSetDevice(c->device));
    if (hipMalloc(dptr, bytes ? bytes : 1) != hipSuccess) return fail(MHE_ERR_MEMORY, "device allocation failed");
    return MHE_OK;
}

// MHE_ALLOC_TRACE=1: track live stream-ordered allocations and report double frees, frees of
// unknown pointers and overlapping live ranges (debugging aid)
static std::mutex g_trace_mu;
static std::map<uintptr_t, size_t> g_live;
static int trace_on()
{
    static int on = -1;
    if (on < 0)
    {
        const char *e = getenv("MHE_ALLOC_TRACE");
        on = e && e[0] >= '1';
    }
    return on;
}


// trace mode: the range [p, p + words) must lie inside one live stream-ordered allocation
static void trace_range(const char *fn, const char *what, const void *p, size_t words)
{
    if (!trace_on() || !p) return;
    std::lock_guard<std::mutex> g(g_trace_mu);
    const uintptr_t a = (uintptr_t)p, e = a + words * 8;
    auto it = g_live.upper_bound(a);
    if (it == g_live.begin()) return; // not a tracked allocation (workspace, hipMalloc)
    --it;
    if (it->first + it->second < a) return;
    if (e > it->first + it->second)
        fprintf(stderr, "[alloc-trace] %s: %s range [%p, +%zu words) exceeds allocation %p of %zu words by %zu words\n",
                fn, what, p, words, (void *)it->first, it->second / 8, (size_t)(e - (it->first + it->second)) / 8);
}
// trace level 2: at every instrumented entry, synchronise and check the first 4 KiB of every live
// allocation's guard; a hit names the previous instrumented call as the writer
static const char *g_prev_fn = "(none)";
static size_t g_prev_info[4];
static void trace_check_all(const char *fn, size_t i0, size_t i1, size_t i2, size_t i3)
{
    static int lvl = -1;
    if (lvl < 0)
    {
        const char *e = getenv("MHE_ALLOC_TRACE");
        lvl = e ? atoi(e) : 0;
    }
    if (lvl < 2) return;
    (void)hipDeviceSynchronize();
    std::lock_guard<std::mutex> g(g_trace_mu);
    std::vector<unsigned char> buf(4096);
    for (auto &kv : g_live)
    {
        (void)hipMemcpy(buf.data(), (const char *)kv.first + kv.second, 4096, hipMemcpyDeviceToHost);
        bool bad = false;
        for (unsigned char b : buf) bad |= b != 0xAB;
        if (bad)
        {
            fprintf(stderr, "[alloc-trace] guard of %#lx (%zu words) hit before %s; previous call %s(%zu, %zu, %zu, %zu)\n",
                    (unsigned long)kv.first, kv.second / 8, fn, g_prev_fn, g_prev_info[0], g_prev_info[1],
                    g_prev_info[2], g_prev_info[3]);
            (void)hipMemset((char *)kv.first + kv.second, 0xAB, (size_t)16 << 20); // re-arm
        }
    }
    g_prev_fn = fn;
    g_prev_info[0] = i0;
    g_prev_info[1] = i1;
    g_prev_info[2] = i2;
    g_prev_info[3] = i3;
}
#define TR(what, p, words) trace_range(__func__, what, p, (size_t)(words))
#define TRC(a, b, cc, d) trace_check_all(__func__, (size_t)(a), (size_t)(b), (size_t)(cc), (size_t)(d))

MHE_EXPORT int mhe_malloc_async(mhe_ctx *c, void **dptr, size_t bytes, void *stream)
{
    if (!valid_ctx(c) || !dptr) return fail(MHE_ERR_ARG, "invalid argument");
    const size_t kGuard = trace_on() ? ((size_t)16 << 20) : 0;
    if (injected_alloc_failure(c)) return fail(MHE_ERR_MEMORY, "device allocation failed");
    if (mhe_internal_alloc(dptr, (bytes ? bytes : 1) + kGuard, S(stream)) != hipSuccess)
        return fail(MHE_ERR_MEMORY, "device allocation failed");
    if (trace_on())
    {
        (void)hipMemsetAsync((char *)*dptr + (bytes ? bytes : 1), 0xAB, kGuard, S(stream));
        std::lock_guard<std::mutex> g(g_trace_mu);
        const uintptr_t a = (uintptr_t)*dptr, e = a + (bytes ? bytes : 1);
        auto it = g_live.upper_bound(a);
        if (it != g_live.begin())
        {
            auto pv = std::prev(it);
            if (pv->first + pv->second > a)
                fprintf(stderr, "[alloc-trace] overlap: new [%#lx,+%zu) inside live [%#lx,+%zu)\n", (unsigned long)a,
                        bytes, (unsigned long)pv->first, pv->second);
        }
        if (it != g_live.end() && it->first < e)
            fprintf(stderr, "[alloc-trace] overlap: new [%#lx,+%zu) covers live [%#lx,+%zu)\n", (unsigned long)a, bytes,
                    (unsigned long)it->first, it->second);
        g_live[a] = bytes ? bytes : 1;
    }
    return MHE_OK;
}

MHE_EXPORT int mhe_free_async(mhe_ctx *c, void *dptr, void *stream)
{
    if (!valid_ctx(c)) return fail(MHE_ERR_ARG, "invalid argument");
    if (trace_on() && dptr)
    {
        std::lock_guard<std::mutex> g(g_trace_mu);
        auto it = g_live.find((uintptr_t)dptr);
        if (it == g_live.end())
            fprintf(stderr, "[alloc-trace] free of unknown or already freed pointer %p\n", dptr);
        else
        {
            const size_t kGuard = (size_t)16 << 20;
            std::vector<unsigned char> gbuf(kGuard);
            (void)hipStreamSynchronize(S(stream));
            (void)hipMemcpy(gbuf.data(), (char *)dptr + it->second, kGuard, hipMemcpyDeviceToHost);
            size_t first = kGuard, last = 0;
            for (size_t i = 0; i < kGuard; i++)
                if (gbuf[i] != 0xAB)
                {
                    first = std::min(first, i);
                    last = i;
                }
            if (first < kGuard)
                fprintf(stderr, "[alloc-trace] OVERRUN of allocation %p (%zu bytes = %zu words): guard bytes [%zu, %zu] written\n",
                        dptr, it->second, it->second / 8, first, last);
            g_live.erase(it);
        }
    }
    HIP_TRY(mhe_internal_free(dptr, S(stream)));
    return MHE_OK;
}

MHE_EXPORT int mhe_free(mhe_ctx *c, void *dptr)
{
    if (!valid_ctx(c)) return fail(MHE_ERR_ARG, "invalid argument");
    HIP_TRY(hipFree(dptr));
    return MHE_OK;
}

MHE_EXPORT int mhe_memcpy_h2d(mhe_ctx *c, void *dst, const void *src, size_t bytes, void *stream)
{
    if (!valid_ctx(c)) return fail(MHE_ERR_ARG, "invalid argument");
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, S(stream)));
    return MHE_OK;
}

MHE_EXPORT int mhe_memcpy_d2h(mhe_ctx *c, void *dst, const void *src, size_t bytes, void *stream)
{
    if (!valid_ctx(c)) return fail(MHE_ERR_ARG, "invalid argument");
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, S(stream)));
    return MHE_OK;
}

MHE_EXPORT int mhe_memcpy_d2d(mhe_ctx *c, void *dst, const void *src, size_t bytes, void *stream)
{
    TR("dst", dst, bytes / 8); TR("src", src, bytes / 8);
    TRC(0, 0, 0, 0);
    if (!valid_ctx(c)) return fail(MHE_ERR_ARG, "invalid argument");
    if (bytes && dst != src)
    {
        mhe_launch l{};
        l.kind = MHE_LK_COPY;
        l.a = (const u64 *)src;
        l.out = (u64 *)dst;
        l.bytes = bytes;
        l.stream = stream;
        if (hooked(c, l)) return l.rc;
    }
    HIP_TRY(mhe_internal_copy_d2d(dst, src, bytes, S(stream)));
    return MHE_OK;
}

// one launch as the entry point would have run it (the hook off)
static int launch_one(mhe_ctx *c, mhe_launch &l)
{
    switch (l.kind)
    {
    case MHE_LK_ADDSUB:
        return l.op == 0   ? mhe_add(c, l.a, l.b, l.out, l.polys, l.limbs, l.stream)
               : l.op == 1 ? mhe_sub(c, l.a, l.b, l.out, l.polys, l.limbs, l.stream)
                           : mhe_negate(c, l.a, l.out, l.polys, l.limbs, l.stream);
    case MHE_LK_MULPLAIN: return mhe_multiply_plain(c, l.a, l.b, l.out, l.polys, l.limbs, l.stream);
    case MHE_LK_MULPLAIN_ADD: return mhe_multiply_plain_add(c, l.a, l.b, l.out, l.polys, l.limbs, l.stream);
    case MHE_LK_SCALAR:
        return l.op == 0   ? mhe_multiply_scalar(c, l.a, l.scalars, l.out, l.polys, l.limbs, l.stream)
               : l.op == 1 ? mhe_add_scalar(c, l.a, l.scalars, l.out, l.polys, l.limbs, l.stream)
                           : mhe_set_scalar(c, l.scalars, l.out, l.polys, l.limbs, l.stream);
    case MHE_LK_TENSOR:
        return l.op ? mhe_ct_square(c, l.a, l.out, l.limbs, l.stream) : mhe_ct_multiply(c, l.a, l.b, l.out, l.limbs, l.stream);
    case MHE_LK_COPY: return mhe_memcpy_d2d(c, l.out, l.a, l.bytes, l.stream);
    }
    return fail(MHE_ERR_ARG, "unknown launch kind");
}

static bool same_shape(const mhe_launch &x, const mhe_launch &y)
{
    if (x.kind != y.kind || x.op != y.op || x.polys != y.polys || x.limbs != y.limbs || x.bytes != y.bytes ||
        x.stream != y.stream)
        return false;
    if (x.kind == MHE_LK_SCALAR)
        for (int l = 0; l < x.limbs; l++)
            if (x.scalars[l] != y.scalars[l]) return false;
    return true;
}

MHE_EXPORT int mhe_set_launch_hook(mhe_launch_hook hook, void *user)
{
    tl_hook = hook;
    tl_hook_user = user;
    return MHE_OK;
}

MHE_EXPORT int mhe_launch_run(mhe_ctx *c, mhe_launch *const *ls, int count)
{
    if (!valid_ctx(c)) return fail(MHE_ERR_ARG, "context is not valid");
    if (count < 0 || (count && !ls)) return fail(MHE_ERR_ARG, "invalid argument");
    struct Off
    {
        Off() { tl_hook_off++; }
        ~Off() { tl_hook_off--; }
    } off;
    std::vector<char> done((size_t)count, 0);
    int first_err = MHE_OK;
    for (int i = 0; i < count; i++)
    {
        if (done[i]) continue;
        // entries of i's shape, in order, up to MHE_MAXB per launch
        int grp[MHE_MAXB], B = 0;
        for (int j = i; j < count && B < MHE_MAXB; j++)
            if (!done[j] && same_shape(*ls[i], *ls[j])) grp[B++] = j;
        for (int k = 0; k < B; k++) done[grp[k]] = 1;
        mhe_launch &l0 = *ls[grp[0]];
        const bool aligned16 = l0.kind != MHE_LK_COPY || (l0.bytes & 15) == 0;
        bool ok_batch = B > 1 && aligned16;
        if (ok_batch && l0.kind == MHE_LK_COPY)
            for (int k = 0; k < B; k++)
                ok_batch = ok_batch && (((uintptr_t)ls[grp[k]]->a | (uintptr_t)ls[grp[k]]->out) & 15) == 0;
        if (!ok_batch)
        {
            for (int k = 0; k < B; k++)
            {
                mhe_launch &l = *ls[grp[k]];
                l.rc = launch_one(c, l);
                if (l.rc && !first_err) first_err = l.rc;
            }
            continue;
        }
        ElemPtrs P{};
        for (int k = 0; k < B; k++)
        {
            P.a[k] = ls[grp[k]]->a;
            P.b[k] = ls[grp[k]]->b;
            P.out[k] = ls[grp[k]]->out;
        }
        const hipStream_t st = S(l0.stream);
        if (l0.kind == MHE_LK_COPY)
        {
            const size_t cnt = l0.bytes / 16;
            const unsigned grid = (unsigned)std::min<size_t>((cnt + 255) / 256, 4096);
            hipLaunchKernelGGL(k_copy16_b, dim3(grid, (unsigned)B), dim3(256), 0, st, P, cnt);
        }
        else
        {
            ScalarTab t{};
            if (l0.kind == MHE_LK_SCALAR)
                for (int l = 0; l < l0.limbs; l++)
                {
                    t.v[l] = l0.scalars[l];
                    t.vq[l] = host::shoup(l0.scalars[l], c->q[l]);
                }
            // a tensor product covers one pair of 2-poly ciphertexts ([limbs] residues per output poly)
            const size_t total2 = ((size_t)(l0.kind == MHE_LK_TENSOR ? 1 : l0.polys) * l0.limbs << c->log_n) / 2;
            const int opk = l0.kind == MHE_LK_ADDSUB ? MHE_OPK_ADDSUB
                            : l0.kind == MHE_LK_SCALAR ? MHE_OPK_SCALAR
                            : l0.kind == MHE_LK_TENSOR ? MHE_OPK_TENSOR
                                                        : MHE_OPK_MULPLAIN;
            count_op(c, opk, l0.limbs, (unsigned long long)B * (l0.kind == MHE_LK_TENSOR ? 1 : l0.polys));
            if (l0.kind == MHE_LK_MULPLAIN_ADD) count_op(c, MHE_OPK_ADDSUB, l0.limbs, (unsigned long long)B * l0.polys);
            hipLaunchKernelGGL(k_elem_b, dim3(ELEM_GRID(total2).x, (unsigned)B), dim3(256), 0, st, P, c->primes, t,
                               l0.limbs, c->log_n, total2, l0.kind, l0.op, c->nm.fp ? 1 : 0);
        }
        const hipError_t e = hipGetLastError();
        const int rc = e == hipSuccess ? MHE_OK : fail(MHE_ERR_DEVICE, hipGetErrorString(e));
        for (int k = 0; k < B; k++) ls[grp[k]]->rc = rc;
        if (rc && !first_err) first_err = rc;
    }
    return first_err;
}

MHE_EXPORT int mhe_ctx_set_timing(mhe_ctx *c, int on)
{
    if (!valid_ctx(c)) return fail(MHE_ERR_ARG, "context is not valid");
    c->timing = on ? 1 : 0;
    return MHE_OK;
}

static bool hoist_ok(const mhe_ctx *c);

MHE_EXPORT int mhe_trim(mhe_ctx *c)
{
    if (!valid_ctx(c)) return fail(MHE_ERR_ARG, "context is not valid");
    HIP_TRY(hipSetDevice(c->device));
    release_cached_blocks();
    return MHE_OK;
}

MHE_EXPORT int mhe_debug_fail_switch(mhe_ctx *c, int nth)
{
    if (!valid_ctx(c) || nth < 0) return fail(MHE_ERR_ARG, "invalid argument");
    c->fail_switch.store(nth);
    return MHE_OK;
}

MHE_EXPORT int mhe_alloc_stats(uint64_t *retries, uint64_t *failures, int reset)
{
    if (!retries || !failures) return fail(MHE_ERR_ARG, "invalid argument");
    *retries = reset ? g_alloc_retries.exchange(0) : g_alloc_retries.load();
    *failures = reset ? g_alloc_failures.exchange(0) : g_alloc_failures.load();
    return MHE_OK;
}

MHE_EXPORT int mhe_debug_fail_alloc(mhe_ctx *c, int nth)
{
    if (!valid_ctx(c) || nth < 0) return fail(MHE_ERR_ARG, "invalid argument");
    c->fail_alloc.store(nth);
    return MHE_OK;
}

MHE_EXPORT int mhe_ctx_set_hoist(mhe_ctx *c, int on, int check)
{
    if (!valid_ctx(c)) return fail(MHE_ERR_ARG, "context is not valid");
    c->ks_hoist = on ? 1 : 0;
    c->hoist_check = check ? 1 : 0;
    return MHE_OK;
}

MHE_EXPORT int mhe_ctx_get_hoist(mhe_ctx *c, int *on, int *check)
{
    if (!valid_ctx(c) || !on || !check) return fail(MHE_ERR_ARG, "invalid argument");
    *on = hoist_ok(c) ? 1 : 0;
    *check = c->hoist_check.load();
    return MHE_OK;
}

MHE_EXPORT int mhe_hoist_stats(mhe_ctx *c, uint64_t *rotations, uint64_t *mac_launches, uint64_t *check_mismatches,
                               int reset)
{
    if (!valid_ctx(c) || !rotations || !mac_launches || !check_mismatches) return fail(MHE_ERR_ARG, "invalid argument");
    *rotations = reset ? c->hoist_rot.exchange(0) : c->hoist_rot.load();
    *mac_launches = reset ? c->hoist_mac.exchange(0) : c->hoist_mac.load();
    *check_mismatches = reset ? c->hoist_bad.exchange(0) : c->hoist_bad.load();
    return MHE_OK;
}

MHE_EXPORT int mhe_scratch_bytes(mhe_ctx *c, uint64_t *workspace, uint64_t *hoisting, uint64_t *masks, int *streams)
{
    if (!valid_ctx(c) || !workspace || !hoisting || !masks || !streams) return fail(MHE_ERR_ARG, "invalid argument");
    {
        std::lock_guard<std::mutex> g(c->mu);
        *workspace = *hoisting = 0;
        for (auto &kv : c->ws)
        {
            *workspace += kv.second.bytes;
            *hoisting += kv.second.hoist_bytes;
        }
        *streams = (int)c->ws.size();
    }
    std::lock_guard<std::mutex> g(c->mask_mu);
    *masks = (uint64_t)c->masks.size() * c->K * c->n * sizeof(u64);
    return MHE_OK;
}

MHE_EXPORT int mhe_kernel_time(mhe_ctx *c, int kernel, double *total_ms, int *launches)
{
    if (!valid_ctx(c) || kernel < 0 || kernel > 1 || !total_ms || !launches) return fail(MHE_ERR_ARG, "invalid argument");
    std::lock_guard<std::mutex> g(c->mu);
    double ms = 0;
    int cnt = 0;
    for (auto &kv : c->ws)
    {
        Workspace &w = kv.second;
        for (size_t i = 0; i < w.ev_used[kernel]; i++)
        {
            float t = 0;
            HIP_TRY(hipEventSynchronize(w.ev[kernel][i].second));
            HIP_TRY(hipEventElapsedTime(&t, w.ev[kernel][i].first, w.ev[kernel][i].second));
            ms += t;
            cnt++;
        }
        w.ev_used[kernel] = 0;
    }
    *total_ms = ms;
    *launches = cnt;
    return MHE_OK;
}

MHE_EXPORT int mhe_stream_create(mhe_ctx *c, void **stream)
{
    if (!valid_ctx(c) || !stream) return fail(MHE_ERR_ARG, "invalid argument");
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s;
    HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = s;
    return MHE_OK;
}

MHE_EXPORT int mhe_stream_destroy(mhe_ctx *c, void *stream)
{
    if (!valid_ctx(c)) return fail(MHE_ERR_ARG, "invalid argument");
    {
        std::lock_guard<std::mutex> g(c->mu);
        auto it = c->ws.find(S(stream));
        if (it != c->ws.end())
        {
            (void)hipStreamSynchronize(S(stream));
            if (it->second.base) (void)hipFree(it->second.base);
            if (it->second.hoist_base) (void)hipFree(it->second.hoist_base);
            if (it->second.flags) (void)hipFree(it->second.flags);
            for (auto &v : it->second.ev)
                for (auto &e : v)
                {
                    (void)hipEventDestroy(e.first);
                    (void)hipEventDestroy(e.second);
                }
            c->ws.erase(it);
        }
    }
    HIP_TRY(hipStreamDestroy(S(stream)));
    return MHE_OK;
}

MHE_EXPORT int mhe_stream_sync(mhe_ctx *c, void *stream)
{
    if (!valid_ctx(c)) return fail(MHE_ERR_ARG, "invalid argument");
    HIP_TRY(hipStreamSynchronize(S(stream)));
    return MHE_OK;
}

MHE_EXPORT int mhe_op_counts(mhe_ctx *c, int kind, uint64_t *counts, int levels, int reset)
{
    if (!valid_ctx(c)) return fail(MHE_ERR_ARG, "context is not valid");
    if (kind < 0 || kind >= MHE_OPK_KINDS || !counts || levels < 1) return fail(MHE_ERR_ARG, "invalid argument");
    for (int l = 0; l < levels; l++)
        counts[l] = l < MHE_OPK_LEVELS ? (reset ? c->opc[kind][l].exchange(0) : c->opc[kind][l].load()) : 0;
    if (reset)
        for (int l = levels; l < MHE_OPK_LEVELS; l++) c->opc[kind][l].store(0);
    return MHE_OK;
}

MHE_EXPORT int mhe_key_traffic(mhe_ctx *c, uint64_t *bytes, int reset)
{
    if (!valid_ctx(c) || !bytes) return fail(MHE_ERR_ARG, "invalid argument");
    *bytes = reset ? c->key_bytes.exchange(0) : c->key_bytes.load();
    return MHE_OK;
}

// Format 1 (doubles): prepare (dir 1) or unprepare (dir 0) the limb slots of a key in place: a slot
// of a prime below 2^51 holds its residues as doubles (-0.0 for zero, so every word is >=
// KEY_PREP_MIN); other slots keep SEAL's layout.  blockIdx.y: digit * 2 * key_limbs + poly *
// key_limbs + limb.
__global__ void k_key_pack(u64 *__restrict__ key, const unsigned char *__restrict__ packed, int key_limbs, int log_n,
                           int dir)
{
    const size_t n = (size_t)1 << log_n;
    const int slot = blockIdx.y;
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n || !packed[slot % key_limbs]) return;
    u64 *d = key + (size_t)slot * n;
    const u64 v = d[i];
    d[i] = dir ? (v ? (u64)__double_as_longlong((double)v) : 0x8000000000000000ull) : key_word_u(v);
}

// Format 2 (48-bit planes): pack (dir 1) or unpack (dir 0) the slots of one digit: src is a copy of
// the digit's 2 x key_limbs slots, dst the key's.  A slot of a prime below 2^48: a 32-bit plane [n]
// then a 16-bit plane [n] (natural order) and KEY_PACK_TAG in the last word; other slots copied.
__global__ void k_key_pack48(const u64 *__restrict__ src, u64 *__restrict__ dst, const unsigned char *__restrict__ packed,
                             int key_limbs, int log_n, int dir)
{
    const size_t n = (size_t)1 << log_n;
    const int slot = blockIdx.y; // poly * key_limbs + limb
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const u64 *s = src + (size_t)slot * n;
    u64 *d = dst + (size_t)slot * n;
    if (!packed[slot % key_limbs])
    {
        d[i] = s[i];
        return;
    }
    if (dir)
    {
        const u64 v = s[i];
        reinterpret_cast<u32 *>(d)[i] = (u32)v;
        reinterpret_cast<unsigned short *>(reinterpret_cast<u32 *>(d) + n)[i] = (unsigned short)(v >> 32);
        if (i == n - 1) d[n - 1] = KEY_PACK_TAG; // in the slot's unused last quarter
    }
    else
    {
        const u32 lo = reinterpret_cast<const u32 *>(s)[i];
        const unsigned short hi = reinterpret_cast<const unsigned short *>(reinterpret_cast<const u32 *>(s) + n)[i];
        d[i] = (u64)lo | ((u64)hi << 32);
    }
}

static int key_pack_run(mhe_ctx *c, u64 *key, int digits, int key_limbs, int dir, int fmt, hipStream_t st)
{
    const size_t n = c->n, slots1 = 2 * (size_t)key_limbs;
    std::vector<unsigned char> pk(key_limbs);
    for (int l = 0; l < key_limbs; l++) pk[l] = key_limb_packed(c, l, key_limbs, fmt) ? 1 : 0;
    HIP_TRY(hipSetDevice(c->device));
    u64 *tmp = nullptr; // format 2: one digit's copy, then the limb table
    const size_t tmp_words = fmt == 2 ? slots1 * n : 0;
    if (hipMalloc(&tmp, tmp_words * sizeof(u64) + 256 + (size_t)key_limbs) != hipSuccess)
        return fail(MHE_ERR_MEMORY, "key prepare: scratch allocation failed");
    unsigned char *pkd = reinterpret_cast<unsigned char *>(tmp + tmp_words);
    int rc = MHE_OK;
    if (hipMemcpyAsync(pkd, pk.data(), key_limbs, hipMemcpyHostToDevice, st) != hipSuccess) rc = fail(MHE_ERR_DEVICE, "key prepare: copy");
    if (fmt == 2)
    {
        for (int J = 0; J < digits && rc == MHE_OK; J++)
        {
            u64 *dg = key + (size_t)J * slots1 * n;
            if (hipMemcpyAsync(tmp, dg, slots1 * n * sizeof(u64), hipMemcpyDeviceToDevice, st) != hipSuccess)
            {
                rc = fail(MHE_ERR_DEVICE, "key prepare: copy");
                break;
            }
            hipLaunchKernelGGL(k_key_pack48, dim3((unsigned)((n + 255) / 256), (unsigned)slots1), dim3(256), 0, st, tmp,
                               dg, pkd, key_limbs, c->log_n, dir);
            if (hipGetLastError() != hipSuccess) rc = fail(MHE_ERR_DEVICE, "key prepare: launch");
        }
    }
    else
    {
        // grid.y is at most 65535 slots per launch: whole groups of key_limbs slots each, so the
        // kernel's slot % key_limbs stays the limb
        const size_t slots = slots1 * (size_t)digits, per = (65535 / (size_t)key_limbs) * (size_t)key_limbs;
        for (size_t s0 = 0; s0 < slots && rc == MHE_OK;)
        {
            const size_t cnt = std::min(per, slots - s0);
            hipLaunchKernelGGL(k_key_pack, dim3((unsigned)((n + 255) / 256), (unsigned)cnt), dim3(256), 0, st,
                               key + s0 * n, pkd, key_limbs, c->log_n, dir);
            if (hipGetLastError() != hipSuccess) rc = fail(MHE_ERR_DEVICE, "key prepare: launch");
            s0 += cnt;
        }
    }
    // the scratch is freed only after the stream has used it
    if (hipStreamSynchronize(st) != hipSuccess && rc == MHE_OK) rc = fail(MHE_ERR_DEVICE, "key prepare: sync");
    (void)hipFree(tmp);
    return rc;
}

// the format mhe_key_prepare makes: MHE_KEY_FMT=2 chooses the 48-bit planes, default doubles
static int default_key_format()
{
    static const int f = [] {
        const char *e = getenv("MHE_KEY_FMT");
        return (e && atoi(e) == 2) ? 2 : 1;
    }();
    return f;
}

MHE_EXPORT int mhe_key_prepare_as(mhe_ctx *c, uint64_t *key, int digits, int key_limbs, int format, void *s)
{
    if (!valid_ctx(c) || !key || digits < 1 || key_limbs < 2 || key_limbs > c->K || digits > key_limbs - 1 ||
        (format != MHE_KEY_FMT_DOUBLE && format != MHE_KEY_FMT_PACK48))
        return fail(MHE_ERR_ARG, "invalid argument");
    int tagged = 0;
    int r = key_tagged(c, key, key_limbs, S(s), &tagged);
    if (r) return r;
    if (tagged) return fail(MHE_ERR_ARG, "key prepare: key is already prepared");
    return key_pack_run(c, key, digits, key_limbs, 1, format, S(s));
}

MHE_EXPORT int mhe_key_prepare(mhe_ctx *c, uint64_t *key, int digits, int key_limbs, void *s)
{
    return mhe_key_prepare_as(c, key, digits, key_limbs, default_key_format(), s);
}

MHE_EXPORT int mhe_key_unprepare(mhe_ctx *c, uint64_t *key, int digits, int key_limbs, void *s)
{
    if (!valid_ctx(c) || !key || digits < 1 || key_limbs < 2 || key_limbs > c->K || digits > key_limbs - 1)
        return fail(MHE_ERR_ARG, "invalid argument");
    int tagged = 0;
    int r = key_tagged(c, key, key_limbs, S(s), &tagged);
    if (r) return r;
    if (!tagged) return fail(MHE_ERR_ARG, "key unprepare: key is not prepared");
    return key_pack_run(c, key, digits, key_limbs, 0, tagged, S(s));
}

MHE_EXPORT int mhe_key_traffic_prepared(mhe_ctx *c, uint64_t *bytes, int reset)
{
    if (!valid_ctx(c) || !bytes) return fail(MHE_ERR_ARG, "invalid argument");
    *bytes = reset ? c->key_bytes_prep.exchange(0) : c->key_bytes_prep.load();
    return MHE_OK;
}

MHE_EXPORT int mhe_key_is_prepared(mhe_ctx *c, const uint64_t *key, int key_limbs, int *prepared, void *s)
{
    if (!valid_ctx(c) || !key || !prepared || key_limbs < 2 || key_limbs > c->K) return fail(MHE_ERR_ARG, "invalid argument");
    return key_tagged(c, key, key_limbs, S(s), prepared);
}

MHE_EXPORT int mhe_stream_wait(mhe_ctx *c, void *waiter, void *waitee)
{
    // device-side ordering: work enqueued on `waiter` after this call starts after everything
    // enqueued on `waitee` before it (no host blocking)
    if (!valid_ctx(c)) return fail(MHE_ERR_ARG, "invalid argument");
    if (waiter == waitee) return MHE_OK;
    HIP_TRY(hipSetDevice(c->device)); // the event must belong to the engine's device
    // A ring of events per thread and device, re-recorded in turn: a stream wait captures the
    // event's state at the call, so a later record of the same event does not move it.  (Creating
    // and destroying an event per wait cost host time, and destroying one still pending crashed
    // under rocprofv3's API tracing in multi-stream runs, profiles/r04d.)
    struct Ring
    {
        int device = -1;
        hipEvent_t ev[64] = {};
        unsigned next = 0;
    };
    static thread_local Ring ring[8];
    Ring &r = ring[c->device & 7];
    if (r.device != c->device)
    {
        for (auto &e : r.ev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        r.device = c->device;
    }
    hipEvent_t ev = r.ev[r.next++ & 63];
    hipError_t e = hipEventRecord(ev, S(waitee));
    if (e == hipSuccess) e = hipStreamWaitEvent(S(waiter), ev, 0);
    if (e != hipSuccess) return fail(MHE_ERR_DEVICE, hipGetErrorString(e));
    return MHE_OK;
}

static int check_poly_args(mhe_ctx *c, const void *a, int polys, int limbs)
{
    if (!valid_ctx(c)) return fail(MHE_ERR_ARG, "context is not valid");
    if (!a || polys < 1 || limbs < 1 || limbs > c->K) return fail(MHE_ERR_ARG, "invalid polynomial arguments");
    return MHE_OK;
}

MHE_EXPORT int mhe_ntt_forward(mhe_ctx *c, uint64_t *data, int polys, int limbs, int lazy, void *stream)
{
    TR("data", data, (size_t)polys * limbs * ((size_t)1 << c->log_n));
    TRC(0, 0, 0, 0);
    int r = check_poly_args(c, data, polys, limbs);
    if (r) return r;
    return run_ntt_fwd(c, data, data, polys, limbs, lazy ? 0 : 1, S(stream));
}

MHE_EXPORT int mhe_ntt_inverse(mhe_ctx *c, uint64_t *data, int polys, int limbs, int lazy, void *stream)
{
    TR("data", data, (size_t)polys * limbs * ((size_t)1 << c->log_n));
    TRC(0, 0, 0, 0);
    int r = check_poly_args(c, data, polys, limbs);
    if (r) return r;
    return run_ntt_inv(c, data, data, polys, limbs, lazy ? 0 : 1, S(stream));
}

static int launch_addsub(mhe_ctx *c, const u64 *a, const u64 *b, u64 *out, int polys, int limbs, int op, void *st)
{
    int r = check_poly_args(c, a, polys, limbs);
    if (r) return r;
    if (!out || (op < 2 && !b)) return fail(MHE_ERR_ARG, "invalid polynomial arguments");
    {
        mhe_launch l{};
        l.kind = MHE_LK_ADDSUB;
        l.op = op;
        l.a = a;
        l.b = b;
        l.out = out;
        l.polys = polys;
        l.limbs = limbs;
        l.stream = st;
        if (hooked(c, l)) return l.rc;
    }
    count_op(c, MHE_OPK_ADDSUB, limbs, (unsigned long long)polys);
    size_t total2 = ((size_t)polys * limbs << c->log_n) / 2;
    hipLaunchKernelGGL(k_addsub, ELEM_GRID(total2), dim3(256), 0, S(st), a, b, out, c->primes, limbs, c->log_n,
                       total2, op);
    HIP_LAUNCH_CHECK();
    return MHE_OK;
}

MHE_EXPORT int mhe_add(mhe_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, int polys, int limbs, void *s)
{
    TR("out", out, (size_t)polys * limbs * ((size_t)1 << c->log_n)); TR("a", a, (size_t)polys * limbs * ((size_t)1 << c->log_n)); TR("b", b, (size_t)polys * limbs * ((size_t)1 << c->log_n));
    TRC(0, 0, 0, 0);
    return launch_addsub(c, a, b, out, polys, limbs, 0, s);
}

MHE_EXPORT int mhe_sub(mhe_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, int polys, int limbs, void *s)
{
    TR("out", out, (size_t)polys * limbs * ((size_t)1 << c->log_n)); TR("a", a, (size_t)polys * limbs * ((size_t)1 << c->log_n)); TR("b", b, (size_t)polys * limbs * ((size_t)1 << c->log_n));
    TRC(0, 0, 0, 0);
    return launch_addsub(c, a, b, out, polys, limbs, 1, s);
}

MHE_EXPORT int mhe_negate(mhe_ctx *c, const uint64_t *a, uint64_t *out, int polys, int limbs, void *s)
{
    TR("out", out, (size_t)polys * limbs * ((size_t)1 << c->log_n)); TR("a", a, (size_t)polys * limbs * ((size_t)1 << c->log_n));
    TRC(0, 0, 0, 0);
    return launch_addsub(c, a, nullptr, out, polys, limbs, 2, s);
}

MHE_EXPORT int mhe_multiply_plain(mhe_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, int polys,
                                  int limbs, void *s)
{
    TR("out", out, (size_t)polys * limbs * ((size_t)1 << c->log_n)); TR("a", a, (size_t)polys * limbs * ((size_t)1 << c->log_n)); TR("b", b, (size_t)limbs * ((size_t)1 << c->log_n));
    TRC(0, 0, 0, 0);
    int r = check_poly_args(c, a, polys, limbs);
    if (r) return r;
    if (!b || !out) return fail(MHE_ERR_ARG, "invalid polynomial arguments");
    {
        mhe_launch l{};
        l.kind = MHE_LK_MULPLAIN;
        l.a = a;
        l.b = b;
        l.out = out;
        l.polys = polys;
        l.limbs = limbs;
        l.stream = s;
        if (hooked(c, l)) return l.rc;
    }
    count_op(c, MHE_OPK_MULPLAIN, limbs, (unsigned long long)polys);
    size_t total2 = ((size_t)polys * limbs << c->log_n) / 2;
    hipLaunchKernelGGL(k_mulplain, ELEM_GRID(total2), dim3(256), 0, S(s), a, b, out, c->primes, limbs, c->log_n,
                       total2, c->nm.fp ? 1 : 0);
    HIP_LAUNCH_CHECK();
    return MHE_OK;
}

MHE_EXPORT int mhe_multiply_plain_add(mhe_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *acc, int polys,
                                      int limbs, void *s)
{
    int r = check_poly_args(c, a, polys, limbs);
    if (r) return r;
    if (!b || !acc) return fail(MHE_ERR_ARG, "invalid polynomial arguments");
    {
        mhe_launch l{};
        l.kind = MHE_LK_MULPLAIN_ADD;
        l.a = a;
        l.b = b;
        l.out = acc;
        l.polys = polys;
        l.limbs = limbs;
        l.stream = s;
        if (hooked(c, l)) return l.rc;
    }
    count_op(c, MHE_OPK_MULPLAIN, limbs, (unsigned long long)polys);
    count_op(c, MHE_OPK_ADDSUB, limbs, (unsigned long long)polys);
    size_t total2 = ((size_t)polys * limbs << c->log_n) / 2;
    hipLaunchKernelGGL(k_mulplain_add, ELEM_GRID(total2), dim3(256), 0, S(s), a, b, acc, c->primes, limbs, c->log_n,
                       total2, c->nm.fp ? 1 : 0);
    HIP_LAUNCH_CHECK();
    return MHE_OK;
}

MHE_EXPORT int mhe_multiply_plain_sum(mhe_ctx *c, int count, const uint64_t *const *a, const uint64_t *const *b,
                                      uint64_t *out, int accumulate, int polys, int limbs, void *s)
{
    if (count < 1 || !a || !b || !out) return fail(MHE_ERR_ARG, "invalid polynomial arguments");
    for (int k = 0; k < count; k++)
    {
        int r = check_poly_args(c, a[k], polys, limbs);
        if (r) return r;
        if (!b[k]) return fail(MHE_ERR_ARG, "invalid polynomial arguments");
    }
    count_op(c, MHE_OPK_MULPLAIN, limbs, (unsigned long long)polys * count);
    count_op(c, MHE_OPK_ADDSUB, limbs, (unsigned long long)polys * (count - 1 + (accumulate ? 1 : 0)));
    const size_t total2 = ((size_t)polys * limbs << c->log_n) / 2;
    for (int k0 = 0; k0 < count; k0 += MHE_SUM_TERMS)
    {
        const int cnt = std::min(MHE_SUM_TERMS, count - k0);
        SumPtrs P{};
        for (int k = 0; k < cnt; k++)
        {
            P.a[k] = a[k0 + k];
            P.b[k] = b[k0 + k];
        }
        hipLaunchKernelGGL(k_mulplain_sum, ELEM_GRID(total2), dim3(256), 0, S(s), P, cnt, out,
                           (accumulate || k0 > 0) ? 1 : 0, c->primes, limbs, c->log_n, total2, c->nm.fp ? 1 : 0);
        HIP_LAUNCH_CHECK();
    }
    return MHE_OK;
}

static int launch_scalar(mhe_ctx *c, const u64 *a, const u64 *scalars, u64 *out, int polys, int limbs, int op,
                         void *s)
{
    int r = check_poly_args(c, a, polys, limbs);
    if (r) return r;
    if (!scalars || !out) return fail(MHE_ERR_ARG, "invalid polynomial arguments");
    ScalarTab t;
    for (int l = 0; l < limbs; l++)
    {
        if (scalars[l] >= c->q[l]) return fail(MHE_ERR_ARG, "scalar must be less than modulus");
        t.v[l] = scalars[l];
        t.vq[l] = host::shoup(scalars[l], c->q[l]);
    }
    {
        mhe_launch hl{};
        hl.kind = MHE_LK_SCALAR;
        hl.op = op;
        hl.a = a;
        hl.out = out;
        hl.polys = polys;
        hl.limbs = limbs;
        hl.stream = s;
        for (int l = 0; l < limbs; l++) hl.scalars[l] = scalars[l];
        if (hooked(c, hl)) return hl.rc;
    }
    count_op(c, MHE_OPK_SCALAR, limbs, (unsigned long long)polys);
    size_t total2 = ((size_t)polys * limbs << c->log_n) / 2;
    hipLaunchKernelGGL(k_scalar, ELEM_GRID(total2), dim3(256), 0, S(s), a, out, c->primes, t, limbs, c->log_n,
                       total2, op);
    HIP_LAUNCH_CHECK();
    return MHE_OK;
}

MHE_EXPORT int mhe_multiply_scalar(mhe_ctx *c, const uint64_t *a, const uint64_t *scalars, uint64_t *out, int polys,
                                   int limbs, void *s)
{
    TR("out", out, (size_t)polys * limbs * ((size_t)1 << c->log_n)); TR("a", a, (size_t)polys * limbs * ((size_t)1 << c->log_n));
    TRC(0, 0, 0, 0);
    return launch_scalar(c, a, scalars, out, polys, limbs, 0, s);
}

MHE_EXPORT int mhe_add_scalar(mhe_ctx *c, const uint64_t *a, const uint64_t *scalars, uint64_t *out, int polys,
                              int limbs, void *s)
{
    TR("out", out, (size_t)polys * limbs * ((size_t)1 << c->log_n)); TR("a", a, (size_t)polys * limbs * ((size_t)1 << c->log_n));
    TRC(0, 0, 0, 0);
    return launch_scalar(c, a, scalars, out, polys, limbs, 1, s);
}

MHE_EXPORT int mhe_set_scalar(mhe_ctx *c, const uint64_t *scalars, uint64_t *out, int polys, int limbs, void *s)
{
    return launch_scalar(c, out, scalars, out, polys, limbs, 2, s);
}

static int launch_tensor(mhe_ctx *c, const u64 *a, const u64 *b, u64 *out3, int L, int square, hipStream_t st)
{
    count_op(c, MHE_OPK_TENSOR, L, 1);
    size_t total2 = ((size_t)L << c->log_n) / 2;
    hipLaunchKernelGGL(k_tensor, ELEM_GRID(total2), dim3(256), 0, st, a, b, out3, c->primes, L, c->log_n, total2,
                       square, c->nm.fp ? 1 : 0);
    HIP_LAUNCH_CHECK();
    return MHE_OK;
}

MHE_EXPORT int mhe_ct_multiply(mhe_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out3, int limbs, void *s)
{
    TR("out3", out3, (size_t)3 * limbs * ((size_t)1 << c->log_n)); TR("a", a, (size_t)2 * limbs * ((size_t)1 << c->log_n)); TR("b", b, (size_t)2 * limbs * ((size_t)1 << c->log_n));
    TRC(0, 0, 0, 0);
    int r = check_poly_args(c, a, 2, limbs);
    if (r) return r;
    if (!b || !out3) return fail(MHE_ERR_ARG, "invalid polynomial arguments");
    mhe_launch l{};
    l.kind = MHE_LK_TENSOR;
    l.a = a;
    l.b = b;
    l.out = out3;
    l.polys = 2;
    l.limbs = limbs;
    l.stream = s;
    if (hooked(c, l)) return l.rc;
    return launch_tensor(c, a, b, out3, limbs, 0, S(s));
}

MHE_EXPORT int mhe_ct_square(mhe_ctx *c, const uint64_t *a, uint64_t *out3, int limbs, void *s)
{
    TR("out3", out3, (size_t)3 * limbs * ((size_t)1 << c->log_n)); TR("a", a, (size_t)2 * limbs * ((size_t)1 << c->log_n));
    TRC(0, 0, 0, 0);
    int r = check_poly_args(c, a, 2, limbs);
    if (r) return r;
    if (!out3) return fail(MHE_ERR_ARG, "invalid polynomial arguments");
    mhe_launch l{};
    l.kind = MHE_LK_TENSOR;
    l.op = 1;
    l.a = a;
    l.b = a;
    l.out = out3;
    l.polys = 2;
    l.limbs = limbs;
    l.stream = s;
    if (hooked(c, l)) return l.rc;
    return launch_tensor(c, a, a, out3, limbs, 1, S(s));
}

MHE_EXPORT int mhe_switch_key(mhe_ctx *c, uint64_t *ct, const uint64_t *target, const uint64_t *key, int key_limbs,
                              int limbs, void *s)
{
    TR("ct", ct, (size_t)2 * limbs * ((size_t)1 << c->log_n)); TR("target", target, (size_t)limbs * ((size_t)1 << c->log_n)); TR("key", key, (size_t)limbs * 2 * key_limbs * ((size_t)1 << c->log_n));
    TRC(0, 0, 0, 0);
    int r = check_limbs(c, limbs, 1);
    if (r) return r;
    if (!ct || !target || !key) return fail(MHE_ERR_ARG, "target_iter");
    return run_switch_key(c, ct, target, key, key_limbs, limbs, S(s));
}

MHE_EXPORT int mhe_relinearize(mhe_ctx *c, uint64_t *ct3, const uint64_t *key, int key_limbs, int limbs, void *s)
{
    TR("ct3", ct3, (size_t)3 * limbs * ((size_t)1 << c->log_n)); TR("key", key, (size_t)limbs * 2 * key_limbs * ((size_t)1 << c->log_n));
    TRC(0, 0, 0, 0);
    int r = check_limbs(c, limbs, 1);
    if (r) return r;
    if (!ct3 || !key) return fail(MHE_ERR_ARG, "relin_keys is not valid for encryption parameters");
    return run_switch_key(c, ct3, ct3 + ((size_t)2 * limbs << c->log_n), key, key_limbs, limbs, S(s));
}

static int launch_galois(mhe_ctx *c, const u64 *in, u32 elt, u64 *out, int polys, int limbs, hipStream_t st)
{
    if (!(elt & 1) || elt >= 2 * c->n) return fail(MHE_ERR_ARG, "Galois element is not valid");
    count_op(c, MHE_OPK_GALOIS, limbs, (unsigned long long)polys);
    size_t total = (size_t)polys * limbs << c->log_n;
    hipLaunchKernelGGL(k_galois, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, in, out, elt, c->log_n,
                       total);
    HIP_LAUNCH_CHECK();
    return MHE_OK;
}

MHE_EXPORT int mhe_permute_galois(mhe_ctx *c, const uint64_t *in, uint32_t elt, uint64_t *out, int polys, int limbs,
                                  void *s)
{
    TR("out", out, (size_t)polys * limbs * ((size_t)1 << c->log_n)); TR("in", in, (size_t)polys * limbs * ((size_t)1 << c->log_n));
    TRC(0, 0, 0, 0);
    int r = check_poly_args(c, in, polys, limbs);
    if (r) return r;
    if (!out || out == in) return fail(MHE_ERR_ARG, "result cannot point to the same value as operand");
    return launch_galois(c, in, elt, out, polys, limbs, S(s));
}

MHE_EXPORT int mhe_apply_galois(mhe_ctx *c, uint64_t *ct, uint32_t elt, const uint64_t *key, int key_limbs, int limbs,
                                void *s)
{
    TR("ct", ct, (size_t)2 * limbs * ((size_t)1 << c->log_n)); TR("key", key, (size_t)limbs * 2 * key_limbs * ((size_t)1 << c->log_n));
    TRC(0, 0, 0, 0);
    int r = check_limbs(c, limbs, 1);
    if (r) return r;
    if (!ct || !key) return fail(MHE_ERR_ARG, "Galois key not present");
    hipStream_t st = S(s);
    Workspace *w;
    r = get_ws(c, st, c->K - 1, &w);
    if (r) return r;
    const size_t ps = (size_t)limbs << c->log_n;
    // evaluator.cpp:2193-2214: c0 <- perm(c0) (via tmp), tmp <- perm(c1), c1 <- 0, then KS(tmp)
    r = launch_galois(c, ct, elt, w->tmp, 1, limbs, st);
    if (r) return r;
    HIP_TRY(mhe_internal_copy_d2d(ct, w->tmp, ps * sizeof(u64), st));
    r = launch_galois(c, ct + ps, elt, w->tmp, 1, limbs, st);
    if (r) return r;
    if (!c->galois_fused) HIP_TRY(hipMemsetAsync(ct + ps, 0, ps * sizeof(u64), st));
    return run_switch_key(c, ct, w->tmp, key, key_limbs, limbs, st, nullptr, c->galois_fused); // c1 <- 0 + KS_1
}

MHE_EXPORT int mhe_apply_galois_to(mhe_ctx *c, const uint64_t *in, uint64_t *out, uint32_t elt, const uint64_t *key,
                                   int key_limbs, int limbs, void *s)
{
    TR("out", out, (size_t)2 * limbs * ((size_t)1 << c->log_n)); TR("in", in, (size_t)2 * limbs * ((size_t)1 << c->log_n));
    TRC(0, 0, 0, 0);
    int r = check_limbs(c, limbs, 1);
    if (r) return r;
    if (!in || !out || !key) return fail(MHE_ERR_ARG, "Galois key not present");
    if (in == out) return fail(MHE_ERR_ARG, "result cannot point to the same value as operand");
    hipStream_t st = S(s);
    Workspace *w;
    r = get_ws(c, st, c->K - 1, &w);
    if (r) return r;
    const size_t ps = (size_t)limbs << c->log_n;
    // evaluator.cpp:2193-2214: out0 <- perm(c0), out1 <- perm(c1) (one launch), then the key switch
    // of out1 with out0 += KS_0 and out1 = KS_1 (SEAL zeroes c1 and adds; same words)
    if (c->galois_fused)
    {
        r = launch_galois(c, in, elt, out, 2, limbs, st);
        if (r) return r;
        return run_switch_key(c, out, out + ps, key, key_limbs, limbs, st, nullptr, 1);
    }
    r = launch_galois(c, in, elt, out, 1, limbs, st);
    if (r) return r;
    r = launch_galois(c, in + ps, elt, w->tmp, 1, limbs, st);
    if (r) return r;
    HIP_TRY(hipMemsetAsync(out + ps, 0, ps * sizeof(u64), st));
    return run_switch_key(c, out, w->tmp, key, key_limbs, limbs, st);
}

// ------------------------------------------------------------------ hoisted rotations (hoist.h)
// The ModUp buffers of up to `entries` hoisted inputs on stream st ([K][K-1][n] each: every level),
// the key products of up to MHE_MAXB * MHE_HOIST_R of their rotations and the inputs' flags.
static int get_hoist(mhe_ctx *c, hipStream_t st, int entries, int ws_entries, int L, Workspace **out)
{
    Workspace *w;
    int r = get_ws(c, st, c->K - 1, &w, std::max(entries, ws_entries));
    if (r) return r;
    std::lock_guard<std::mutex> g(w->mu);
    // per input [L+1][L][n] (the pass's level), the key products of up to MHE_MAXB * MHE_HOIST_R
    // rotations at that level; grown (after draining the stream) when a pass needs more
    if (w->hoist_entries < entries || w->hoist_limbs < L)
    {
        const int E = std::max(entries, w->hoist_entries), HL = std::max(L, w->hoist_limbs);
        HIP_TRY(hipSetDevice(c->device));
        if (w->hoist_base)
        {
            HIP_TRY(hipStreamSynchronize(st));
            HIP_TRY(hipFree(w->hoist_base));
        }
        w->hoist_base = nullptr;
        w->hoist_entries = 0;
        w->hoist_limbs = 0;
        w->hoist_bytes = 0;
        const size_t per = (size_t)(HL + 1) * HL * c->n, pacc = (size_t)2 * (HL + 1) * c->n;
        const int na = MHE_MAXB * MHE_HOIST_R;
        const size_t bytes = ((size_t)E * per + (size_t)na * pacc) * sizeof(u64);
        if (injected_alloc_failure(c) || scratch_alloc((void **)&w->hoist_base, bytes) != hipSuccess)
        {
            w->hoist_base = nullptr;
            return fail(MHE_ERR_MEMORY, "workspace allocation failed");
        }
        for (int i = 0; i < E; i++) w->hoist[i] = w->hoist_base + (size_t)i * per;
        for (int i = 0; i < na; i++) w->hacc[i] = w->hoist_base + (size_t)E * per + (size_t)i * pacc;
        w->hoist_entries = E;
        w->hoist_limbs = HL;
        w->hoist_bytes = bytes;
    }
    if (!w->flags && hipMalloc(&w->flags, MHE_MAXB * sizeof(int)) != hipSuccess)
        return fail(MHE_ERR_MEMORY, "workspace allocation failed");
    *out = w;
    return MHE_OK;
}

// M^g = NTT of Galois element g's negation mask under every prime of the context, [K][n]
// canonical; built once per element on stream st (which then waits for it: other streams use the
// table without an event).
static int get_mask(mhe_ctx *c, u32 elt, hipStream_t st, const u64 **out)
{
    std::lock_guard<std::mutex> g(c->mask_mu);
    auto it = c->masks.find(elt);
    if (it != c->masks.end())
    {
        *out = it->second;
        return MHE_OK;
    }
    u64 *m = nullptr;
    const size_t total = (size_t)c->K * c->n;
    HIP_TRY(hipSetDevice(c->device));
    if (hipMalloc(&m, total * sizeof(u64)) != hipSuccess) return fail(MHE_ERR_MEMORY, "Galois mask allocation failed");
    hipLaunchKernelGGL(k_negmask, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, m, elt, c->K, c->log_n);
    JobFwdPlain j;
    j.src = m;
    j.dst = m;
    j.primes = c->primes;
    j.tw = c->tw;
    j.limbs = c->K;
    j.log_n = c->log_n;
    j.mode = 0;
    fwd_col(j, c->log_n, c->K, c->nm, st);
    j.mode = 1;
    fwd_row(j, c->log_n, c->K, c->nm, st);
    HIP_LAUNCH_CHECK();
    HIP_TRY(hipStreamSynchronize(st));
    c->masks[elt] = m;
    *out = m;
    return MHE_OK;
}

static void launch_hoist_mac(int R, dim3 grid, hipStream_t st, const HoistPtrs &hp, const PrimeDev *primes,
                             const TwF *cm, int L, int K, int log_n)
{
    switch (R)
    {
#define HM(r) case r: hipLaunchKernelGGL((k_ks_hoist_mac<r>), grid, dim3(256), 0, st, hp, primes, cm, L, K, log_n); break;
        HM(1) HM(2) HM(3) HM(4) HM(5) HM(6) HM(7) HM(8)
#undef HM
    }
}
static void launch_hoist_mac_sh(int R, dim3 grid, hipStream_t st, const HoistShared &hs, const PrimeDev *primes,
                                const TwF *cm, int L, int K, int log_n)
{
    switch (R)
    {
#define HM(r) case r: hipLaunchKernelGGL((k_ks_hoist_mac_sh<r>), grid, dim3(1024), 0, st, hs, primes, cm, L, K, log_n); break;
        HM(1) HM(2) HM(3) HM(4) HM(5) HM(6) HM(7) HM(8)
#undef HM
    }
}

static bool hoist_ok(const mhe_ctx *c)
{
    return c->ks_hoist && c->ks_fused && c->galois_fused && c->ks_colgroups > 0 && c->nm.fp == 1 && c->nm_ks.fp == 1 &&
           c->cmodf;
}

// counts words that differ between a and b (mhe_ctx_set_hoist's check); first[0] = lowest index
__global__ void k_cmp_words(const u64 *__restrict__ a, const u64 *__restrict__ b, size_t total,
                            unsigned long long *bad)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= total || a[i] == b[i]) return;
    atomicAdd(bad, 1ull);
    atomicMin(bad + 1, (unsigned long long)i);
}

// The check of a hoisted pass: every rotation again by SEAL's order (permutation, then the classic
// key switch of the permuted c1) into scratch, compared word for word with the hoisted output.
static int hoist_check_pass(mhe_ctx *c, const u64 *const *in, int count, const int *ent_in, u64 *const *out,
                            const u32 *elts, const u64 *const *keys, const int *key_limbs, int L, hipStream_t st,
                            const int *flags)
{
    const size_t ps = (size_t)L * c->n;
    u64 *tmp = nullptr;
    unsigned long long *cnt = nullptr;
    HIP_TRY(hipSetDevice(c->device));
    if (hipMalloc(&tmp, (size_t)MHE_MAXB * 2 * ps * sizeof(u64)) != hipSuccess)
        return fail(MHE_ERR_MEMORY, "hoist check: allocation failed");
    if (hipMalloc(&cnt, 2 * MHE_MAXB * sizeof(unsigned long long) + MHE_MAXB * sizeof(int)) != hipSuccess)
    {
        (void)hipFree(tmp);
        return fail(MHE_ERR_MEMORY, "hoist check: allocation failed");
    }
    int *fl = reinterpret_cast<int *>(cnt + 2 * MHE_MAXB);
    int r = MHE_OK;
    for (int i0 = 0; i0 < count && r == MHE_OK; i0 += MHE_MAXB)
    {
        const int B = std::min(MHE_MAXB, count - i0);
        GalPtrs gp{};
        KsJob jobs[MHE_MAXB];
        std::vector<unsigned long long> init(2 * MHE_MAXB);
        for (int e = 0; e < B; e++)
        {
            const int i = i0 + e;
            u64 *t = tmp + (size_t)e * 2 * ps;
            gp.in[e] = in[ent_in[i]];
            gp.out[e] = t;
            gp.elt[e] = elts[i];
            jobs[e] = KsJob{ t, t + ps, keys[i], key_limbs[i], nullptr };
            init[2 * e] = 0;
            init[2 * e + 1] = ~0ull;
        }
        HIP_TRY(hipMemcpyAsync(cnt, init.data(), init.size() * sizeof(unsigned long long), hipMemcpyHostToDevice, st));
        for (int e = 0; e < B; e++)
            HIP_TRY(hipMemcpyAsync(fl + e, flags + ent_in[i0 + e], sizeof(int), hipMemcpyDeviceToDevice, st));
        hipLaunchKernelGGL(k_galois_b, dim3((unsigned)((2 * ps + 255) / 256), (unsigned)B), dim3(256), 0, st, gp,
                           c->log_n, 2 * ps);
        HIP_LAUNCH_CHECK();
        if ((r = run_switch_key_batch(c, jobs, B, L, st, 1))) break;
        for (int e = 0; e < B; e++)
            hipLaunchKernelGGL(k_cmp_words, dim3((unsigned)((2 * ps + 255) / 256)), dim3(256), 0, st,
                               tmp + (size_t)e * 2 * ps, out[i0 + e], 2 * ps, cnt + 2 * e);
        HIP_LAUNCH_CHECK();
        std::vector<unsigned long long> got(2 * MHE_MAXB);
        std::vector<int> hf(MHE_MAXB);
        HIP_TRY(hipMemcpyAsync(got.data(), cnt, got.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(hf.data(), fl, MHE_MAXB * sizeof(int), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        for (int e = 0; e < B; e++)
        {
            if (!got[2 * e]) continue;
            c->hoist_bad += got[2 * e];
            const unsigned long long f = got[2 * e + 1];
            fprintf(stderr,
                    "[hoist check] stream %p L %d entry %d/%d (input %d, elt %u, key %p, key_limbs %d, zero flag %d): "
                    "%llu words differ, first at poly %llu limb %llu slot %llu\n",
                    (void *)st, L, i0 + e, count, ent_in[i0 + e], elts[i0 + e], (const void *)keys[i0 + e],
                    key_limbs[i0 + e], hf[e], got[2 * e], f / ps, (f % ps) / c->n, f % c->n);
        }
    }
    (void)hipStreamSynchronize(st);
    (void)hipFree(tmp);
    (void)hipFree(cnt);
    return r;
}

// Rotations of H <= MHE_MAXB inputs at L limbs, entry i rotating input ent_in[i] (index into in)
// by elts[i] into out[i]: ModUp of every input once (INTT -> column pass -> row pass, canonical
// D in the hoist buffers, plus the zero scan), then per chunk of entries the permutation of c0 /
// c1 into out, the hoisted key MAC (hoist.h), the classic ModUp + MAC for flagged inputs only
// (their kernels return at once otherwise), and the ModDown (c1 written).
static int run_galois_hoisted(mhe_ctx *c, const u64 *const *in, int H, int count, const int *ent_in,
                              u64 *const *out, const u32 *elts, const u64 *const *keys, const int *key_limbs, int L,
                              hipStream_t st)
{
    Workspace *w;
    int r = get_hoist(c, st, H, std::min(count, MHE_MAXB), L, &w); // step 3 uses up to MHE_MAXB entry slots
    if (r) return r;
    const int log_n = c->log_n;
    const size_t n = c->n, ps = (size_t)L * n;
    std::vector<const u64 *> masks(count);
    std::vector<u32> elt_inv(count);
    for (int i = 0; i < count; i++)
    {
        if ((r = get_mask(c, elts[i], st, &masks[i]))) return r;
        u64 inv = 0;
        host::invmod(elts[i], 2 * n, inv); // odd: a unit mod 2N
        elt_inv[i] = (u32)inv;
    }
    // 1. ModUp of each input's c1: INTT (evaluator.cpp:2351-2354) into entry slot h's coeff, the zero
    //    scan, the column pass into hoist[h] (64-bit, natural order), the row pass in place
    {
        JobB<JobStrided> j;
        j.per = L;
        for (int h = 0; h < H; h++)
            j.j[h] = JobStrided{ in[h] + ps, w->e[h].coeff, n, n, 0, 1, c->primes, c->itw, log_n, 0 };
        inv_row(j, log_n, H * L, c->nm, st);
        for (int h = 0; h < H; h++)
        {
            j.j[h].src = w->e[h].coeff;
            j.j[h].mode = 1;
        }
        inv_col(j, log_n, H * L, c->nm, st);
        HIP_TRY(hipMemsetAsync(w->flags, 0, MHE_MAXB * sizeof(int), st));
        for (int h = 0; h < H; h++)
            hipLaunchKernelGGL(k_zero_scan, dim3((unsigned)((ps + 255) / 256)), dim3(256), 0, st, w->e[h].coeff, log_n, ps,
                               w->flags + h);
        KsPtrs kp{};
        for (int h = 0; h < H; h++)
        {
            kp.coeff[h] = w->e[h].coeff;
            kp.inter[h] = w->e[h].modup;
        }
        const int IG = c->ks_colgroups < L + 1 ? c->ks_colgroups : L + 1;
        modup_col(kp, H, c->primes, c->tw, L, c->K, log_n, c->nm_ks, 0, L + 1, IG, 0, st);
        auto row = [&](auto brev) {
            JobB<JobModUpRowH<decltype(brev)::value>> rj;
            rj.per = (L + 1) * L;
            for (int h = 0; h < H; h++) rj.j[h] = { w->e[h].modup, w->hoist[h], c->primes, c->tw, L, c->K, log_n };
            fwd_row(rj, log_n, H * (L + 1) * L, c->nm, st);
        };
        if (log_n == 16)
            row(std::true_type{});
        else
            row(std::false_type{});
        HIP_LAUNCH_CHECK();
    }
    // 2. the hoisted key MAC: items of one input and up to MHE_HOIST_R of its rotations (sorted by
    //    key, so the items of images rotated alike list the same keys and share their rows), up to
    //    MHE_MAXB items per launch; rotation i's key products go to w->hacc[i]
    const int pack = (c->ks_pack && c->ks_colgroups > 0) ? 1 : 0;
    {
        std::vector<std::vector<int>> per(H);
        for (int i = 0; i < count; i++) per[ent_in[i]].push_back(i);
        std::vector<std::pair<int, std::vector<int>>> items;
        for (int h = 0; h < H; h++)
        {
            std::stable_sort(per[h].begin(), per[h].end(), [&](int a, int b) { return keys[a] < keys[b]; });
            for (size_t r0 = 0; r0 < per[h].size(); r0 += MHE_HOIST_R)
                items.emplace_back(h, std::vector<int>(per[h].begin() + r0,
                                                       per[h].begin() + std::min(per[h].size(), r0 + MHE_HOIST_R)));
        }
        // items with one key list (the images of a FiberBatch rotated alike): the shared-key kernel,
        // up to MHE_MAXB items per launch; the rest one launch per up to MHE_MAXB items
        std::vector<char> done(items.size(), 0);
        for (size_t z0 = 0; z0 < items.size(); z0++)
        {
            if (done[z0]) continue;
            std::vector<size_t> same{ z0 };
            for (size_t z = z0 + 1; z < items.size() && same.size() < (size_t)MHE_MAXB; z++)
            {
                if (done[z] || items[z].second.size() != items[z0].second.size()) continue;
                bool eq = true;
                for (size_t r = 0; eq && r < items[z].second.size(); r++)
                {
                    const int a = items[z].second[r], b = items[z0].second[r];
                    eq = keys[a] == keys[b] && key_limbs[a] == key_limbs[b] && elts[a] == elts[b];
                }
                if (eq) same.push_back(z);
            }
            if (same.size() < 2) continue;
            HoistShared hs{};
            hs.Z = (int)same.size();
            const std::vector<int> &r0 = items[z0].second;
            for (size_t r = 0; r < r0.size(); r++)
            {
                hs.key[r] = keys[r0[r]];
                hs.mask[r] = masks[r0[r]];
                hs.einv[r] = elt_inv[r0[r]];
                hs.key_limbs[r] = key_limbs[r0[r]];
            }
            for (int z = 0; z < hs.Z; z++)
            {
                const auto &it = items[same[z]];
                hs.D[z] = w->hoist[it.first];
                hs.c1[z] = in[it.first] + ps;
                hs.flag[z] = w->flags + it.first;
                for (size_t r = 0; r < it.second.size(); r++) hs.acc[z][r] = w->hacc[it.second[r]];
                done[same[z]] = 1;
            }
            hipEvent_t *tm = timing_slot(c, w, TK_KS_ROW_MAC, st);
            const int per_wg = r0.size() <= 4 ? 8 : 4; // 4 lane groups x items per lane
            launch_hoist_mac_sh((int)r0.size(), dim3((unsigned)(n / 256), (unsigned)(L + 1), (unsigned)((hs.Z + per_wg - 1) / per_wg)),
                                st, hs, c->primes, c->cmodf, L, c->K, log_n);
            c->hoist_mac++;
            timing_end(tm, st);
        }
        std::vector<std::pair<int, std::vector<int>>> left;
        for (size_t z = 0; z < items.size(); z++)
            if (!done[z]) left.push_back(items[z]);
        items.swap(left);
        // one rotation count per launch (k_ks_hoist_mac<R>): items ordered by it
        std::stable_sort(items.begin(), items.end(),
                         [](const std::pair<int, std::vector<int>> &a, const std::pair<int, std::vector<int>> &b) {
                             return a.second.size() > b.second.size();
                         });
        for (size_t z0 = 0; z0 < items.size();)
        {
            size_t zn = z0 + 1;
            while (zn < items.size() && zn - z0 < (size_t)MHE_MAXB && items[zn].second.size() == items[z0].second.size()) zn++;
            const int Z = (int)(zn - z0);
            HoistPtrs hp{};
            for (int z = 0; z < Z; z++)
            {
                const int h = items[z0 + z].first;
                const std::vector<int> &rs = items[z0 + z].second;
                hp.D[z] = w->hoist[h];
                hp.c1[z] = in[h] + ps;
                hp.flag[z] = w->flags + h;
                hp.R[z] = (int)rs.size();
                for (size_t r = 0; r < rs.size(); r++)
                {
                    const int i = rs[r];
                    hp.key[z][r] = keys[i];
                    hp.mask[z][r] = masks[i];
                    hp.acc[z][r] = w->hacc[i];
                    hp.einv[z][r] = elt_inv[i];
                    hp.key_limbs[z][r] = key_limbs[i];
                }
            }
            const dim3 grid((unsigned)(n / 256), (unsigned)(L + 1), (unsigned)Z);
            hipEvent_t *tm = timing_slot(c, w, TK_KS_ROW_MAC, st);
            launch_hoist_mac(hp.R[0], grid, st, hp, c->primes, c->cmodf, L, c->K, log_n);
            c->hoist_mac++;
            timing_end(tm, st);
            z0 = zn;
        }
        HIP_LAUNCH_CHECK();
    }
    // 3. per MHE_MAXB rotations: c0 / c1 permuted into out, the classic ModUp + MAC of flagged
    //    inputs (their kernels return at once otherwise), the ModDown (c1 written)
    std::vector<int> order(count);
    for (int i = 0; i < count; i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return keys[a] < keys[b]; });
    for (int i0 = 0; i0 < count; i0 += MHE_MAXB)
    {
        const int B = std::min(MHE_MAXB, count - i0);
        GalPtrs gp{};
        KsPtrs kp{};
        KsJob jobs[MHE_MAXB];
        u64 *accs[MHE_MAXB];
        JobB<JobStrided> ij;
        ij.per = L;
        int share = B > 1 ? 1 : 0;
        for (int e = 0; e < B; e++)
        {
            const int i = order[i0 + e], h = ent_in[i];
            gp.in[e] = in[h];
            gp.out[e] = out[i];
            gp.elt[e] = elts[i];
            jobs[e] = KsJob{ out[i], out[i] + ps, keys[i], key_limbs[i], nullptr };
            accs[e] = w->hacc[i];
            // the classic path of a flagged input: INTT of the permuted c1, ModUp, fused MAC
            ij.j[e] = JobStrided{ out[i] + ps, w->e[e].coeff, n, n, 0, 1, c->primes, c->itw, log_n, 0, w->flags + h };
            kp.coeff[e] = w->e[e].coeff;
            kp.inter[e] = w->e[e].modup;
            kp.target[e] = out[i] + ps;
            kp.key[e] = keys[i];
            kp.acc[e] = w->hacc[i];
            kp.key_limbs[e] = key_limbs[i];
            kp.run_if[e] = w->flags + h;
            if (keys[i] != keys[order[i0]] || key_limbs[i] != key_limbs[order[i0]]) share = 0;
        }
        if (!c->ks_share) share = 0;
        int kpack = 1;
        for (int e = 0; e < B; e++)
            if ((r = ks_check_key(c, jobs[e], L, st, &kpack))) return r;
        count_op(c, MHE_OPK_GALOIS, L, 2ull * B);
        count_op(c, MHE_OPK_KEYSWITCH, L, (unsigned long long)B);
        const size_t total = 2 * ps;
        hipLaunchKernelGGL(k_galois_b, dim3((unsigned)((total + 255) / 256), (unsigned)B), dim3(256), 0, st, gp, log_n,
                           total);
        inv_row(ij, log_n, B * L, c->nm, st);
        for (int e = 0; e < B; e++)
        {
            ij.j[e].src = w->e[e].coeff;
            ij.j[e].mode = 1;
        }
        inv_col(ij, log_n, B * L, c->nm, st);
        const int IG = c->ks_colgroups < L + 1 ? c->ks_colgroups : L + 1;
        modup_col(kp, B, c->primes, c->tw, L, c->K, log_n, c->nm_ks, 0, L + 1, IG, pack, st);
        ks_row_mac_chunk(kp, B, c->primes, c->tw, L, c->K, log_n, c->nm_ks, 0, L + 1, pack, kpack, share, c->itw, 0, st);
        HIP_LAUNCH_CHECK();
        run_moddown(c, jobs, B, L, w, 0, 1, st, accs);
    }
    c->hoist_rot += (unsigned long long)count;
    if (c->hoist_check) return hoist_check_pass(c, in, count, ent_in, out, elts, keys, key_limbs, L, st, w->flags);
    return MHE_OK;
}

MHE_EXPORT int mhe_apply_galois_batch(mhe_ctx *c, int count, const uint64_t *const *in, uint64_t *const *out,
                                      const uint32_t *elts, const uint64_t *const *keys, const int *key_limbs, int limbs,
                                      void *s)
{
    int r = check_limbs(c, limbs, 1);
    if (r) return r;
    if (count < 0 || (count && (!in || !out || !elts || !keys || !key_limbs))) return fail(MHE_ERR_ARG, "invalid argument");
    hipStream_t st = S(s);
    const size_t ps = (size_t)limbs << c->log_n;
    for (int i = 0; i < count; i++)
    {
        if (!in[i] || !out[i] || !keys[i]) return fail(MHE_ERR_ARG, "Galois key not present");
        if (!(elts[i] & 1) || elts[i] >= 2 * c->n) return fail(MHE_ERR_ARG, "Galois element is not valid");
        // every key is checked before the first launch, so a bad key leaves no output half-written
        if (key_limbs[i] < limbs + 1 || key_limbs[i] > c->K)
            return fail(MHE_ERR_ARG, "kswitch_keys is not valid for encryption parameters");
        // outputs must be disjoint from every input and from each other (all are written before the
        // first key switch reads its input's permutation back from its own output)
        for (int j = 0; j < count; j++)
        {
            const bool ov_in = ranges_overlap(out[i], 2 * ps, in[j], 2 * ps);
            const bool ov_out = j != i && ranges_overlap(out[i], 2 * ps, out[j], 2 * ps);
            if (ov_in || ov_out) return fail(MHE_ERR_ARG, "result cannot point to the same value as operand");
        }
    }
    if (!c->galois_fused)
    {
        for (int i = 0; i < count; i++)
            if ((r = mhe_apply_galois_to(c, in[i], out[i], elts[i], keys[i], key_limbs[i], limbs, s))) return r;
        return MHE_OK;
    }
    // inputs rotated more than once share their ModUp (hoist.h), up to MHE_MAXB inputs per pass
    std::vector<int> rest;
    if (hoist_ok(c) && count > 1 && c->n >= 256)
    {
        std::vector<const u64 *> uin;
        std::vector<std::vector<int>> uent;
        for (int i = 0; i < count; i++)
        {
            size_t u = 0;
            while (u < uin.size() && uin[u] != in[i]) u++;
            if (u == uin.size())
            {
                uin.push_back(in[i]);
                uent.emplace_back();
            }
            uent[u].push_back(i);
        }
        std::vector<const u64 *> hin;
        std::vector<int> ent_in;
        std::vector<u64 *> hout;
        std::vector<u32> hel;
        std::vector<const u64 *> hkey;
        std::vector<int> hkl;
        auto flush = [&]() -> int {
            if (hin.empty()) return MHE_OK;
            const int rr = run_galois_hoisted(c, hin.data(), (int)hin.size(), (int)ent_in.size(), ent_in.data(), hout.data(),
                                              hel.data(), hkey.data(), hkl.data(), limbs, st);
            hin.clear();
            ent_in.clear();
            hout.clear();
            hel.clear();
            hkey.clear();
            hkl.clear();
            return rr;
        };
        for (size_t u = 0; u < uin.size(); u++)
        {
            if (uent[u].size() < 2)
            {
                rest.push_back(uent[u][0]);
                continue;
            }
            // at most MHE_MAXB inputs and MHE_MAXB * MHE_HOIST_R rotations per pass (w->hacc)
            if ((hin.size() == MHE_MAXB || ent_in.size() + uent[u].size() > (size_t)MHE_MAXB * MHE_HOIST_R) &&
                (r = flush()))
                return r;
            if (uent[u].size() > (size_t)MHE_MAXB * MHE_HOIST_R)
            {
                // more rotations than one pass holds: the classic path (never in the callers' shapes)
                for (int i : uent[u]) rest.push_back(i);
                continue;
            }
            const int h = (int)hin.size();
            hin.push_back(uin[u]);
            for (int i : uent[u])
            {
                ent_in.push_back(h);
                hout.push_back(out[i]);
                hel.push_back(elts[i]);
                hkey.push_back(keys[i]);
                hkl.push_back(key_limbs[i]);
            }
        }
        if ((r = flush())) return r;
    }
    else
        for (int i = 0; i < count; i++) rest.push_back(i);
    // entries of one key side by side: a launch of them shares the key stream (k_ks_row_mac share)
    std::stable_sort(rest.begin(), rest.end(), [&](int a, int b) { return keys[a] < keys[b]; });
    const int nrest = (int)rest.size();
    for (int i0 = 0; i0 < nrest; i0 += MHE_MAXB)
    {
        const int B = std::min(MHE_MAXB, nrest - i0);
        // out_e <- perm_e(in_e), both polys, one launch (evaluator.cpp:2193-2214; SEAL zeroes c1 and
        // adds KS_1, the same words as writing it)
        GalPtrs gp{};
        KsJob jobs[MHE_MAXB];
        for (int e = 0; e < B; e++)
        {
            const int i = rest[i0 + e];
            gp.in[e] = in[i];
            gp.out[e] = out[i];
            gp.elt[e] = elts[i];
            jobs[e] = KsJob{ out[i], out[i] + ps, keys[i], key_limbs[i], nullptr };
        }
        const size_t total = 2 * ps;
        count_op(c, MHE_OPK_GALOIS, limbs, 2ull * B);
        hipLaunchKernelGGL(k_galois_b, dim3((unsigned)((total + 255) / 256), (unsigned)B), dim3(256), 0, st, gp, c->log_n,
                           total);
        HIP_LAUNCH_CHECK();
        if ((r = run_switch_key_batch(c, jobs, B, limbs, st, 1))) return r;
    }
    return MHE_OK;
}

MHE_EXPORT int mhe_rescale_batch(mhe_ctx *c, int count, const uint64_t *const *in, uint64_t *const *out, int size,
                                 int limbs, void *s)
{
    if (!valid_ctx(c)) return fail(MHE_ERR_ARG, "context is not valid");
    if (limbs < 2) return fail(MHE_ERR_RANGE, "end of modulus switching chain reached");
    if (limbs > c->K || size < 1 || size > 3 || count < 0 || (count && (!in || !out)))
        return fail(MHE_ERR_ARG, "encrypted is not valid for encryption parameters");
    const size_t iw = ((size_t)size * limbs) << c->log_n, ow = ((size_t)size * (limbs - 1)) << c->log_n;
    for (int i = 0; i < count; i++)
    {
        if (!in[i] || !out[i]) return fail(MHE_ERR_ARG, "encrypted is not valid for encryption parameters");
        // an output may share no word with any entry's input or with another output: the last pass
        // writes out[i] while other workgroups of the same launch still read their inputs
        for (int j = 0; j < count; j++)
            if (ranges_overlap(out[i], ow, in[j], iw) || (j != i && ranges_overlap(out[i], ow, out[j], ow)))
                return fail(MHE_ERR_ARG, "rescale output must not alias its input");
    }
    for (int i0 = 0; i0 < count; i0 += MHE_MAXB)
    {
        const int B = std::min(MHE_MAXB, count - i0);
        int r = run_rescale_batch(c, in + i0, out + i0, B, size, limbs, S(s));
        if (r) return r;
    }
    return MHE_OK;
}

MHE_EXPORT int mhe_switch_key_batch(mhe_ctx *c, int count, uint64_t *const *ct, const uint64_t *const *target,
                                    const uint64_t *const *keys, const int *key_limbs, int limbs, void *s)
{
    int r = check_limbs(c, limbs, 1);
    if (r) return r;
    if (count < 0 || (count && (!ct || !target || !keys || !key_limbs))) return fail(MHE_ERR_ARG, "invalid argument");
    for (int i = 0; i < count; i++)
    {
        if (!ct[i] || !target[i] || !keys[i]) return fail(MHE_ERR_ARG, "target_iter");
        // every key before the first launch: the switches work in place, chunk by chunk
        if (key_limbs[i] < limbs + 1 || key_limbs[i] > c->K)
            return fail(MHE_ERR_ARG, "kswitch_keys is not valid for encryption parameters");
    }
    for (int i0 = 0; i0 < count; i0 += MHE_MAXB)
    {
        const int B = std::min(MHE_MAXB, count - i0);
        KsJob jobs[MHE_MAXB];
        for (int e = 0; e < B; e++) jobs[e] = KsJob{ ct[i0 + e], target[i0 + e], keys[i0 + e], key_limbs[i0 + e], nullptr };
        if ((r = run_switch_key_batch(c, jobs, B, limbs, S(s)))) return r;
    }
    return MHE_OK;
}

MHE_EXPORT int mhe_rescale_to_next(mhe_ctx *c, const uint64_t *in, uint64_t *out, int size, int limbs, void *s)
{
    TR("out", out, (size_t)size * (limbs - 1) * ((size_t)1 << c->log_n)); TR("in", in, (size_t)size * limbs * ((size_t)1 << c->log_n));
    TRC(0, 0, 0, 0);
    if (!valid_ctx(c)) return fail(MHE_ERR_ARG, "context is not valid");
    if (limbs < 2) return fail(MHE_ERR_RANGE, "end of modulus switching chain reached");
    if (limbs > c->K || size < 1 || size > 3 || !in || !out)
        return fail(MHE_ERR_ARG, "encrypted is not valid for encryption parameters");
    if (in == out) return fail(MHE_ERR_ARG, "rescale output must not alias its input");
    return run_rescale(c, in, out, size, limbs, S(s));
}

MHE_EXPORT int mhe_modraise(mhe_ctx *c, const uint64_t *in, uint64_t *out, int size, int limbs, void *s)
{
    TR("out", out, (size_t)size * limbs * ((size_t)1 << c->log_n)); TR("in", in, (size_t)size * ((size_t)1 << c->log_n));
    TRC(0, 0, 0, 0);
    if (!valid_ctx(c)) return fail(MHE_ERR_ARG, "context is not valid");
    if (!in || !out || size < 1 || limbs < 1 || limbs > c->K) return fail(MHE_ERR_ARG, "invalid polynomial arguments");
    const size_t total = ((size_t)size * limbs) << c->log_n;
    hipLaunchKernelGGL(k_modraise, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, S(s), in, out, c->primes,
                       limbs, c->log_n, total);
    HIP_LAUNCH_CHECK();
    return MHE_OK;
}

MHE_EXPORT int mhe_mod_switch_drop(mhe_ctx *c, const uint64_t *in, uint64_t *out, int size, int limbs, void *s)
{
    TR("out", out, (size_t)size * (limbs - 1) * ((size_t)1 << c->log_n)); TR("in", in, (size_t)size * limbs * ((size_t)1 << c->log_n));
    TRC(0, 0, 0, 0);
    if (!valid_ctx(c)) return fail(MHE_ERR_ARG, "context is not valid");
    if (limbs < 2) return fail(MHE_ERR_RANGE, "end of modulus switching chain reached");
    if (!in || !out || size < 1) return fail(MHE_ERR_ARG, "invalid polynomial arguments");
    const size_t src_pitch = ((size_t)limbs << c->log_n) * sizeof(u64);
    const size_t dst_pitch = ((size_t)(limbs - 1) << c->log_n) * sizeof(u64);
    if (in != out)
    {
        for (int p = 0; p < size; p++)
            HIP_TRY(mhe_internal_copy_d2d((char *)out + p * dst_pitch, (const char *)in + p * src_pitch, dst_pitch,
                                          S(s)));
        return MHE_OK;
    }
    // In place: component p moves down by p limbs.  One copy per limb, ascending: every copy's
    // source and destination are disjoint (they are p*n words apart), and a destination never
    // covers a source that a later copy still has to read.
    const size_t limb_bytes = sizeof(u64) << c->log_n;
    for (int p = 1; p < size; p++)
        for (int l = 0; l + 1 < limbs; l++)
            HIP_TRY(mhe_internal_copy_d2d((char *)out + p * dst_pitch + l * limb_bytes,
                                          (const char *)in + p * src_pitch + l * limb_bytes, limb_bytes, S(s)));
    return MHE_OK;
}

MHE_EXPORT int mhe_hmult_batch(mhe_ctx *c, int count, const uint64_t *const *a, const uint64_t *const *b,
                               const uint64_t *key, int key_limbs, uint64_t *const *out, int limbs, void *s)
{
    // mhe_hmult of every entry, MHE_MAXB per key switch: the tensor products into per-entry
    // scratch, then one batched key switch (all entries share the relinearization key, so
    // k_ks_row_mac reads it once per XCD) with the fused rescale tail -- bit-identical to count
    // mhe_hmult calls
    int r = check_limbs(c, limbs, 2);
    if (r) return r;
    if (count < 0 || (count && (!a || !b || !out)) || !key) return fail(MHE_ERR_ARG, "invalid argument");
    if (key_limbs < limbs + 1 || key_limbs > c->K) return fail(MHE_ERR_ARG, "kswitch_keys is not valid for encryption parameters");
    const size_t iw = (size_t)2 * limbs * c->n, ow = (size_t)2 * (limbs - 1) * c->n;
    for (int i = 0; i < count; i++)
    {
        if (!a[i] || !b[i] || !out[i]) return fail(MHE_ERR_ARG, "invalid argument");
        // out[i] may overlap its own operands (they are consumed by the tensor product before the
        // tail writes out[i]) but no other entry's operands (a later chunk reads them after this
        // chunk's tail) and no other output
        for (int j = 0; j < count; j++)
        {
            if (j == i) continue;
            if (ranges_overlap(out[i], ow, out[j], ow)) return fail(MHE_ERR_ARG, "outputs must be distinct");
            if (ranges_overlap(out[i], ow, a[j], iw) || ranges_overlap(out[i], ow, b[j], iw))
                return fail(MHE_ERR_ARG, "result cannot point to the same value as another entry's operand");
        }
    }
    hipStream_t st = S(s);
    const size_t n = c->n;
    for (int i0 = 0; i0 < count; i0 += MHE_MAXB)
    {
        const int B = std::min(MHE_MAXB, count - i0);
        Workspace *w;
        if ((r = get_ws(c, st, c->K - 1, &w, B))) return r;
        KsJob jobs[MHE_MAXB];
        for (int e = 0; e < B; e++)
        {
            const int i = i0 + e;
            if ((r = launch_tensor(c, a[i], b[i], w->e[e].ct3, limbs, a[i] == b[i], st))) return r;
            jobs[e] = KsJob{ w->e[e].ct3, w->e[e].ct3 + ((size_t)2 * limbs * n), key, key_limbs,
                             c->hmult_fused ? out[i] : nullptr };
        }
        if ((r = run_switch_key_batch(c, jobs, B, limbs, st))) return r;
        if (!c->hmult_fused)
        {
            const u64 *in[MHE_MAXB];
            u64 *o[MHE_MAXB];
            for (int e = 0; e < B; e++)
            {
                in[e] = w->e[e].ct3;
                o[e] = out[i0 + e];
            }
            if ((r = run_rescale_batch(c, in, o, B, 2, limbs, st))) return r;
        }
    }
    return MHE_OK;
}

MHE_EXPORT int mhe_hmult(mhe_ctx *c, const uint64_t *a, const uint64_t *b, const uint64_t *key, int key_limbs,
                         uint64_t *out, int limbs, void *s)
{
    int r = check_limbs(c, limbs, 2);
    if (r) return r;
    if (!a || !b || !key || !out) return fail(MHE_ERR_ARG, "invalid argument");
    hipStream_t st = S(s);
    Workspace *w;
    r = get_ws(c, st, c->K - 1, &w);
    if (r) return r;
    if ((r = launch_tensor(c, a, b, w->ct3, limbs, a == b, st))) return r;
    if (c->hmult_fused)
        return run_switch_key(c, w->ct3, w->ct3 + ((size_t)2 * limbs << c->log_n), key, key_limbs, limbs, st, out);
    if ((r = run_switch_key(c, w->ct3, w->ct3 + ((size_t)2 * limbs << c->log_n), key, key_limbs, limbs, st))) return r;
    return run_rescale(c, w->ct3, out, 2, limbs, st);
}
