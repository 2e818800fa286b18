// CKKS encoding for libmhe.
//
// CKKSEncoder::encode (SEAL/ckks.h:457-640) is a double-precision FFT followed by rounding, an
// RNS reduction and a per-limb NTT.  Bit-exactness with SEAL needs SEAL's exact sequence of
// non-fused double operations (the reference builds its encoder without FMA); IEEE double
// arithmetic is the same on the host and on the GPU, so the whole encode runs on the device,
// compiled with -ffp-contract=off, in SEAL's operation order:
//   * ComplexRoots (util/croots.cpp:17-66): polar(1, 2*PI*i/m) for i <= m/8, 8-fold symmetry,
//     computed once on the host (sincos) and kept in HBM per device;
//   * index map 5^i (ckks.cpp:34-49) computed per slot on the device;
//   * DWTHandler::transform_from_rev over complex<double> with scalar scale/n
//     (util/dwthandler.h:202-314, ckks.h:46-81): the first 12 stages in LDS (4096-point blocks),
//     the remaining stages one launch each;
//   * std::round, then the coefficient's integer value mod q_j (SEAL's 1-word, 2-word and
//     multi-word paths all reduce the same integer, so one per-coefficient decomposition gives
//     their residues).
// The slot values travel through a pinned staging ring, so encode never waits for the device.
// SEAL's "encoded values are too large" check needs max |coeff|: a host bound
// (scale / n) * 2 * sum |v_i| settles it for every ordinary input; only when the bound comes
// within a bit of the limit is the exact device maximum read back (one stream sync).
#include <hip/hip_runtime.h>

#include <cmath>
#include <complex>
#include <cstring>
#include <mutex>
#include <string>

extern "C" hipError_t mhe_internal_copy_d2d(void *dst, const void *src, size_t bytes, hipStream_t st);
extern "C" hipError_t mhe_internal_alloc(void **p, size_t bytes, hipStream_t st);
extern "C" hipError_t mhe_internal_free(void *p, hipStream_t st);
#include <vector>

#include "../../include/mhe.h"
#include "arith.h"

typedef unsigned __int128 u128;
typedef std::complex<double> cd;

// shared with mhe.hip
int mhe_internal_fail(int code, const char *msg);
int mhe_internal_ntt_forward(mhe_ctx *c, uint64_t *data, int polys, int limbs, int full, hipStream_t st);
int mhe_internal_primes(mhe_ctx *c, const PrimeDev **dev, const uint64_t **host, int *count, int *log_n);

struct mhe_encoder
{
    int log_n = 0;
    size_t n = 0, slots = 0;
    std::vector<size_t> index_map;
    std::vector<cd> inv_root_powers;
    std::vector<cd> root_powers;

    // device state (lazily created on the first encode of each device)
    // Pinned upload slots, reused round robin.  Reusing a slot waits (under `mu`, so for every
    // thread) until its last upload has run, and that upload sits behind whatever its stream had
    // queued -- with 8 slots, 3 host threads x 8 fibers wrapped the ring within one merged step and
    // every thread stalled behind another stream's key switches.  64 slots (32 MB at n = 2^16) are
    // reused only after ~0.1 s of encodes, when no stream is that far behind.
    static constexpr int kRing = 64;
    struct DevRoots
    {
        int dev;
        double2 *roots;
    };
    mutable std::mutex mu;
    mutable std::vector<DevRoots> dev_roots;
    mutable double *ring = nullptr; // kRing slots of 2 * slots doubles (re, im), pinned
    mutable hipEvent_t ring_ev[kRing] = {};
    mutable int ring_dev = -1;
    mutable unsigned ring_next = 0;
    ~mhe_encoder()
    {
        for (auto &d : dev_roots) (void)hipFree(d.roots);
        if (ring) (void)hipHostFree(ring);
        for (auto &ev : ring_ev)
            if (ev) (void)hipEventDestroy(ev);
    }
};

namespace
{
u32 rev_bits(u32 x, int bits)
{
    return bits ? (__builtin_bitreverse32(x) >> (32 - bits)) : 0;
}

struct ComplexRoots
{
    size_t m;
    std::vector<cd> roots;
    explicit ComplexRoots(size_t degree) : m(degree), roots(degree / 8 + 1)
    {
        const double PI_ = 3.1415926535897932384626433832795028842;
        for (size_t i = 0; i <= m / 8; i++)
        {
            // std::polar(1, theta) as SEAL's GCC Release build evaluates it: one sincos() call
            // (separate cos()/sin() differ in the last bit for a few angles)
            double sn, cs;
            ::sincos(2 * PI_ * static_cast<double>(i) / static_cast<double>(m), &sn, &cs);
            roots[i] = cd(cs, sn);
        }
    }
    cd get(size_t index) const
    {
        index &= m - 1;
        if (index <= m / 8) return roots[index];
        if (index <= m / 4) return cd(roots[m / 4 - index].imag(), roots[m / 4 - index].real());
        if (index <= m / 2) return -std::conj(get(m / 2 - index));
        if (index <= 3 * m / 4) return -get(index - m / 2);
        return std::conj(get(m - index));
    }
};

// SEAL's ContextData::total_coeff_modulus_bit_count: bit length of prod q_j.
int total_bits(const uint64_t *q, int limbs)
{
    std::vector<u64> prod(limbs + 1, 0);
    prod[0] = 1;
    int words = 1;
    for (int j = 0; j < limbs; j++)
    {
        u64 carry = 0;
        for (int w = 0; w < words; w++)
        {
            u128 t = (u128)prod[w] * q[j] + carry;
            prod[w] = (u64)t;
            carry = (u64)(t >> 64);
        }
        if (carry) prod[words++] = carry;
    }
    return 64 * (words - 1) + (64 - __builtin_clzll(prod[words - 1]));
}

u64 words_mod(const u64 *w, int nw, u64 q)
{
    u128 r = 0;
    for (int k = nw - 1; k >= 0; k--) r = ((r << 64) | w[k]) % q;
    return (u64)r;
}
} // namespace

// ---- device encode kernels -------------------------------------------------------------
namespace
{
__device__ __forceinline__ u32 rev_bits_dev(u32 x, int bits)
{
    return __builtin_bitreverse32(x) >> (32 - bits);
}

// cv[index_map[i]] = v_i, cv[index_map[i + slots]] = conj(v_i) (ckks.h:488-497); cv pre-zeroed
__global__ void k_enc_scatter(const double *vals, size_t count, int has_im, double2 *cv, int log_n)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    const u64 m = (u64)2 << log_n;
    u64 pos = 1, b = 5;
    for (u64 e = i; e; e >>= 1)
    {
        if (e & 1) pos = (pos * b) & (m - 1);
        b = (b * b) & (m - 1);
    }
    const double re = vals[i], im = has_im ? vals[count + i] : 0.0;
    cv[rev_bits_dev((u32)((pos - 1) >> 1), log_n)] = double2{ re, im };
    cv[rev_bits_dev((u32)((m - pos - 1) >> 1), log_n)] = double2{ re, -im };
}

// one butterfly of transform_from_rev in SEAL's operation order (complex products as
// (ac - bd, ad + bc), no contraction); the last stage folds in the scalar
__device__ __forceinline__ void enc_bfly(double2 &x, double2 &y, double2 r, bool last, double scalar)
{
    const double2 u = x, v = y;
    const double2 s = double2{ u.x + v.x, u.y + v.y }, d = double2{ u.x - v.x, u.y - v.y };
    if (last)
    {
        r = double2{ r.x * scalar, r.y * scalar };
        x = double2{ s.x * scalar, s.y * scalar };
    }
    else
        x = s;
    y = double2{ d.x * r.x - d.y * r.y, d.x * r.y + d.y * r.x };
}

constexpr int kEncLogBlock = 12;

// stages 0 .. lb-1 (gap 1 .. 2^(lb-1)) of one 2^lb-point block in LDS
__global__ __launch_bounds__(256) void k_enc_fft_block(double2 *cv, const double2 *roots, int log_n, int lb,
                                                       double scalar)
{
    __shared__ double2 sh[1 << kEncLogBlock];
    const size_t n = (size_t)1 << log_n, B = (size_t)1 << lb, base = (size_t)blockIdx.x << lb;
    for (size_t t = threadIdx.x; t < B; t += 256) sh[t] = cv[base + t];
    __syncthreads();
    for (int st = 0; st < lb; st++)
    {
        const size_t m = n >> (st + 1), gap = (size_t)1 << st;
        for (size_t t = threadIdx.x; t < B / 2; t += 256)
        {
            const size_t k = t >> st, x = (k << (st + 1)) + (t & (gap - 1));
            const double2 r = roots[n - 2 * m + 1 + (base >> (st + 1)) + k];
            enc_bfly(sh[x], sh[x + gap], r, m == 1, scalar);
        }
        __syncthreads();
    }
    for (size_t t = threadIdx.x; t < B; t += 256) cv[base + t] = sh[t];
}

// stages lb .. log_n-1 (gap 2^lb .. 2^(log_n-1)) in one launch: they only pair elements with the same
// low lb bits, so a lane holds the 2^(log_n-lb) <= 16 elements of one such column in registers and
// runs the stages in order -- the same butterflies on the same values as one k_enc_fft_stage launch
// per stage, so the same doubles, in one launch instead of log_n - lb
template <int LR> // log_n - lb
__global__ __launch_bounds__(256) void k_enc_fft_tail(double2 *cv, const double2 *roots, int log_n, int lb,
                                                      double scalar)
{
    constexpr int R = 1 << LR;
    const size_t n = (size_t)1 << log_n, c = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= ((size_t)1 << lb)) return;
    double2 v[R];
#pragma unroll
    for (int j = 0; j < R; j++) v[j] = cv[c + ((size_t)j << lb)];
#pragma unroll
    for (int s = 0; s < LR; s++)
    {
        const int st = lb + s;
        const size_t m = n >> (st + 1);
#pragma unroll
        for (int j = 0; j < R; j++)
            if (!(j & (1 << s)))
            {
                const double2 r = roots[n - 2 * m + 1 + (size_t)(j >> (s + 1))];
                enc_bfly(v[j], v[j + (1 << s)], r, m == 1, scalar);
            }
    }
#pragma unroll
    for (int j = 0; j < R; j++) cv[c + ((size_t)j << lb)] = v[j];
}

// one later stage (gap 2^st) over the whole vector
__global__ void k_enc_fft_stage(double2 *cv, const double2 *roots, int log_n, int st, double scalar)
{
    const size_t n = (size_t)1 << log_n, t = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= n / 2) return;
    const size_t m = n >> (st + 1), gap = (size_t)1 << st, k = t >> st, x = (k << (st + 1)) + (t & (gap - 1));
    enc_bfly(cv[x], cv[x + gap], roots[n - 2 * m + 1 + k], m == 1, scalar);
}

// max |Re cv_i| as ordered bit patterns (non-negative doubles order like their u64 bits)
__global__ void k_enc_absmax(const double2 *cv, size_t n, unsigned long long *mx)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    unsigned long long v = i < n ? (unsigned long long)__double_as_longlong(fabs(cv[i].x)) : 0ull;
    for (int o = 32; o; o >>= 1) v = max(v, (unsigned long long)__shfl_xor(v, o));
    if ((threadIdx.x & 63) == 0) atomicMax(mx, v);
}

// out[j][i] = round(Re cv_i) mod q_j, sign applied (ckks.h:545-640)
__global__ void k_enc_round_reduce(const double2 *cv, u64 *out, const PrimeDev *primes, int limbs, int log_n)
{
    const size_t n = (size_t)1 << log_n;
    const size_t g = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= n * limbs) return;
    const size_t i = g & (n - 1);
    const PrimeDev p = primes[g >> log_n];
    double c = round(cv[i].x);
    const bool neg = signbit(c);
    c = fabs(c);
    u64 r;
    if (c < 0x1p64)
        r = barrett64((u64)c, p);
    else
    {
        u64 w[17];
        int nw = 0;
        while (c >= 1 && nw < 17)
        {
            w[nw++] = (u64)fmod(c, 0x1p64);
            c /= 0x1p64;
        }
        r = 0;
        for (int k = nw - 1; k >= 0; k--) r = barrett128(w[k], r, p);
    }
    out[g] = (neg && r) ? p.q - r : r;
}
} // namespace

extern "C" __attribute__((visibility("default"))) int mhe_encoder_create(mhe_encoder **out, int log_n)
{
    if (!out || log_n < 2 || log_n > 17) return mhe_internal_fail(MHE_ERR_ARG, "poly_modulus_degree is invalid");
    mhe_encoder *e = new mhe_encoder;
    const size_t n = size_t(1) << log_n, m = n << 1;
    e->log_n = log_n;
    e->n = n;
    e->slots = n >> 1;
    e->index_map.resize(n);
    u64 pos = 1;
    for (size_t i = 0; i < e->slots; i++)
    {
        const u64 index1 = (pos - 1) >> 1, index2 = (m - pos - 1) >> 1;
        e->index_map[i] = rev_bits((u32)index1, log_n);
        e->index_map[e->slots | i] = rev_bits((u32)index2, log_n);
        pos = (pos * 5) & (m - 1);
    }
    e->root_powers.assign(n, cd(0, 0));
    e->inv_root_powers.assign(n, cd(0, 0));
    ComplexRoots cr(m);
    for (size_t i = 1; i < n; i++)
    {
        e->root_powers[i] = cr.get(rev_bits((u32)i, log_n));
        e->inv_root_powers[i] = std::conj(cr.get(rev_bits((u32)(i - 1), log_n) + 1));
    }
    *out = e;
    return MHE_OK;
}

extern "C" __attribute__((visibility("default"))) int mhe_encoder_destroy(mhe_encoder *e)
{
    delete e;
    return MHE_OK;
}

extern "C" __attribute__((visibility("default"))) int mhe_ckks_encode_at(mhe_ctx *c, const mhe_encoder *e,
                                                                        const double *re, const double *im,
                                                                        size_t count, double scale, int bound_limbs,
                                                                        int limbs, uint64_t *out, void *stream)
{
    const PrimeDev *primes;
    const uint64_t *q;
    int K, log_n;
    if (mhe_internal_primes(c, &primes, &q, &K, &log_n)) return mhe_internal_fail(MHE_ERR_ARG, "context is not valid");
    if (!e || e->log_n != log_n) return mhe_internal_fail(MHE_ERR_ARG, "encoder does not match the context");
    if (!re && count > 0) return mhe_internal_fail(MHE_ERR_ARG, "values cannot be null");
    if (count > e->slots) return mhe_internal_fail(MHE_ERR_ARG, "values_size is too large");
    if (limbs < 1 || limbs > bound_limbs || bound_limbs > K || !out)
        return mhe_internal_fail(MHE_ERR_ARG, "parms_id is not valid for encryption parameters");
    const int tb = total_bits(q, bound_limbs);
    if (scale <= 0 || (static_cast<int>(std::log2(scale)) + 1 >= tb))
        return mhe_internal_fail(MHE_ERR_ARG, ("scale out of bounds (encoding 2^" + std::to_string(std::log2(scale)) +
                                               " at " + std::to_string(bound_limbs) + " limbs, " + std::to_string(tb) +
                                               " bits)").c_str());
    const size_t n = e->n;
    hipStream_t st = (hipStream_t)stream;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return mhe_internal_fail(MHE_ERR_DEVICE, "no device");

    // host bound on max |coeff| (each value and its conjugate enter with unit-modulus weights)
    double l1 = 0;
    for (size_t i = 0; i < count; i++) l1 += std::fabs(re[i]) + (im ? std::fabs(im[i]) : 0.0);
    const double fix = scale / static_cast<double>(n);
    const double bound = fix * 2 * l1 * (1 + 1e-6) + 1;
    const bool exact_check = !(std::isfinite(bound) &&
                               static_cast<int>(std::ceil(std::log2(std::max<double>(bound, 1.0)))) + 1 < tb);

    std::unique_lock<std::mutex> lk(e->mu);
    const double2 *roots = nullptr;
    for (auto &d : e->dev_roots)
        if (d.dev == dev) roots = d.roots;
    if (!roots)
    {
        double2 *r = nullptr;
        if (hipMalloc((void **)&r, n * sizeof(double2)) != hipSuccess)
            return mhe_internal_fail(MHE_ERR_MEMORY, "encoder roots allocation failed");
        if (hipMemcpy(r, e->inv_root_powers.data(), n * sizeof(double2), hipMemcpyHostToDevice) != hipSuccess)
        {
            (void)hipFree(r);
            return mhe_internal_fail(MHE_ERR_DEVICE, "encoder roots upload failed");
        }
        e->dev_roots.push_back({ dev, r });
        roots = r;
    }
    // staging: [cv: n double2][values: 2 * count doubles][max word]
    const size_t vwords = count * (im ? 2 : 1);
    char *buf = nullptr;
    const size_t bytes = n * sizeof(double2) + vwords * sizeof(double) + sizeof(u64);
    if (mhe_internal_alloc((void **)&buf, bytes, st) != hipSuccess)
        return mhe_internal_fail(MHE_ERR_MEMORY, "encode staging allocation failed");
    double2 *cv = (double2 *)buf;
    double *vals = (double *)(cv + n);
    unsigned long long *mx = (unsigned long long *)(vals + vwords);
    hipError_t err = hipMemsetAsync(cv, 0, n * sizeof(double2), st);
    if (err == hipSuccess && vwords)
    {
        if (e->ring_dev < 0)
        {
            if (hipHostMalloc((void **)&e->ring, mhe_encoder::kRing * 2 * e->slots * sizeof(double)) == hipSuccess)
            {
                e->ring_dev = dev;
                for (auto &ev : e->ring_ev)
                    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) e->ring_dev = -2;
            }
            else
                e->ring_dev = -2;
        }
        if (e->ring_dev == dev)
        {
            const unsigned slot = e->ring_next++ % mhe_encoder::kRing;
            double *h = e->ring + (size_t)slot * 2 * e->slots;
            err = hipEventSynchronize(e->ring_ev[slot]); // the slot's previous upload is done
            if (err == hipSuccess)
            {
                std::memcpy(h, re, count * sizeof(double));
                if (im) std::memcpy(h + count, im, count * sizeof(double));
                err = hipMemcpyAsync(vals, h, vwords * sizeof(double), hipMemcpyHostToDevice, st);
            }
            if (err == hipSuccess) err = hipEventRecord(e->ring_ev[slot], st);
        }
        else
        {
            // another device than the ring's: synchronous upload from the caller's arrays
            err = hipMemcpyAsync(vals, re, count * sizeof(double), hipMemcpyHostToDevice, st);
            if (err == hipSuccess && im)
                err = hipMemcpyAsync(vals + count, im, count * sizeof(double), hipMemcpyHostToDevice, st);
            if (err == hipSuccess) err = hipStreamSynchronize(st);
        }
    }
    lk.unlock();
    if (err == hipSuccess && count)
        hipLaunchKernelGGL(k_enc_scatter, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st, vals, count,
                           im ? 1 : 0, cv, log_n);
    if (err == hipSuccess)
    {
        const int lb = std::min(log_n, kEncLogBlock);
        hipLaunchKernelGGL(k_enc_fft_block, dim3((unsigned)(n >> lb)), dim3(256), 0, st, cv, roots, log_n, lb, fix);
        const dim3 tg((unsigned)(((1u << lb) + 255) / 256));
        if (log_n - lb == 4)
            hipLaunchKernelGGL(k_enc_fft_tail<4>, tg, dim3(256), 0, st, cv, roots, log_n, lb, fix);
        else if (log_n - lb == 3)
            hipLaunchKernelGGL(k_enc_fft_tail<3>, tg, dim3(256), 0, st, cv, roots, log_n, lb, fix);
        else if (log_n - lb == 2)
            hipLaunchKernelGGL(k_enc_fft_tail<2>, tg, dim3(256), 0, st, cv, roots, log_n, lb, fix);
        else if (log_n - lb == 1)
            hipLaunchKernelGGL(k_enc_fft_tail<1>, tg, dim3(256), 0, st, cv, roots, log_n, lb, fix);
        else
            for (int s2 = lb; s2 < log_n; s2++)
                hipLaunchKernelGGL(k_enc_fft_stage, dim3((unsigned)((n / 2 + 255) / 256)), dim3(256), 0, st, cv, roots,
                                   log_n, s2, fix);
        err = hipGetLastError();
    }
    if (err == hipSuccess && exact_check)
    {
        // SEAL's check on the exact maximum (ckks.h:525-540)
        unsigned long long h_mx = 0;
        err = hipMemsetAsync(mx, 0, sizeof(u64), st);
        if (err == hipSuccess)
        {
            hipLaunchKernelGGL(k_enc_absmax, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, cv, n, mx);
            err = hipMemcpyAsync(&h_mx, mx, sizeof(u64), hipMemcpyDeviceToHost, st);
        }
        if (err == hipSuccess) err = hipStreamSynchronize(st);
        if (err == hipSuccess)
        {
            double max_coeff;
            std::memcpy(&max_coeff, &h_mx, sizeof(double));
            const int max_bits = static_cast<int>(std::ceil(std::log2(std::max<double>(max_coeff, 1.0)))) + 1;
            if (!(max_bits < tb)) // NaN compares false: rejected as well
            {
                (void)mhe_internal_free(buf, st);
                return mhe_internal_fail(MHE_ERR_ARG, "encoded values are too large");
            }
        }
    }
    if (err == hipSuccess)
    {
        const size_t total = n * limbs;
        hipLaunchKernelGGL(k_enc_round_reduce, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, cv, out,
                           primes, limbs, log_n);
        err = hipGetLastError();
    }
    (void)mhe_internal_free(buf, st);
    if (err != hipSuccess) return mhe_internal_fail(MHE_ERR_DEVICE, hipGetErrorString(err));
    return mhe_internal_ntt_forward(c, out, 1, limbs, 1, st);
}

extern "C" __attribute__((visibility("default"))) int mhe_ckks_encode(mhe_ctx *c, const mhe_encoder *e,
                                                                     const double *re, const double *im,
                                                                     size_t count, double scale, int limbs,
                                                                     uint64_t *out, void *stream)
{
    return mhe_ckks_encode_at(c, e, re, im, count, scale, limbs, limbs, out, stream);
}

extern "C" __attribute__((visibility("default"))) int mhe_ckks_encode_scalar_at(mhe_ctx *c, double value, double scale,
                                                                               int bound_limbs, int limbs,
                                                                               uint64_t *residues)
{
    const PrimeDev *primes;
    const uint64_t *q;
    int K, log_n;
    if (mhe_internal_primes(c, &primes, &q, &K, &log_n)) return mhe_internal_fail(MHE_ERR_ARG, "context is not valid");
    if (limbs < 1 || limbs > bound_limbs || bound_limbs > K || !residues)
        return mhe_internal_fail(MHE_ERR_ARG, "parms_id is not valid for encryption parameters");
    const int tb = total_bits(q, bound_limbs);
    if (scale <= 0 || (static_cast<int>(std::log2(scale)) >= tb)) return mhe_internal_fail(MHE_ERR_ARG, "scale out of bounds");
    value *= scale;
    const int coeff_bits = static_cast<int>(std::log2(std::fabs(value))) + 2;
    if (coeff_bits >= tb) return mhe_internal_fail(MHE_ERR_ARG, "encoded value is too large");
    const double two64 = std::pow(2.0, 64);
    double coeffd = std::round(value);
    const bool is_neg = std::signbit(coeffd);
    coeffd = std::fabs(coeffd);
    u64 w[64] = { 0 };
    int nw = 1;
    if (coeff_bits <= 64)
        w[0] = static_cast<u64>(std::fabs(coeffd));
    else if (coeff_bits <= 128)
    {
        w[0] = static_cast<u64>(std::fmod(coeffd, two64));
        w[1] = static_cast<u64>(coeffd / two64);
        nw = 2;
    }
    else
    {
        nw = 0;
        while (coeffd >= 1)
        {
            w[nw++] = static_cast<u64>(std::fmod(coeffd, two64));
            coeffd /= two64;
        }
        if (!nw) nw = 1;
    }
    for (int j = 0; j < limbs; j++)
    {
        const u64 r = words_mod(w, nw, q[j]);
        residues[j] = (is_neg && r) ? q[j] - r : r;
    }
    return MHE_OK;
}

extern "C" __attribute__((visibility("default"))) int mhe_ckks_encode_scalar(mhe_ctx *c, double value, double scale,
                                                                            int limbs, uint64_t *residues)
{
    return mhe_ckks_encode_scalar_at(c, value, scale, limbs, limbs, residues);
}

// ------------------------------------------------------------------------------------ decode
// CKKSEncoder::decode (ckks.h:644-761).  The inverse NTT runs on the GPU; CRT composition
// (RNSBase::compose_array, util/rns.cpp:354-400 -- its result is the canonical value in
// [0, Q), so any exact composition gives SEAL's words), the sparse-slot mask (ckks.h:704-713),
// SEAL's word-by-word double conversion (ckks.h:715-753) and transform_to_rev
// (util/dwthandler.h:94-190) run on the host in SEAL's operation order.
namespace
{
void fft_to_rev(cd *values, int log_n, const cd *roots)
{
    const size_t n = size_t(1) << log_n;
    size_t gap = n >> 1, m = 1;
    for (; m < (n >> 1); m <<= 1)
    {
        size_t offset = 0;
        for (size_t i = 0; i < m; i++)
        {
            const cd r = *++roots;
            cd *x = values + offset, *y = x + gap;
            for (size_t j = 0; j < gap; j++)
            {
                const cd u = *x, v = *y * r;
                *x++ = u + v;
                *y++ = u - v;
            }
            offset += gap << 1;
        }
        gap >>= 1;
    }
    for (size_t i = 0; i < m; i++)
    {
        const cd r = *++roots;
        const cd u = values[0], v = values[1] * r;
        values[0] = u + v;
        values[1] = u - v;
        values += 2;
    }
}

// a (L words) * s -> out (L words, truncated: every product here is < Q)
void mp_mul_scalar(const u64 *a, size_t L, u64 s, u64 *out)
{
    u64 carry = 0;
    for (size_t k = 0; k < L; k++)
    {
        const u128 p = (u128)a[k] * s + carry;
        out[k] = (u64)p;
        carry = (u64)(p >> 64);
    }
}

bool mp_geq(const u64 *a, const u64 *b, size_t L)
{
    for (size_t k = L; k-- > 0;)
        if (a[k] != b[k]) return a[k] > b[k];
    return true;
}

void mp_sub(u64 *a, const u64 *b, size_t L)
{
    u64 borrow = 0;
    for (size_t k = 0; k < L; k++)
    {
        const u128 d = (u128)a[k] - b[k] - borrow;
        a[k] = (u64)d;
        borrow = (u64)(d >> 64) & 1;
    }
}

u64 inv_mod(u64 a, u64 q)
{
    // extended Euclid on signed 128-bit
    __int128 t = 0, nt = 1, r = q, nr = a % q;
    while (nr)
    {
        const __int128 qq = r / nr, tt = t - qq * nt, rr = r - qq * nr;
        t = nt;
        nt = tt;
        r = nr;
        nr = rr;
    }
    if (t < 0) t += q;
    return (u64)t;
}
} // namespace

extern "C" __attribute__((visibility("default"))) int mhe_ckks_decode(mhe_ctx *c, const mhe_encoder *e,
                                                                     const uint64_t *plain, int limbs, double scale,
                                                                     size_t sparse_slots, double *re, double *im,
                                                                     void *stream)
{
    const PrimeDev *primes;
    const uint64_t *q;
    int K, log_n;
    if (mhe_internal_primes(c, &primes, &q, &K, &log_n)) return mhe_internal_fail(MHE_ERR_ARG, "context is not valid");
    if (!e || e->log_n != log_n) return mhe_internal_fail(MHE_ERR_ARG, "encoder does not match the context");
    if (limbs < 1 || limbs > K || !plain) return mhe_internal_fail(MHE_ERR_ARG, "plain is not valid for encryption parameters");
    if (!re) return mhe_internal_fail(MHE_ERR_ARG, "destination cannot be null");
    if (!sparse_slots) sparse_slots = e->slots;
    if (sparse_slots > e->slots || (sparse_slots & (sparse_slots - 1)))
        return mhe_internal_fail(MHE_ERR_ARG, "sparse_slots must be a power of two <= slots");
    if (scale <= 0 || static_cast<int>(std::log2(scale)) >= total_bits(q, limbs))
        return mhe_internal_fail(MHE_ERR_ARG, "scale out of bounds");
    const size_t n = e->n, L = (size_t)limbs;
    hipStream_t st = (hipStream_t)stream;

    std::vector<u64> x(n * L);
    {
        u64 *tmp = nullptr;
        if (mhe_internal_alloc((void **)&tmp, n * L * sizeof(u64), st) != hipSuccess)
            return mhe_internal_fail(MHE_ERR_MEMORY, "decode staging allocation failed");
        hipError_t err = mhe_internal_copy_d2d(tmp, plain, n * L * sizeof(u64), st);
        int rc = err == hipSuccess ? mhe_ntt_inverse(c, tmp, 1, limbs, 0, stream) : MHE_ERR_DEVICE;
        if (rc == MHE_OK)
        {
            err = hipMemcpyAsync(x.data(), tmp, n * L * sizeof(u64), hipMemcpyDeviceToHost, st);
            if (err == hipSuccess) err = hipStreamSynchronize(st);
            if (err != hipSuccess) rc = MHE_ERR_DEVICE;
        }
        (void)mhe_internal_free(tmp, st);
        if (rc != MHE_OK) return rc == MHE_ERR_DEVICE ? mhe_internal_fail(rc, "decode transfer failed") : rc;
    }

    // RNSBase constants: Q, Q/q_j, (Q/q_j)^{-1} mod q_j
    std::vector<u64> Q(L, 0), punct(L * L, 0), inv_punct(L), tmp(L);
    Q[0] = 1;
    for (size_t j = 0; j < L; j++)
    {
        mp_mul_scalar(Q.data(), L, q[j], tmp.data());
        Q = tmp;
    }
    for (size_t j = 0; j < L; j++)
    {
        u64 *p = &punct[j * L];
        p[0] = 1;
        u64 pm = 1;
        for (size_t k = 0; k < L; k++)
        {
            if (k == j) continue;
            mp_mul_scalar(p, L, q[k], tmp.data());
            std::memcpy(p, tmp.data(), L * sizeof(u64));
            pm = (u64)(((u128)pm * (q[k] % q[j])) % q[j]);
        }
        inv_punct[j] = inv_mod(pm, q[j]);
    }
    std::vector<u64> thr(Q);
    {
        thr[0] += 1; // Q is odd: no carry out of word 0
        for (size_t k = 0; k < L; k++) thr[k] = (thr[k] >> 1) | (k + 1 < L ? thr[k + 1] << 63 : 0);
    }
    const size_t sparsity = e->slots / sparse_slots;
    const double two64 = std::pow(2.0, 64), inv_scale = 1.0 / scale;
    std::vector<cd> res(n);
    std::vector<u64> acc(L);
    for (size_t i = 0; i < n; i++)
    {
        if (sparsity > 1 && ((i - 1) & (sparsity - 1)) != sparsity - 1)
        {
            res[i] = 0.0;
            continue;
        }
        if (L == 1)
            acc[0] = x[i];
        else
        {
            std::fill(acc.begin(), acc.end(), 0);
            for (size_t j = 0; j < L; j++)
            {
                const u64 t = (u64)(((u128)x[j * n + i] * inv_punct[j]) % q[j]);
                mp_mul_scalar(&punct[j * L], L, t, tmp.data());
                u64 carry = 0;
                for (size_t k = 0; k < L; k++)
                {
                    const u128 s = (u128)acc[k] + tmp[k] + carry;
                    acc[k] = (u64)s;
                    carry = (u64)(s >> 64);
                }
                if (carry || mp_geq(acc.data(), Q.data(), L)) mp_sub(acc.data(), Q.data(), L);
            }
        }
        double v = 0.0, s64 = inv_scale;
        if (mp_geq(acc.data(), thr.data(), L))
        {
            for (size_t j = 0; j < L; j++, s64 *= two64)
            {
                if (acc[j] > Q[j])
                {
                    const u64 diff = acc[j] - Q[j];
                    v += diff ? static_cast<double>(diff) * s64 : 0.0;
                }
                else
                {
                    const u64 diff = Q[j] - acc[j];
                    v -= diff ? static_cast<double>(diff) * s64 : 0.0;
                }
            }
        }
        else
        {
            for (size_t j = 0; j < L; j++, s64 *= two64)
                v += acc[j] ? static_cast<double>(acc[j]) * s64 : 0.0;
        }
        res[i] = cd(v, 0.0);
    }
    fft_to_rev(res.data(), log_n, e->root_powers.data());
    for (size_t i = 0; i < sparse_slots; i++)
    {
        const cd z = res[e->index_map[i]];
        re[i] = z.real();
        if (im) im[i] = z.imag();
    }
    return MHE_OK;
}
