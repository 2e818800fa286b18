// CPU test of the bootstrapping host math (include/mhe_boot.h); no GPU calls.
//  1. The merged CoeffToSlot diagonals (lt_coefficients_3), applied the way the BSGS routines
//     apply them (rotation by offset, 2n-slot extension, conjugate-add), map the slots of a
//     sparse-packed message to its 2n real coefficients / K in bit-reversed order.
//  2. SlotToCoeff (+ rotate-by-n add) maps those coefficient slots back to the message slots.
//  3. The cosine fit on the union of intervals meets the error bound, and the Chebyshev heap
//     division is an identity (p = q T_m + r).
#include "mhe_boot.h"

#include <cmath>
#include <cstring>
#include <cstdio>
#include <random>

using cd = std::complex<double>;
static int g_fail = 0, g_checks = 0;
#define CHECK(cond)                                                                  \
    do                                                                               \
    {                                                                                \
        g_checks++;                                                                  \
        if (!(cond))                                                                 \
        {                                                                            \
            g_fail++;                                                                \
            std::fprintf(stderr, "  FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond); \
        }                                                                            \
    } while (0)

// out[x] = sum_idx G[idx][x] v[(x + off(idx)) mod P]
static std::vector<cd> apply(const boot::LTDiags &G, int step, bool cyclic, const std::vector<cd> &v)
{
    const int P = (int)v.size();
    const int totlen = cyclic ? (int)G.size() - 1 : ((int)G.size() - 1) / 2;
    std::vector<cd> out(P, 0.0);
    for (int idx = 0; idx < (int)G.size(); idx++)
    {
        const int off = (cyclic ? idx : idx - totlen) * step;
        for (int x = 0; x < P; x++) out[x] += G[idx][x % G[idx].size()] * v[((x + off) % P + P) % P];
    }
    return out;
}

static int bitrev(int x, int bits)
{
    int r = 0;
    for (int i = 0; i < bits; i++) r |= ((x >> i) & 1) << (bits - 1 - i);
    return r;
}

static void check_lt(int logn, int logNh, int K)
{
    const int n = 1 << logn;
    boot::LTDiags f1, f2, f3, i1, i2, i3;
    boot::lt_coefficients_3(logn, logNh, K, f1, f2, f3, i1, i2, i3);
    std::mt19937_64 g(logn);
    std::uniform_real_distribution<double> U(-1, 1);
    std::vector<double> t(2 * n);
    for (auto &x : t) x = U(g);
    // slots of the sparse message m(Y) = sum t_j Y^j, Y^{2n} = -1: w_k = sum_j (t_j + i t_{j+n}) zeta^{5^k j}
    std::vector<cd> w(n);
    long p5 = 1;
    for (int k = 0; k < n; k++)
    {
        cd acc = 0;
        for (int j = 0; j < n; j++)
            acc += cd(t[j], t[j + n]) * std::polar(1.0, 2 * M_PI * (double)((p5 * j) % (4 * n)) / (4.0 * n));
        w[k] = acc;
        p5 = (p5 * 5) % (4 * n);
    }
    const double rep = (double)(1 << (logNh - logn)); // subsum factor
    std::vector<cd> v(n);
    for (int k = 0; k < n; k++) v[k] = w[k] * rep;
    // CoeffToSlot (sflinv_3 + conjugate add)
    const int c1 = (int)std::floor(logn / 3.0), c2 = (int)std::floor((logn - c1) / 2.0);
    auto a1 = apply(i1, 1 << (logn - c1), true, v);
    auto a2 = apply(i2, 1 << (logn - c1 - c2), false, a1);
    std::vector<cd> a2d(2 * n);
    for (int x = 0; x < 2 * n; x++) a2d[x] = a2[x % n];
    auto a3 = apply(i3, 1, false, a2d);
    double err = 0;
    std::vector<cd> r(2 * n);
    for (int x = 0; x < 2 * n; x++)
    {
        r[x] = a3[x] + std::conj(a3[x]);
        const int j = bitrev(x % n, logn) + (x >= n ? n : 0);
        err = std::max(err, std::abs(r[x] - cd(t[j] / K, 0)));
    }
    std::printf("logn %d: CoeffToSlot max error %.3g\n", logn, err);
    CHECK(err < 1e-12);
    // SlotToCoeff (sfl_half_3 without the runtime scale) + rotate by n and add
    const int s3 = (int)std::floor(logn / 3.0), s2 = (int)std::floor((logn - s3) / 2.0), s1 = logn - s3 - s2;
    auto b1 = apply(f1, 1, false, r);
    auto b2 = apply(f2, 1 << s1, false, b1);
    auto b3 = apply(f3, 1 << (s1 + s2), false, b2);
    double err2 = 0;
    for (int x = 0; x < n; x++) err2 = std::max(err2, std::abs((b3[x] + b3[x + n]) * (double)K - w[x]));
    std::printf("logn %d: SlotToCoeff round trip max error %.3g\n", logn, err2);
    CHECK(err2 < 1e-9 * n);
    // rotation-step set covers every BSGS step (addLeftRotKeys_Linear_to_vector_3 via a stub)
    CHECK(f1.size() == (size_t)(2 * ((1 << s1) - 1) + 1));
    CHECK(i1.size() == (size_t)(1 << c1));
}

// ULPs between two doubles of the same sign (0 when equal)
static long ulps(double a, double b)
{
    if (a == b) return 0;
    if ((a < 0) != (b < 0)) return 1L << 62;
    long ia, ib;
    std::memcpy(&ia, &a, 8);
    std::memcpy(&ib, &b, 8);
    return std::labs(ia - ib);
}

// The reference-order diagonals (lt_coefficients_3: genfftcoeff_3 / geninvfftcoeff_3's loops) against
// the independent sparse-matrix derivation (lt_coefficients_3_merged): same shapes, and every double
// within a few ULPs of the other relative to the diagonal's scale -- the two sum the same products in
// different orders.  Reports how many doubles differ at all.
static void check_lt_orders(int logn, int logNh, int K)
{
    boot::LTDiags a[6], b[6];
    boot::lt_coefficients_3(logn, logNh, K, a[0], a[1], a[2], a[3], a[4], a[5]);
    boot::lt_coefficients_3_merged(logn, logNh, K, b[0], b[1], b[2], b[3], b[4], b[5]);
    long total = 0, differ = 0, max_ulp = 0;
    double max_rel = 0;
    for (int g = 0; g < 6; g++)
    {
        CHECK(a[g].size() == b[g].size());
        for (std::size_t i = 0; i < std::min(a[g].size(), b[g].size()); i++)
        {
            CHECK(a[g][i].size() == b[g][i].size());
            double scale = 0;
            for (const cd &z : a[g][i]) scale = std::max(scale, std::abs(z));
            for (std::size_t x = 0; x < std::min(a[g][i].size(), b[g][i].size()); x++)
                for (int part = 0; part < 2; part++)
                {
                    const double u = part ? a[g][i][x].imag() : a[g][i][x].real();
                    const double v = part ? b[g][i][x].imag() : b[g][i][x].real();
                    total++;
                    if (u != v)
                    {
                        differ++;
                        if (std::abs(u) > 1e-3 * scale) max_ulp = std::max(max_ulp, ulps(u, v));
                        max_rel = std::max(max_rel, std::abs(u - v) / (scale > 0 ? scale : 1.0));
                    }
                }
        }
    }
    std::printf("logn %d (logNh %d): reference-order vs merged diagonals: %ld of %ld doubles differ, max %ld ULP "
                "(entries above 1e-3 of their diagonal), max |diff| / scale %.3g\n",
                logn, logNh, differ, total, max_ulp, max_rel);
    CHECK(max_rel < 1e-14);
}

int main()
{
    for (int logn : { 3, 5, 6, 8 }) check_lt(logn, 10, 25);
    for (int logn : { 3, 5, 6, 8, 10 }) check_lt_orders(logn, 10, 25);
    check_lt_orders(14, 15, 25); // the ResNet bootstrapper_1 shape (logn 14, N = 2^16)
    check_lt_orders(12, 15, 25);

    // cosine approximation of the ResNet setting (cnn/infer_seal.cpp:289-296): K = 25, deg 59,
    // log width 10, two double-angle steps (cos(2 pi (x - 1/4) / 4))
    RemezCos rc(25, 10.0, 59, 4);
    boot::Polynomial p;
    rc.generate_optimal_poly(p);
    const double e = rc.max_error(p);
    std::printf("cosine fit: deg %ld, max error %.3g (2^%.1f)\n", p.deg, e, std::log2(e));
    CHECK(p.deg == 59);
    CHECK(e < std::pow(2.0, -28));
    double cmax = 0;
    for (double c : p.chebcoeff) cmax = std::max(cmax, std::abs(c));
    CHECK(cmax < 2.0);

    // heap: the ResNet shape and the identity p = q T_m + r at every internal node
    p.generate_poly_heap();
    std::printf("heap k=%ld m=%ld len=%ld\n", p.heap_k, p.heap_m, p.heaplen);
    CHECK(p.heap_k * (1L << p.heap_m) > p.deg);
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> U(-1, 1);
    long chebdeg = p.heap_k << p.heap_m;
    for (long lvl = 0; lvl < p.heap_m; lvl++)
    {
        chebdeg >>= 1;
        for (long j = (1L << lvl) - 1; j < (1L << (lvl + 1)) - 1; j++)
        {
            if (!p.poly_heap[j] || !p.poly_heap[2 * (j + 1) - 1]) continue;
            for (int s = 0; s < 20; s++)
            {
                const double x = U(g);
                const double tm = std::cos(chebdeg * std::acos(x));
                const double lhs = p.poly_heap[j]->evaluate(x);
                const double rhs = p.poly_heap[2 * (j + 1) - 1]->evaluate(x) * tm + p.poly_heap[2 * (j + 1)]->evaluate(x);
                CHECK(std::abs(lhs - rhs) < 1e-9);
            }
        }
    }
    // linear arcsine (inverse_deg 1): slope within (1/2pi, asin(a)/(2 pi a))
    RemezArcsin ra(-std::log2(std::sin(2 * M_PI * std::pow(2.0, -10))), 1);
    boot::Polynomial q;
    ra.generate_optimal_poly(q);
    const double a = std::sin(2 * M_PI * std::pow(2.0, -10));
    std::printf("arcsine slope %.17g\n", q.coeff[1]);
    CHECK(q.coeff[1] > 1 / (2 * M_PI) && q.coeff[1] < std::asin(a) / (2 * M_PI * a));

    std::printf("%d checks, %d failed\n", g_checks, g_fail);
    return g_fail ? 1 : 0;
}
