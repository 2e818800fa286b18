// CPU test of the Remez exchange restated in seal/boot.cpp (cnn_ckks/common/Remez.cpp with
// ckks_bootstrapping/RemezCos.h):
//   remez_test equi <K> <log_width> <deg> <scale_factor>
//       the minimax polynomial's error must equioscillate: on a dense scan of every interval
//       [i - w, i + w] the local extrema of the error, reduced to runs of one sign, give at least
//       deg + 2 alternating points whose |error| agree up to the rounding of the coefficients to
//       doubles; prints them and the generation time.
//   remez_test coeffs <K> <log_width> <deg> <scale_factor>
//       prints the deg + 1 Chebyshev coefficients (%.17g), one per line.
#include "mhe_boot.h"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

int main(int argc, char **argv)
{
    if (argc < 6)
    {
        std::fprintf(stderr, "usage: remez_test equi|coeffs K log_width deg scale_factor\n");
        return 2;
    }
    if (!std::strcmp(argv[1], "asin"))
    {
        // remez_test asin <log_width of the cosine> <deg> 0 0: ModularReducer's inverse polynomial
        // (ModularReducer.cpp:13-17: RemezArcsin at -log2(sin(2 pi 2^-log_width)))
        const double lw = std::atof(argv[2]);
        RemezArcsin ra(-std::log2(std::sin(2 * M_PI * std::pow(2.0, -lw))), std::atol(argv[3]));
        boot::Polynomial p;
        ra.generate_optimal_poly(p);
        const std::vector<double> &c = p.chebcoeff;
        for (double v : c) std::printf("%.17g\n", v);
        return 0;
    }
    const long K = std::atol(argv[2]), deg = std::atol(argv[4]), sf = std::atol(argv[5]);
    const double lw = std::atof(argv[3]);
    RemezCos rc(K, lw, deg, sf);
    const auto t0 = std::chrono::steady_clock::now();
    int it = 0;
    double spread = 0;
    const std::vector<double> c = rc.chebyshev_coefficients(&it, &spread);
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (!std::strcmp(argv[1], "coeffs"))
    {
        for (double v : c) std::printf("%.17g\n", v);
        return 0;
    }
    boot::Polynomial p;
    p.set_chebyshev(c);
    auto target = [&](long double x) {
        return sf % 2 == 0 ? std::cos(2 * M_PIl * (x - 0.25L) / sf) : std::sin(2 * M_PIl * x / sf);
    };
    auto err = [&](long double x) {
        // long double Clenshaw of the double coefficients
        const long double u = x / K;
        long double b1 = 0, b2 = 0;
        for (long j = deg; j >= 1; j--)
        {
            const long double b0 = 2 * u * b1 - b2 + c[j];
            b2 = b1;
            b1 = b0;
        }
        return u * b1 - b2 + c[0] - target(x);
    };
    const long double w = std::pow(2.0L, -lw);
    std::vector<long double> ext; // signed local extrema (one per run of one sign)
    long double run_best = 0;
    int run_sign = 0;
    const int S = 4096;
    for (long i = -(K - 1); i <= K - 1; i++)
    {
        long double prev2 = 0, prev = 0;
        for (int s = 0; s <= S; s++)
        {
            const long double x = i - w + 2 * w * s / S;
            const long double e = err(x);
            const bool endpt = s == 0 || s == S;
            bool is_ext = false;
            if (endpt)
                is_ext = true;
            if (s >= 2 && ((prev > prev2 && prev >= e) || (prev < prev2 && prev <= e))) is_ext = true;
            auto take = [&](long double v) {
                const int sg = v > 0 ? 1 : -1;
                if (sg != run_sign)
                {
                    if (run_sign) ext.push_back(run_best);
                    run_sign = sg;
                    run_best = v;
                }
                else if (std::fabs(v) > std::fabs(run_best))
                    run_best = v;
            };
            if (is_ext && !endpt && s >= 2) take(prev);
            if (endpt) take(e);
            prev2 = prev;
            prev = e;
        }
    }
    ext.push_back(run_best);
    long double mx = 0, mn = 1e30L;
    for (auto v : ext)
    {
        mx = std::max(mx, std::fabs(v));
        mn = std::min(mn, std::fabs(v));
    }
    std::printf("Remez K=%ld log_width=%g deg=%ld scale_factor=%ld: %d iterations, %.2f s, spread 2^%.1f\n", K, lw, deg,
                sf, it, secs, std::log2(spread));
    std::printf("alternating extrema %zu (need %ld), |error| in [%.12Lg, %.12Lg], relative spread %.3Lg\n", ext.size(),
                deg + 2, mn, mx, (mx - mn) / mn);
    // the coefficients were rounded to doubles: that moves the error by at most sum_j |c_j| 2^-53
    // anywhere, so the alternation levels agree to twice that (the dense scan's own location
    // error, ~ curvature x (2w/S)^2, is far below it)
    long double csum = 0;
    for (double v : c) csum += std::fabs((long double)v);
    const long double bound = 2 * csum * std::ldexp(1.0L, -53) + 1e-18L;
    std::printf("double-rounding bound on the level spread: %.3Lg (observed %.3Lg)\n", bound, mx - mn);
    const bool ok = (long)ext.size() >= deg + 2 && (mx - mn) <= bound;
    std::printf("%s\n", ok ? "ok" : "FAILED");
    return ok ? 0 : 1;
}
