// GPU tests of the GPT-2 layer (include/mhe_gpt2.h) at the reference's GPT-2 parameters
// (gpt2/util.h INIT(): N = 2^16, {49} + 21 x {46} + 14 x {49} + {60 special}, hamming weight 192,
// scale 2^46).  Two kinds of checks:
//  * the reference's own doctest cases with their expected values (gpt2_ckks/run/
//    run_approx_test.cpp: SignFunctionF :362, SignFunctionG :387, SignFunction :412, GeluP :441,
//    GeluQ :464, Goldschmidt :490, Exp :537, QuickSum :563, RowMatMul :231), compared with
//    doctest::Approx's rule |a - b| < 1.19e-5 (1 + max(|a|, |b|)) -- or 1e-3 absolute where the
//    reference's expected value is the exact function rather than the approximation;
//  * config C5's bar: the decrypted approximation over all 32768 slots within 1e-3 of the same
//    polynomial evaluated in plain doubles (the plain restatement below).
#include "mhe_boot.h"
#include "mhe_gpt2.h"

#include "../../include/mhe.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <random>
#include <string>
#include <unordered_map>

using namespace seal;
using namespace gpt2;

static int g_fail = 0;

static bool approx(double a, double b) { return std::fabs(a - b) < 1.1920929e-5 * (1 + std::max(std::fabs(a), std::fabs(b))); }

static void report(const std::string &name, bool ok, double err, double secs)
{
    std::printf("[%s] %s  max err %.3g  (%.3f s enqueue)\n", ok ? "PASS" : "FAIL", name.c_str(), err, secs);
    if (!ok) g_fail++;
}

// ---------------------------------------------------------------- plain restatement (doubles)
static double T2(double x) { return 2 * x * x - 1; }
static double T3(double x) { return 2 * x * T2(x) - x; }
static double T4(double x) { return 2 * T2(x) * T2(x) - 1; }
static double T8(double x) { return 2 * T4(x) * T4(x) - 1; }
static double sign_poly(double x, double fq1, double fr1, double frq2_q, double frq2_r, double fq3)
{
    return fq1 * x * T2(x) + fr1 * x + (frq2_q * T3(x) + frq2_r * x) * T4(x) + fq3 * x * T8(x);
}
static double plain_f(double x) { return sign_poly(x, -0.6767578125, 1.563049316, -0.02685546875, 0.1384277344, 0.002136230469); }
static double plain_g(double x) { return sign_poly(x, -1.121704102, 1.978370667, -0.6178588867, 0.403533935, 0.3557052612); }
static double plain_sign(double x) { return plain_f(plain_f(plain_g(plain_g(x)))); }
static double plain_gelu_p(double x) { return (-0.005337069175 * x - 0.05745879353) * T2(x) + (-0.4187418723 * x - 0.55528939); }
static double plain_gelu_q(double x)
{
    return (-0.00324699876 * x + 0.1634058825) * T2(x) + (0.5027208006 * x + 0.1750485092) +
           (0.0001533078376 * x * x + 0.0002609111473 * x - 0.004401064777) * T4(x);
}

static int run_all(int log_scale);

int main(int argc, char **argv)
{
    std::setvbuf(stdout, nullptr, _IONBF, 0);
    try
    {
        return run_all(argc > 1 ? std::atoi(argv[1]) : LOGQ);
    }
    catch (const std::exception &e)
    {
        std::printf("exception: %s\nFAILED\n", e.what());
        return 1;
    }
}

static int run_all(int log_scale)
{
    const long logN = 16;
    const int logp = LOGP, logq = LOGQ, log_special_prime = 60, remaining_level = 21, boot_level = BOOT_LEVEL;
    EncryptionParameters params(scheme_type::ckks);
    std::vector<int> bits{ logq };
    for (int i = 0; i < remaining_level; i++) bits.push_back(logp);
    for (int i = 0; i < boot_level; i++) bits.push_back(logq);
    bits.push_back(log_special_prime);
    const std::size_t n = (std::size_t)1 << logN;
    params.set_poly_modulus_degree(n);
    params.set_coeff_modulus(CoeffModulus::Create(n, bits));
    params.set_secret_key_hamming_weight(192);
    const double scale = std::pow(2.0, log_scale);
    std::printf("input scale 2^%d\n", log_scale);
    const auto t0 = std::chrono::steady_clock::now();
    SEALContext context(params);
    KeyGenerator keygen(context);
    PublicKey public_key;
    RelinKeys relin_keys;
    GaloisKeys gal_keys;
    keygen.create_public_key(public_key);
    keygen.create_relin_keys(relin_keys);
    // INIT()'s steps plus the right-rotations by 1..16 (steps 32752..32767): the reference list lacks
    // 32764/32763/32762, so SEAL -- and this library -- raise "Galois key not present" for the
    // rotation by -4 inside RowMatMul (MatrixMul.cpp:180, NAF of -4 is a single term)
    std::vector<int> steps = gpt2_rotation_steps((int)logN);
    for (int k = 1; k <= 16; k++)
        if (std::find(steps.begin(), steps.end(), 32768 - k) == steps.end()) steps.push_back(32768 - k);
    // GPT2_QKV=1 adds the qk/sv attention matmul cases, and with them sv_matmul's rotations by
    // rots*256 (MatrixMul.cpp:551), which INIT()'s list also lacks
    const bool qkv = std::getenv("GPT2_QKV") != nullptr;
    if (qkv)
        for (int r = 1; r < 64; r++)
            if (std::find(steps.begin(), steps.end(), r * 256) == steps.end()) steps.push_back(r * 256);
    keygen.create_galois_keys(steps, gal_keys);
    set_encode_scale(std::pow(2.0, log_scale));
    CKKSEncoder encoder(context);
    Encryptor encryptor(context, public_key);
    Evaluator evaluator(context, encoder);
    Decryptor decryptor(context, keygen.secret_key());
    std::printf("setup (GPT-2 chain, %zu primes): %.2f s\n", bits.size(),
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());

    auto enc = [&](const std::vector<double> &v) {
        Plaintext p;
        Ciphertext c;
        encoder.encode(v, scale, p);
        encryptor.encrypt(p, c);
        return c;
    };
    auto dec = [&](const Ciphertext &c) {
        Plaintext p;
        std::vector<double> v;
        decryptor.decrypt(c, p);
        encoder.decode(p, v);
        return v;
    };
    using Fn = std::function<void(Ciphertext &, Ciphertext &)>;
    auto timed = [&](const Fn &f, Ciphertext &in, Ciphertext &out) {
        const auto s = std::chrono::steady_clock::now();
        f(in, out);
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - s).count();
    };
    // reference doctest case: inputs, expected outputs, doctest::Approx
    auto doctest_case = [&](const std::string &name, const Fn &f, std::vector<double> v, const std::vector<double> &expect,
                            double abs_tol = 0) {
        std::printf("-- %s\n", name.c_str());
        Ciphertext in = enc(v), out;
        const double s = timed(f, in, out);
        const auto got = dec(out);
        bool ok = true;
        double err = 0;
        for (std::size_t i = 0; i < expect.size(); i++)
        {
            err = std::max(err, std::fabs(got[i] - expect[i]));
            ok &= abs_tol > 0 ? std::fabs(got[i] - expect[i]) < abs_tol : approx(got[i], expect[i]);
        }
        std::printf("  out: %zu limbs, scale 2^%.2f, got", out.coeff_modulus_size(), std::log2(out.scale()));
        for (std::size_t i = 0; i < expect.size(); i++) std::printf(" %.6g", got[i]);
        std::printf("\n");
        report(name + " (run_approx_test.cpp)", ok, err, s);
    };
    // C5 bar: all slots vs the plain restatement within 1e-3
    std::mt19937_64 rng(2026);
    auto plain_case = [&](const std::string &name, const Fn &f, double (*ref)(double), double lo, double hi) {
        std::printf("-- %s\n", name.c_str());
        std::uniform_real_distribution<double> U(lo, hi);
        std::vector<double> v(encoder.slot_count());
        for (auto &x : v) x = U(rng);
        Ciphertext in = enc(v), out;
        const double s = timed(f, in, out);
        const auto got = dec(out);
        double err = 0;
        for (std::size_t i = 0; i < v.size(); i++) err = std::max(err, std::fabs(got[i] - ref(v[i])));
        std::printf("  %s: output level %zu limbs\n", name.c_str(), out.coeff_modulus_size());
        report(name + " vs plain restatement, 32768 slots", err < 1e-3, err, s);
    };

    {
        // primitive checks on this chain (60-bit special prime: integer key switching)
        std::vector<double> v(encoder.slot_count());
        for (std::size_t i = 0; i < v.size(); i++) v[i] = std::sin(0.001 * (double)i);
        Ciphertext x = enc(v), t;
        auto maxerr = [&](const Ciphertext &c, const std::function<double(double)> &ref) {
            const auto got = dec(c);
            double e = 0;
            for (std::size_t i = 0; i < v.size(); i++) e = std::max(e, std::fabs(got[i] - ref(v[i])));
            return e;
        };
        double e0 = maxerr(x, [](double a) { return a; });
        evaluator.multiply_const(x, 0.5, t);
        evaluator.rescale_to_next_inplace(t);
        double e1 = maxerr(t, [](double a) { return 0.5 * a; });
        evaluator.add_const_inplace(t, 0.25);
        double e2 = maxerr(t, [](double a) { return 0.5 * a + 0.25; });
        evaluator.square(x, t);
        double e3a = maxerr(t, [](double a) { return a * a; });
        evaluator.relinearize_inplace(t, relin_keys);
        double e3b = maxerr(t, [](double a) { return a * a; });
        evaluator.rescale_to_next_inplace(t);
        double e3 = maxerr(t, [](double a) { return a * a; });
        evaluator.rotate_vector(x, 1, gal_keys, t);
        const auto r = dec(t);
        double e4 = 0;
        for (std::size_t i = 0; i + 1 < v.size(); i++) e4 = std::max(e4, std::fabs(r[i] - v[i + 1]));
        std::printf("primitives: enc %.3g, mulconst+rescale %.3g, addconst %.3g, square(size3) %.3g, relin %.3g, "
                    "rescale %.3g, rotate %.3g\n", e0, e1, e2, e3a, e3b, e3, e4);
        report("primitives on the GPT-2 chain", std::max({ e0, e1, e2, e3a, e3b, e3, e4 }) < 1e-6, std::max({ e0, e1, e2, e3a, e3b, e3, e4 }), 0);
    }
    Fn sign_f = [&](Ciphertext &i, Ciphertext &o) { compute_sign_f(i, o, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys); };
    Fn sign_g = [&](Ciphertext &i, Ciphertext &o) { compute_sign_g(i, o, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys); };
    Fn sign = [&](Ciphertext &i, Ciphertext &o) { sign_function(i, o, 2, 2, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys); };
    Fn gelu_p = [&](Ciphertext &i, Ciphertext &o) { compute_gelu_p(i, o, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys); };
    Fn gelu_q = [&](Ciphertext &i, Ciphertext &o) { compute_gelu_q(i, o, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys); };
    Fn expf = [&](Ciphertext &i, Ciphertext &o) { compute_exp(i, o, 6, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys); };
    Fn inv = [&](Ciphertext &i, Ciphertext &o) { compute_inverse(i, o, 8, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys); };
    Fn qsum = [&](Ciphertext &i, Ciphertext &o) { quickSum(i, o, 8, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys); };

    doctest_case("SignFunctionF", sign_f, { -0.4, 0.5, -1, 1 }, { -0.80238268, 0.9021453857, -1.0, 1.0 });
    doctest_case("SignFunctionG", sign_g, { -0.4, 0.5, -1, 1 }, { -0.899779538, 0.7708721161, -0.998046875, 0.998046875 });
    // the reference expects sign() itself here; the composite reaches it to ~1e-3 at 0.01
    doctest_case("SignFunction", sign, { -0.4, 0.5, 0.01, -0.02 }, { -1, 1, 0.98683881, -0.9999994 }, 2e-3);
    doctest_case("GeluP", gelu_p, { -0.4, 0.5, 1, -1 }, { -0.3501723443, -0.7345966621, -1.036827125, -0.188669242 });
    doctest_case("GeluQ", gelu_q, { -3, 5, 1, -1 }, { -0.5845409261, 13.43445935, 0.8339413477, -0.1655280783 });
    doctest_case("Exp", expf, { 2, -0.05, 10 }, { 7.166276152788219, 0.9512108363005606, 10847.05214173728 });
    {
        std::vector<double> v = { 0.0035, 0.4, 0.67, 2.23284 };
        v.resize(32768, 2.0);
        // The reference's expected vector (169.269..., 2.5, 1.4925) does not follow from its own
        // compute_inverse (n0 = 0.001, d0 = 0.001 x, 8 steps reach only ~0.256 for x = 0.4), so the
        // check is against that iteration restated in doubles, within 1e-3 relative.
        Ciphertext in = enc(v), out;
        const double s = timed(inv, in, out);
        const auto got = dec(out);
        double err = 0;
        bool ok = true;
        for (int i = 0; i < 4; i++)
        {
            double nn = 0.001, d = 0.001 * v[i];
            for (int k = 0; k < 8; k++)
            {
                const double f = 2 - d;
                nn *= f;
                d *= f;
            }
            err = std::max(err, std::fabs(got[i] - nn) / nn);
            ok &= std::fabs(got[i] - nn) < 1e-3 * nn;
        }
        report("Goldschmidt compute_inverse(8) vs plain restatement (relative)", ok, err, s);
    }
    {
        std::vector<double> v = { 1, 2, 3, 4, 5, 6, 7, 8, 1, 2, 3, 4, 5, 6, 7, 8 };
        Ciphertext in = enc(v), out;
        const double s = timed(qsum, in, out);
        const auto got = dec(out);
        double err = 0;
        bool ok = true;
        for (int i = 0; i < 8; i++)
        {
            err = std::max(err, std::fabs(got[i] - 36.0));
            ok &= approx(got[i], 36.0);
        }
        report("QuickSum (run_approx_test.cpp)", ok, err, s);
    }
    plain_case("compute_sign_g", sign_g, plain_g, -1, 1);
    plain_case("compute_sign_f", sign_f, plain_f, -1, 1);
    plain_case("sign_function(2,2)", sign, plain_sign, -1, 1);
    plain_case("compute_gelu_p", gelu_p, plain_gelu_p, -1, 1);
    plain_case("compute_gelu_q", gelu_q, plain_gelu_q, -2, 2);
    {
        // compute_smax (PolyApprox.cpp:595-649) vs the same pipeline restated in doubles:
        // rotate_vector(x, k)[i] = x[(i + k) mod 32768]; quickSum as Fold.cpp:20-45
        const int S = 32768, gamma = 2;
        auto rot = [&](const std::vector<double> &x, int k) {
            std::vector<double> y(S);
            for (int i = 0; i < S; i++) y[i] = x[((i + k) % S + S) % S];
            return y;
        };
        auto qsum = [&](const std::vector<double> &x, int nn) {
            std::vector<double> o(S), r1 = rot(x, 1);
            for (int i = 0; i < S; i++) o[i] = x[i] + r1[i];
            for (int acc = 2; acc < nn; acc *= 2)
            {
                const auto ro = rot(o, acc);
                for (int i = 0; i < S; i++) o[i] += ro[i];
            }
            return o;
        };
        std::uniform_real_distribution<double> U(-1, 1);
        std::vector<double> v(S, 0.0);
        for (int i = 0; i < 128; i++)
            for (int j = 0; j < 128; j++) v[i * 256 + j] = U(rng);
        std::vector<double> e(S), want(S);
        for (int i = 0; i < S; i++)
        {
            const bool pad = (i % 256) >= 128;
            e[i] = pad ? 0.0 : std::pow(1 + v[i] / 64.0, 64);
        }
        auto rolled = rot(e, S - 128);
        for (int i = 0; i < S; i++) rolled[i] += e[i];
        const auto summed = qsum(rolled, 128);
        for (int i = 0; i < S; i++)
        {
            double nn = 0.001, d = 0.001 * summed[i];
            for (int k = 0; k < 4; k++)
            {
                const double f = 2 - d;
                nn *= f;
                d *= f;
            }
            want[i] = e[i] * nn;
        }
        std::printf("-- compute_smax\n");
        Ciphertext c = enc(v);
        const auto t = std::chrono::steady_clock::now();
        compute_smax(c, 6, gamma, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
        const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
        const auto got = dec(c);
        double err = 0;
        for (int i = 0; i < S; i++) err = std::max(err, std::fabs(got[i] - want[i]));
        std::printf("  compute_smax: output %zu limbs\n", c.coeff_modulus_size());
        report("compute_smax(gamma 2) vs plain restatement, 32768 slots", err < 1e-3, err, secs);
    }
    {
        // Bootstrapped pieces on a full-slot Bootstrapper (logn = 15, run_approx_test.cpp's constants:
        // loge 10, K 25, cosine degree 59, 2 double angles, inverse degree 1): computeMax (Fold.cpp:47-88),
        // quickMax (:91-110) and compute_softmax (PolyApprox.cpp:533-593), each against the same
        // operation sequence restated in doubles with bootstrapping taken as the identity
        // INIT()'s scale 2^LOGP (util.h:53), and every input dropped to TOTAL_LEVEL - BOOT_LEVEL = 21 limbs
        // as the QuickMax doctest does: the levels a bootstrap refreshes, all 46-bit primes, where the
        // 2^46 scale is stable (in the 49-bit boot levels each rescale of a 2^46 product loses 3 bits)
        const int S = 32768;
        const double saved_scale = encode_scale(), bscale = std::pow(2.0, LOGP);
        set_encode_scale(bscale);
        auto enc = [&](const std::vector<double> &v) {
            Plaintext p;
            Ciphertext c;
            encoder.encode(v, bscale, p);
            encryptor.encrypt(p, c);
            while ((int)c.coeff_modulus_size() > remaining_level) evaluator.mod_switch_to_next_inplace(c);
            return c;
        };
        Bootstrapper bt(10, (long)logN - 1, (long)logN - 1, remaining_level + boot_level, bscale, 25, 59, 2, 1,
                        context, keygen, encoder, encryptor, decryptor, evaluator, relin_keys, gal_keys);
        std::vector<int> bsteps;
        for (int i = 0; i < (int)logN - 1; i++) bsteps.push_back(1 << i);
        const auto tb = std::chrono::steady_clock::now();
        init_bootstrap(bt, bsteps, (int)logN - 1);
        std::vector<int> missing;
        for (int st : bsteps)
            if (!gal_keys.has_key(seal::GaloisKeys::get_index(mhe_galois_elt_from_step((int)logN, st))))
                missing.push_back(st);
        keygen.create_galois_keys(missing, gal_keys);
        std::printf("full-slot bootstrapper: %zu extra Galois keys, %.2f s\n", missing.size(),
                    std::chrono::duration<double>(std::chrono::steady_clock::now() - tb).count());
        auto rot = [&](const std::vector<double> &x, int k) {
            std::vector<double> y(S);
            for (int i = 0; i < S; i++) y[i] = x[((i + k) % S + S) % S];
            return y;
        };
        auto pmax = [&](const std::vector<double> &a, const std::vector<double> &b) {
            std::vector<double> o(S);
            for (int i = 0; i < S; i++) o[i] = 0.5 * ((a[i] - b[i]) * plain_sign(0.1 * (a[i] - b[i])) + a[i] + b[i]);
            return o;
        };
        auto maxerr = [&](const std::vector<double> &got, const std::vector<double> &want) {
            double e = 0;
            for (int i = 0; i < S; i++) e = std::max(e, std::fabs(got[i] - want[i]));
            return e;
        };
        std::uniform_real_distribution<double> U(-1, 1);
        {
            // bootstrap() accuracy against its prescale kappa, for |x| <= 1 and |x| <= 4 (kappa = 1 is the
            // reference's util.cpp:318 behaviour)
            const double saved_kappa = bootstrap_prescale();
            for (double range : { 1.0, 4.0 })
                for (double kappa : { 1.0, 8.0, 32.0, 128.0, 512.0 })
                {
                    set_bootstrap_prescale(kappa);
                    std::vector<double> v(S);
                    for (auto &x : v) x = range * U(rng);
                    Ciphertext c = enc(v), out;
                    while ((int)c.coeff_modulus_size() > 3) evaluator.mod_switch_to_next_inplace(c);
                    bootstrap(c, out, bt, evaluator);
                    const auto got = dec(out);
                    double e = 0;
                    for (int i = 0; i < S; i++) e = std::max(e, std::fabs(got[i] - v[i]));
                    std::printf("   bootstrap |x| <= %.0f, kappa %4.0f: max err %.3g, %zu limbs out\n", range, kappa, e,
                                out.coeff_modulus_size());
                }
            {
                // a ciphertext rescaled (not dropped) into its last limb, bootstrapped as is
                set_bootstrap_prescale(1.0);
                std::vector<double> v(S);
                for (auto &x : v) x = U(rng);
                Ciphertext c = enc(v), out;
                while ((int)c.coeff_modulus_size() > 2) evaluator.mod_switch_to_next_inplace(c);
                evaluator.multiply_const_inplace(c, 1.0);
                evaluator.rescale_to_next_inplace(c);
                const double s_in = c.scale();
                bootstrap(c, out, bt, evaluator);
                const auto got = dec(out);
                double e = 0;
                for (int i = 0; i < S; i++) e = std::max(e, std::fabs(got[i] - v[i]));
                std::printf("   bootstrap of a rescaled 1-limb ciphertext (scale 2^%.4f): max err %.3g\n", std::log2(s_in), e);
            }
            set_bootstrap_prescale(saved_kappa);
        }
        {
            // the reference's ComputeMax doctest inputs, then all slots random
            std::vector<double> a(S), b(S);
            const double d1[5] = { 0.1, 0.5, 0.003, 0.4, -0.2 }, d2[5] = { 0.3, 0.1, 0.1, -0.6, 0.0001 };
            for (int i = 0; i < S; i++)
            {
                a[i] = i < 5 ? d1[i] : U(rng);
                b[i] = i < 5 ? d2[i] : U(rng);
            }
            Ciphertext ca = enc(a), cb = enc(b), out;
            const auto t = std::chrono::steady_clock::now();
            computeMax(ca, cb, out, bt, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
            const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
            const auto got = dec(out);
            std::printf("-- computeMax: doctest slots %.5f %.5f %.5f %.5f %.5f (expected ~0.3 0.5 0.1 0.4 0.0001), "
                        "%zu limbs\n", got[0], got[1], got[2], got[3], got[4], out.coeff_modulus_size());
            report("computeMax vs plain restatement, 32768 slots", maxerr(got, pmax(a, b)) < 1e-3, maxerr(got, pmax(a, b)),
                   secs);
        }
        {
            // QuickMax doctest values: maxima over 8 consecutive slots (run_approx_test.cpp:621-653); each
            // round ends below 18 limbs and runs a real bootstrap_3
            std::vector<double> v(S);
            for (int i = 0; i < S; i++) v[i] = i < 16 ? 0.1 * (1 + i % 8) : U(rng);
            Plaintext pv;
            Ciphertext c, out;
            encoder.encode(v, bscale, pv);
            encryptor.encrypt(pv, c);
            // one level above the doctest's 21 limbs, so the first bootstrap (at 2 limbs) can prescale
            while ((int)c.coeff_modulus_size() > remaining_level + 1) evaluator.mod_switch_to_next_inplace(c);
            const auto t = std::chrono::steady_clock::now();
            quickMax(c, out, 8, bt, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
            const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
            auto want = v;
            for (int acc = 1; acc < 8; acc *= 2) want = pmax(want, rot(want, acc));
            const auto got = dec(out);
            std::printf("-- quickMax(8): first slots %.5f %.5f (doctest expects 0.8), %zu limbs\n", got[0], got[1],
                        out.coeff_modulus_size());
            report("quickMax(8) vs plain restatement, 32768 slots", maxerr(got, want) < 1e-3, maxerr(got, want), secs);
        }
        {
            // compute_softmax on rows of 128 scores at slot i*256
            std::vector<double> v(S, 0.0);
            for (int i = 0; i < 128; i++)
                for (int j = 0; j < 128; j++) v[i * 256 + j] = U(rng);
            auto x = v;
            {
                const auto r = rot(v, 32640);
                for (int i = 0; i < S; i++) x[i] += r[i];
            }
            auto mx = x;
            for (int acc = 1; acc < 128; acc *= 2) mx = pmax(mx, rot(mx, acc));
            std::vector<double> e(S), want(S);
            for (int i = 0; i < S; i++)
            {
                const bool pad = (i % 256) >= 128;
                e[i] = pad ? 0.0 : std::pow(1 + (x[i] - mx[i]) / 64.0, 64);
            }
            auto rolled = rot(e, -128);
            for (int i = 0; i < S; i++) rolled[i] += e[i];
            auto summed = rolled;
            {
                auto r1 = rot(summed, 1);
                for (int i = 0; i < S; i++) summed[i] += r1[i];
                for (int acc = 2; acc < 128; acc *= 2)
                {
                    const auto ro = rot(summed, acc);
                    for (int i = 0; i < S; i++) summed[i] += ro[i];
                }
            }
            double softmax_err = 0;
            for (int i = 0; i < S; i++)
            {
                double nn = 0.001, d = 0.001 * summed[i];
                for (int k = 0; k < 4; k++)
                {
                    const double f = 2 - d;
                    nn *= f;
                    d *= f;
                }
                want[i] = e[i] * nn;
            }
            for (int r = 0; r < 128; r++)
            {
                // against the exact softmax of the row (the approximation's own error, reported)
                double m = -1e9, z = 0;
                for (int j = 0; j < 128; j++) m = std::max(m, v[r * 256 + j]);
                for (int j = 0; j < 128; j++) z += std::exp(v[r * 256 + j] - m);
                for (int j = 0; j < 128; j++)
                    softmax_err = std::max(softmax_err, std::fabs(want[r * 256 + j] - std::exp(v[r * 256 + j] - m) / z));
            }
            Ciphertext c = enc(v);
            const auto t = std::chrono::steady_clock::now();
            compute_softmax(c, 6, bt, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
            const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
            const auto got = dec(c);
            std::printf("-- compute_softmax: %zu limbs out; the restated pipeline is within %.2g of the exact "
                        "softmax\n", c.coeff_modulus_size(), softmax_err);
            report("compute_softmax (bootstrapped quickMax) vs plain restatement, 32768 slots", maxerr(got, want) < 1e-3,
                   maxerr(got, want), secs);
        }
        set_encode_scale(saved_scale);
    }
    {
        // compute_inv_sqrt (IterApprox.cpp:128-166) and compute_layernorm (:168-246) vs the same
        // operation sequences restated in doubles (taylor_expand as written, :69-120; Newton with
        // fakeBootstrap; layernorm's y * z product and first-row beta as written -- DESIGN.md §8)
        const int S = 32768, row = 768, R = 1024;
        const double guess = 323251;
        auto rot = [&](const std::vector<double> &x, int k) {
            std::vector<double> y(S);
            for (int i = 0; i < S; i++) y[i] = x[((i + k) % S + S) % S];
            return y;
        };
        auto qsum = [&](const std::vector<double> &x, int nn) {
            std::vector<double> o(S), r1 = rot(x, 1);
            for (int i = 0; i < S; i++) o[i] = x[i] + r1[i];
            for (int acc = 2; acc < nn; acc *= 2)
            {
                const auto ro = rot(o, acc);
                for (int i = 0; i < S; i++) o[i] += ro[i];
            }
            return o;
        };
        auto plain_inv_sqrt = [&](double a) {
            double x = -0.5 * (a * std::pow(guess, -1.5)) + 0.375 * std::pow(a * std::pow(guess, -1.25), 2) -
                       0.3125 * std::pow(a * std::pow(guess, -3.5 / 3), 3);
            for (int k = 0; k < 4; k++) x = x * ((x * x) * (-0.5 * a) + 1.5);
            return x;
        };
        {
            std::uniform_real_distribution<double> A(0.6 * guess, 1.6 * guess);
            std::vector<double> a(S), want(S);
            for (int i = 0; i < S; i++) want[i] = plain_inv_sqrt(a[i] = A(rng));
            std::printf("-- compute_inv_sqrt\n");
            Ciphertext c = enc(a), o;
            const auto t = std::chrono::steady_clock::now();
            compute_inv_sqrt(c, o, 4, guess, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
            const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
            const auto got = dec(o);
            double err = 0;
            for (int i = 0; i < S; i++) err = std::max(err, std::fabs(got[i] - want[i]) / std::fabs(want[i]));
            report("compute_inv_sqrt(4, 323251) vs plain restatement, 32768 slots (relative)", err < 1e-3, err, secs);
        }
        {
            std::uniform_real_distribution<double> X(-0.05, 0.05), G(0.5, 1.5), B(-0.5, 0.5);
            std::vector<double> x(S, 0.0), gamma(row), beta(row), mask(S, 0.0), mulf(S, 0.0), betap(S, 0.0);
            for (auto &g : gamma) g = G(rng);
            for (auto &b : beta) b = B(rng);
            for (int i = 0; i < 16; i++)
                for (int j = 0; j < row; j++) x[i * 2 * R + j] = X(rng);
            for (int i = 0; i < 16; i++)
                for (int j = 0; j < R; j++)
                {
                    mask[i * 2 * R + j] = 1.0;
                    if (j < row) mulf[i * 2 * R + j] = gamma[j] * std::sqrt((double)row);
                }
            for (int j = 0; j < row; j++) betap[j] = beta[j];
            auto rolled = rot(x, -R);
            for (int i = 0; i < S; i++) rolled[i] += x[i];
            const auto folded = qsum(rolled, R);
            std::vector<double> want(S);
            double wmax = 0;
            for (int i = 0; i < S; i++)
            {
                const double z = row * x[i] - folded[i];
                want[i] = (z * z * mask[i]) * z * mulf[i] + betap[i];
                wmax = std::max(wmax, std::fabs(want[i]));
            }
            std::printf("-- compute_layernorm\n");
            Ciphertext c = enc(x), o;
            const auto t = std::chrono::steady_clock::now();
            compute_layernorm(c, o, gamma, beta, row, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
            const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
            const auto got = dec(o);
            double err = 0;
            for (int i = 0; i < S; i++) err = std::max(err, std::fabs(got[i] - want[i]));
            std::printf("  compute_layernorm: output %zu limbs, max |want| %.4g\n", o.coeff_modulus_size(), wmax);
            report("compute_layernorm(768) vs plain restatement, 32768 slots (error / max|want|)", err / wmax < 1e-5,
                   err / wmax, secs);
        }
    }
    {
        // surefire_rotate (util.cpp:344-356): a key made on the spot, rotation right by the shift
        const int S = 32768;
        std::uniform_real_distribution<double> U(-1, 1);
        std::vector<double> x(S);
        for (auto &v : x) v = U(rng);
        Ciphertext c = enc(x);
        const auto t = std::chrono::steady_clock::now();
        surefire_rotate(c, 100, keygen, evaluator);
        const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
        const auto got = dec(c);
        double err = 0;
        for (int i = 0; i < S; i++) err = std::max(err, std::fabs(got[i] - x[((i - 100) % S + S) % S]));
        report("surefire_rotate(100): on-the-spot Galois key, right rotation", err < 1e-6, err, secs);
    }
    for (int col = 0; col < 2; col++)
    {
        // attn_proj_row_seal / attn_proj_col_seal (MatrixMul.cpp:244-478), as written, vs the same
        // sequence restated in doubles: working_j = quickSum(rot(w_j * e_0, -1024), 1024); every
        // (rots, pos) adds working_j * e_{pos*2048} into head (abs_pos / 64) % 12; then + bias
        const int S = 32768;
        auto rot = [&](const std::vector<double> &x, int k) {
            std::vector<double> y(S);
            for (int i = 0; i < S; i++) y[i] = x[((i + k) % S + S) % S];
            return y;
        };
        auto qsum = [&](const std::vector<double> &x, int nn) {
            std::vector<double> o(S), r1 = rot(x, 1);
            for (int i = 0; i < S; i++) o[i] = x[i] + r1[i];
            for (int acc = 2; acc < nn; acc *= 2)
            {
                const auto ro = rot(o, acc);
                for (int i = 0; i < S; i++) o[i] += ro[i];
            }
            return o;
        };
        std::uniform_real_distribution<double> U(-1, 1);
        const int n_left = 1, n_w = 2, W_cols = 768;
        std::vector<std::vector<double>> w(n_w, std::vector<double>(S));
        std::vector<double> bias(S);
        for (auto &r : w)
            for (auto &v : r) v = U(rng);
        for (auto &v : bias) v = U(rng);
        std::vector<std::vector<double>> want(12, bias);
        for (int i = 0; i < n_left; i++)
            for (int j = 0; j < n_w; j++)
            {
                std::vector<double> m(S, 0.0);
                m[0] = w[j][0];
                const auto working = qsum(rot(m, -1024), 1024);
                for (int rots = 0; rots < 16; rots++)
                    for (int pos = 0; pos < 16; pos++)
                    {
                        const int abs_pos = (i * 16 + pos) * (col ? 768 : W_cols) + (j * 16 + ((rots + pos) % 16));
                        want[(abs_pos / 64) % 12][pos * 2048] += working[pos * 2048];
                    }
            }
        std::vector<Ciphertext> left{ enc(std::vector<double>(S, 0.5)) }, wc, out;
        for (auto &r : w) wc.push_back(enc(r));
        init_output(12, out, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
        const auto t = std::chrono::steady_clock::now();
        if (col)
            attn_proj_col_seal(left, wc, enc(bias), out, 128, 768, 768, W_cols, keygen, encoder, encryptor, decryptor,
                               evaluator, gal_keys, relin_keys);
        else
            attn_proj_row_seal(left, wc, enc(bias), out, 128, 768, 768, W_cols, keygen, encoder, encryptor, decryptor,
                               evaluator, gal_keys, relin_keys);
        const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
        double err = 0;
        for (int h = 0; h < 12; h++)
        {
            const auto got = dec(out[h]);
            for (int s = 0; s < S; s++) err = std::max(err, std::fabs(got[s] - want[h][s]));
        }
        report(col ? "attn_proj_col_seal (1 x 2 ciphers, 12 heads) vs plain restatement"
                   : "attn_proj_row_seal (1 x 2 ciphers, 12 heads) vs plain restatement",
               err < 1e-3, err, secs);
    }
    if (qkv)
    {
        // qk_matmul (MatrixMul.cpp:480-533) and sv_matmul (:535-584) on one ciphertext each, vs the
        // same sequences restated in doubles; 16384 + 8192 surefire_rotate placements
        const int S = 32768;
        auto rot = [&](const std::vector<double> &x, int k) {
            std::vector<double> y(S);
            for (int i = 0; i < S; i++) y[i] = x[((i + k) % S + S) % S];
            return y;
        };
        auto qsum = [&](const std::vector<double> &x, int nn) {
            std::vector<double> o(S), r1 = rot(x, 1);
            for (int i = 0; i < S; i++) o[i] = x[i] + r1[i];
            for (int acc = 2; acc < nn; acc *= 2)
            {
                const auto ro = rot(o, acc);
                for (int i = 0; i < S; i++) o[i] += ro[i];
            }
            return o;
        };
        std::uniform_real_distribution<double> U(-1, 1);
        std::vector<double> q(S), k(S), sm(S), v(S);
        for (auto *p : { &q, &k, &sm, &v })
            for (auto &x : *p) x = U(rng);
        // inputs at INIT()'s scale 2^46 on the last 6 limbs (46-bit primes): the placements need two
        // levels, and each rotation's key switch costs ~L^2, so this runs ~30x faster than at the top
        const double saved_scale = encode_scale(), s46 = std::pow(2.0, LOGP);
        set_encode_scale(s46);
        auto enc = [&](const std::vector<double> &x) {
            Plaintext p;
            Ciphertext c;
            encoder.encode(x, s46, p);
            encryptor.encrypt(p, c);
            while (c.coeff_modulus_size() > 6) evaluator.mod_switch_to_next_inplace(c);
            return c;
        };
        {
            auto k2 = rot(k, 16384), prod = q;
            for (int s = 0; s < S; s++) prod[s] *= k[s] + k2[s];
            const auto folded = qsum(rot(prod, S - 64), 64);
            std::vector<double> want(S, 0.0);
            for (int rots = 0; rots < 128; rots++)
                for (int pos = 0; pos < 128; pos++) want[pos * 256 + (rots + pos) % 128] += folded[pos * 128];
            std::vector<Ciphertext> Q{ enc(q) }, K{ enc(k) }, out;
            init_output(1, out, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
            std::printf("-- qk_matmul (16384 placements, surefire_rotate through +-2^i keys)\n");
            const auto t = std::chrono::steady_clock::now();
            qk_matmul(Q, K, out, 128, 64, 128, 64, keygen, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
            const auto got = dec(out[0]);
            const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
            double err = 0;
            for (int s = 0; s < S; s++) err = std::max(err, std::fabs(got[s] - want[s]));
            report("qk_matmul (1 ciphertext, 128 x 128 placements) vs plain restatement", err < 1e-3, err, secs);
        }
        {
            std::vector<std::vector<double>> want(128, std::vector<double>(S, 0.0));
            for (int rots = 0; rots < 64; rots++)
            {
                auto c = rot(v, 16384 + rots * 256);
                for (int s = 0; s < S; s++) c[s] *= sm[s];
                const auto folded = qsum(rot(c, S - 128), 128);
                for (int pos = 0; pos < 128; pos++)
                    want[pos][(pos % 16) * 2048 + (rots + pos) % 64] += folded[pos * 256];
            }
            std::vector<Ciphertext> Sc{ enc(sm) }, V{ enc(v) }, out;
            init_output(128, out, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
            std::printf("-- sv_matmul (8192 placements, surefire_rotate through +-2^i keys)\n");
            const auto t = std::chrono::steady_clock::now();
            sv_matmul(Sc, V, out, 128, 128, 128, 64, keygen, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
            double err = 0;
            for (int p = 0; p < 128; p++)
            {
                const auto got = dec(out[p]);
                for (int s = 0; s < S; s++) err = std::max(err, std::fabs(got[s] - want[p][s]));
            }
            const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
            report("sv_matmul (1 ciphertext, 64 x 128 placements into 128 outputs) vs plain restatement", err < 1e-3, err,
                   secs);
        }
        set_encode_scale(saved_scale);
    }
    if (qkv)
    {
        // batch_matmul (MatrixMul.cpp:630-649), qk_matmul_col (:651-725), cipher_plain_128_128
        // (:586-628) vs plain restatements
        const int S = 32768;
        std::uniform_real_distribution<double> U(-1, 1);
        std::unordered_map<std::string, std::vector<double>> weights{ { "test", std::vector<double>(S) } };
        for (auto &x : weights["test"]) x = U(rng);
        const auto &w = weights["test"];
        std::vector<std::vector<double>> L(128, std::vector<double>(S)), R(64, std::vector<double>(S));
        for (auto &r : L)
            for (auto &x : r) x = U(rng);
        for (auto &r : R)
            for (auto &x : r) x = U(rng);
        std::vector<Ciphertext> Lc, Rc, out;
        for (auto &r : L) Lc.push_back(enc(r));
        for (auto &r : R) Rc.push_back(enc(r));
        Ciphertext bias = enc(std::vector<double>(S, 0.0));
        {
            std::vector<double> want(S, 0.0);
            for (int j = 0; j < 128; j++)
                for (int s = 0; s < S; s++) want[s] += L[j][s] * w[s];
            init_output(64, out, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
            std::printf("-- batch_matmul\n");
            const auto t = std::chrono::steady_clock::now();
            batch_matmul(Lc, weights, bias, out, 128, 128, 128, 128, keygen, encoder, encryptor, decryptor, evaluator,
                         gal_keys, relin_keys);
            double err = 0;
            for (int i : { 0, 31, 63 })
            {
                const auto got = dec(out[i]);
                for (int s = 0; s < S; s++) err = std::max(err, std::fabs(got[s] - want[s]));
            }
            const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
            report("batch_matmul (128 x weights[\"test\"] into 64 outputs) vs plain", err < 1e-3, err, secs);
        }
        {
            out.clear();
            init_output(128, out, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
            std::printf("-- qk_matmul_col\n");
            std::vector<Ciphertext> Lh(Lc.begin(), Lc.begin() + 64);
            const auto t = std::chrono::steady_clock::now();
            qk_matmul_col(Lh, Rc, weights, bias, out, 128, 64, 128, 64, keygen, encoder, encryptor, decryptor,
                          evaluator, gal_keys, relin_keys);
            double err = 0;
            for (int i : { 0, 1, 77, 127 })
            {
                const auto got = dec(out[i]);
                for (int s = 0; s < S; s++)
                {
                    double want = 0;
                    for (int j = 0; j < 64; j++) want += L[j][s] * R[j][(s + i) % S];
                    err = std::max(err, std::fabs(got[s] - want));
                }
            }
            const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
            report("qk_matmul_col (64 pairs, 128 rotation rounds) vs plain", err < 1e-3, err, secs);
        }
        {
            std::printf("-- cipher_plain_128_128\n");
            const auto before = dec(out[0]);
            const auto t = std::chrono::steady_clock::now();
            cipher_plain_128_128(Lc[0], weights, bias, out, 128, 128, 128, 128, keygen, encoder, encryptor, decryptor,
                                 evaluator, gal_keys, relin_keys);
            const auto after = dec(out[0]);
            const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
            double err = 0;
            for (int s = 0; s < S; s++) err = std::max(err, std::fabs(after[s] - before[s]));
            report("cipher_plain_128_128 runs its 128 rounds and leaves outputs untouched", err == 0, err, secs);
        }
    }
    {
        // RowMatMul (run_approx_test.cpp:231-297): ones(8 x 2048) x ones(8 x 2048)^T = 2048 everywhere
        std::vector<std::vector<double>> A1(8, std::vector<double>(2048, 1.0)), A1_pre(1, std::vector<double>(32768, 0.0));
        pack_plain_row(A1, 8, 2048, A1_pre);
        std::vector<Ciphertext> a{ enc(A1_pre[0]) }, w{ enc(A1_pre[0]) }, output;
        init_output(1, output, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
        Ciphertext bias = enc(std::vector<double>(32768, 0.0000001));
        const auto s = std::chrono::steady_clock::now();
        row_matrix_multiplication_seal(a, w, bias, output, 8, 2048, 2048, 8, encoder, encryptor, decryptor, evaluator,
                                       gal_keys, relin_keys);
        const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - s).count();
        const auto res = dec(output[0]);
        double err = 0;
        bool ok = true;
        for (int i = 0; i < 8; i++)
            for (int j = 0; j < 8; j++)
            {
                err = std::max(err, std::fabs(res[i * 16 + j] - 2048.0));
                ok &= approx(res[i * 16 + j], 2048.0);
            }
        report("RowMatMul 8x2048 . (8x2048)^T (run_approx_test.cpp)", ok, err, secs);
    }
    {
        // C5-style feed-forward slice: random A (8 x 2048) times random W (8 x 2048)^T by the
        // row-packed encrypted matmul, + bias, then the GELU polynomial p over every slot; checked
        // against the same pipeline in doubles (the matmul result lands at slot i*16 + j,
        // MatrixMul.cpp:171-180; every other slot holds the bias only)
        std::uniform_real_distribution<double> U(-0.05, 0.05), B(-0.5, 0.5);
        std::vector<std::vector<double>> A(8, std::vector<double>(2048)), W(8, std::vector<double>(2048));
        for (auto &r : A)
            for (auto &x : r) x = U(rng);
        for (auto &r : W)
            for (auto &x : r) x = U(rng);
        std::vector<double> bias(32768);
        for (auto &x : bias) x = B(rng);
        std::vector<std::vector<double>> Ap(1, std::vector<double>(32768, 0.0)), Wp(1, std::vector<double>(32768, 0.0));
        pack_plain_row(A, 8, 2048, Ap);
        pack_plain_row(W, 8, 2048, Wp);
        std::vector<double> want(bias);
        for (int i = 0; i < 8; i++)
            for (int j = 0; j < 8; j++)
            {
                double acc = 0;
                for (int k = 0; k < 2048; k++) acc += A[i][k] * W[j][k];
                want[i * 16 + j] += acc;
            }
        for (auto &x : want) x = plain_gelu_p(x);
        std::printf("-- ffn slice\n");
        std::vector<Ciphertext> a{ enc(Ap[0]) }, w{ enc(Wp[0]) }, output;
        init_output(1, output, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
        Ciphertext bc = enc(bias), g;
        const auto t = std::chrono::steady_clock::now();
        row_matrix_multiplication_seal(a, w, bc, output, 8, 2048, 2048, 8, encoder, encryptor, decryptor, evaluator,
                                       gal_keys, relin_keys);
        compute_gelu_p(output[0], g, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
        const auto got = dec(g);
        const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
        double err = 0;
        for (int i = 0; i < 32768; i++) err = std::max(err, std::fabs(got[i] - want[i]));
        std::printf("  ffn slice: output %zu limbs\n", g.coeff_modulus_size());
        report("FFN slice: row matmul 8x2048 . (8x2048)^T + bias -> GELU p vs plain, 32768 slots", err < 1e-3, err, secs);
    }
    std::printf("%s\n", g_fail ? "FAILED" : "ok");
    return g_fail ? 1 : 0;
}
