// GPU test of CKKS bootstrapping (include/mhe_boot.h) in the reference ResNet setting
// (cnn/infer_seal.cpp:287-388): N = 2^16, chain {51, 46 x 16, 51 x 14, 51}, secret-key Hamming
// weight 192, loge 10, boundary K 25, cosine degree 59, 2 double-angle steps, inverse_deg 1,
// sparse slots logn in argv (default 14).  A random real message in [-1, 1] with period 2^logn
// is encrypted, dropped to the last level (1 limb) and bootstrapped; the decryption is compared
// with the message.  Prints the output level, the precision and the time per bootstrap.
#include "mhe_boot.h"

#include "../../include/mhe.h"

#include <chrono>
#include <cmath>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <random>

using namespace seal;

int main(int argc, char **argv)
{
    const long logn = argc > 1 ? std::atol(argv[1]) : 14;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 2;
    const long logN = 16, loge = 10, boundary_K = 25, boot_deg = 59, scale_factor = 2, inverse_deg = 1;
    const int logp = 46, logq = 51, log_special_prime = 51, remaining_level = 16, boot_level = 14;
    const int total_level = remaining_level + boot_level;
    std::vector<int> bits{ logq };
    for (int i = 0; i < remaining_level; i++) bits.push_back(logp);
    for (int i = 0; i < boot_level; i++) bits.push_back(logq);
    bits.push_back(log_special_prime);

    EncryptionParameters parms(scheme_type::ckks);
    parms.set_poly_modulus_degree(1 << logN);
    parms.set_coeff_modulus(CoeffModulus::Create(1 << logN, bits));
    parms.set_secret_key_hamming_weight(192);
    parms.set_random_generator(std::make_shared<Blake2xbPRNGFactory>(std::array<std::uint64_t, 8>{ 1, 2, 3, 4, 5, 6, 7, 8 }));
    const double scale = std::pow(2.0, logp);
    SEALContext context(parms);
    KeyGenerator keygen(context);
    PublicKey public_key;
    keygen.create_public_key(public_key);
    auto secret_key = keygen.secret_key();
    RelinKeys relin_keys;
    keygen.create_relin_keys(relin_keys);
    GaloisKeys gal_keys;
    CKKSEncoder encoder(context);
    Encryptor encryptor(context, public_key);
    Evaluator evaluator(context, encoder);
    Decryptor decryptor(context, secret_key);

    Bootstrapper bt(loge, logn, logN - 1, total_level, scale, boundary_K, boot_deg, scale_factor, inverse_deg, context,
                    keygen, encoder, encryptor, decryptor, evaluator, relin_keys, gal_keys);
    auto t0 = std::chrono::steady_clock::now();
    bt.prepare_mod_polynomial();
    std::vector<int> steps{ 0 };
    for (int i = 0; i < logN - 1; i++) steps.push_back(1 << i);
    bt.addLeftRotKeys_Linear_to_vector_3(steps);
    keygen.create_galois_keys(steps, gal_keys);
    bt.slot_vec.push_back(logn);
    bt.generate_LT_coefficient_3();
    auto t1 = std::chrono::steady_clock::now();
    std::printf("setup (polynomials, %zu Galois steps, LT coefficients): %.2f s\n", steps.size(),
                std::chrono::duration<double>(t1 - t0).count());

    int fail = 0;
    {
        // modraise_inplace written against the surface's seal::util::iter, as the reference writes it
        // (BOOT/Bootstrapper.cpp:2894-2948: centred lift of the one-limb coefficients to every prime
        // of the first level), against the Bootstrapper's GPU version: every word equal
        std::vector<double> v(1 << (logN - 1));
        std::mt19937_64 gg(5);
        std::uniform_real_distribution<double> UU(-1, 1);
        for (auto &x : v) x = UU(gg);
        Plaintext p;
        encoder.encode(v, scale, p);
        Ciphertext a;
        encryptor.encrypt(p, a);
        evaluator.mod_switch_to_inplace(a, context.last_parms_id());
        Ciphertext b = a;
        bt.modraise_inplace(b);
        {
            using seal::util::iter;
            if (a.is_ntt_form()) evaluator.transform_from_ntt_inplace(a);
            Ciphertext src(a);
            a.resize(context, context.first_parms_id(), 2);
            const auto &modulus = iter(context.first_context_data()->parms().coeff_modulus());
            const std::size_t L = a.coeff_modulus_size(), N = a.poly_modulus_degree();
            const std::uint64_t q0 = modulus[0].value();
            for (std::size_t k = 0; k < a.size(); k++)
            {
                const auto s0 = iter(static_cast<const Ciphertext &>(src))[k][0];
                const auto dst = iter(a)[k];
                for (std::size_t j = 0; j < L; j++)
                {
                    const std::uint64_t q = modulus[j].value(), mq0 = j ? q - q0 % q : 0;
                    for (std::size_t i = 0; i < N; i++)
                    {
                        std::uint64_t x = s0[i] % q;
                        if (s0[i] > (q0 >> 1))
                        {
                            x += mq0;
                            x -= x >= q ? q : 0;
                        }
                        dst[j][i] = x;
                    }
                }
            }
            evaluator.transform_to_ntt_inplace(a);
        }
        std::size_t diff = 0;
        const std::uint64_t *x = a.data(), *y = b.data();
        for (std::size_t w = 0; w < a.dyn_array_size(); w++) diff += x[w] != y[w];
        std::printf("modraise via seal::util::iter vs Bootstrapper::modraise_inplace: %zu of %zu words differ (%zu limbs)\n",
                    diff, a.dyn_array_size(), a.coeff_modulus_size());
        if (diff || a.dyn_array_size() != b.dyn_array_size()) fail++;
    }

    const long n = 1L << logn, Nh = 1L << (logN - 1);
    std::mt19937_64 g(2026);
    std::uniform_real_distribution<double> U(-1, 1);
    std::vector<double> z(n), msg(Nh);
    for (auto &x : z) x = U(g);
    for (long i = 0; i < Nh; i++) msg[i] = z[i % n];
    Plaintext pt;
    encoder.encode(msg, scale, pt);
    Ciphertext ct;
    encryptor.encrypt(pt, ct);
    evaluator.mod_switch_to_inplace(ct, context.last_parms_id());
    std::printf("input: %zu limb(s), scale 2^%.2f\n", ct.coeff_modulus_size(), std::log2(ct.scale()));

    if (argc > 3)
    {
        // stage-by-stage checks on fresh encryptions
        auto dec = [&](const Ciphertext &c) {
            Plaintext p;
            decryptor.decrypt(c, p);
            std::vector<std::complex<double>> v;
            encoder.decode(p, v);
            return v;
        };
        auto bitrev = [](long x, int bits) {
            long r = 0;
            for (int i = 0; i < bits; i++) r |= ((x >> i) & 1) << (bits - 1 - i);
            return r;
        };
        const double q0 = (double)context.first_context_data()->parms().coeff_modulus()[0].value();
        // CoeffToSlot: slots of t (real coefficients, 2n of them) -> t[perm] / (K Nh/n)
        std::vector<double> t(2 * n);
        for (auto &x : t) x = U(g) * 10;
        std::vector<std::complex<double>> w(Nh);
        long p5 = 1;
        for (long k = 0; k < n; k++)
        {
            std::complex<double> acc = 0;
            for (long j = 0; j < n; j++)
                acc += std::complex<double>(t[j], t[j + n]) *
                       std::polar(1.0, 2 * M_PI * (double)((p5 * j) % (4 * n)) / (4.0 * n));
            for (long r = k; r < Nh; r += n) w[r] = acc;
            p5 = (p5 * 5) % (4 * n);
        }
        Plaintext pw;
        encoder.encode(w, q0, pw);
        Ciphertext cw, cts;
        encryptor.encrypt(pw, cw);
        std::printf("debug CtS input: %zu limbs\n", cw.coeff_modulus_size());
        bt.coefftoslot_3(cts, cw);
        auto v = dec(cts);
        double e1 = 0;
        const double f = 1.0 / (boundary_K * (double)(Nh / n));
        for (long x = 0; x < Nh; x++)
        {
            const long xx = x % (2 * n);
            const long j = bitrev(xx % n, (int)logn) + (xx >= n ? n : 0);
            e1 = std::max(e1, std::abs(v[x] - std::complex<double>(t[j] * f, 0)));
        }
        std::printf("debug CtS: out %zu limbs, scale 2^%.2f, max error %.3g (values ~%.3g)\n", cts.coeff_modulus_size(),
                    std::log2(cts.scale()), e1, 10 * f);
        // EvalMod: y = (I + eps) / K -> c1 sin(2 pi K y)
        std::vector<double> y(Nh);
        for (auto &x : y)
        {
            const int I = (int)std::floor(U(g) * 20);
            x = (I + U(g) * std::pow(2.0, -11)) / boundary_K;
        }
        Plaintext py;
        encoder.encode(y, cts.scale(), py);
        evaluator.mod_switch_to_inplace(py, cts.parms_id());
        Ciphertext cy, cm;
        encryptor.encrypt(py, cy);
        evaluator.mod_switch_to_inplace(cy, cts.parms_id());
        cy.scale() = cts.scale();
        bt.mod_reducer->modular_reduction(cm, cy);
        auto vm = dec(cm);
        double e2 = 0;
        const double c1 = std::pow(bt.mod_reducer->scale_inverse_coeff, 4);
        for (long x = 0; x < Nh; x++)
            e2 = std::max(e2, std::abs(vm[x].real() - c1 * std::sin(2 * M_PI * boundary_K * y[x])));
        std::printf("debug EvalMod: in %zu limbs -> out %zu limbs, scale 2^%.2f, max error %.3g (c1 %.6g)\n",
                    cy.coeff_modulus_size(), cm.coeff_modulus_size(), std::log2(cm.scale()), e2, c1);
    }
    for (int r = 0; r < reps; r++)
    {
        Ciphertext in = ct, out;
        const auto b0 = std::chrono::steady_clock::now();
        bt.bootstrap_real_3(out, in);
        mhe_stream_sync(context.engine(), context.stream());
        const auto b1 = std::chrono::steady_clock::now();
        Plaintext dp;
        decryptor.decrypt(out, dp);
        std::vector<double> dec;
        encoder.decode(dp, dec);
        double err = 0;
        for (long i = 0; i < Nh; i++) err = std::max(err, std::abs(dec[i] - msg[i]));
        std::printf("bootstrap %d: %.3f s, output %zu limbs, scale 2^%.2f, max error %.3g (2^%.1f), %zu cached pts\n",
                    r, std::chrono::duration<double>(b1 - b0).count(), out.coeff_modulus_size(),
                    std::log2(out.scale()), err, std::log2(err), bt.cached_plaintexts());
        if (!(err < 1e-3)) fail++;
        if (out.coeff_modulus_size() < 3) fail++;
    }
    {
        // batched launches (BSGS rotations, EvalMod products and rescales of one depth) give the
        // same words as every operation run alone
        Ciphertext in0 = ct, in1 = ct, o0, o1;
        set_batched_launches(false);
        bt.bootstrap_real_3(o0, in0);
        set_batched_launches(true);
        bt.bootstrap_real_3(o1, in1);
        const PolyStore &x = o0.store(), &y = o1.store();
        const bool same = o0.parms_id() == o1.parms_id() && o0.scale() == o1.scale() && x.words() == y.words() &&
                          std::memcmp(x.host(), y.host(), x.words() * 8) == 0;
        std::printf("batched vs one-by-one bootstrap: %s (%zu words)\n", same ? "identical" : "DIFFERENT", x.words());
        if (!same) fail++;
    }
    std::printf("galois key memory: %.2f GB\n", gal_keys.device_bytes() / 1e9);
    std::printf("%s\n", fail ? "FAILED" : "ok");
    return fail ? 1 : 0;
}
