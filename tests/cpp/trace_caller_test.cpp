// Caller-sequence trace for the oracle replay (tests/test_trace_parity.py): runs one multiplexed
// convolution at 3 limbs (cnn/cnn_seal.cpp:284-530, with its top-level encryption of zero, so the
// unequal-level branch of add_inplace_reduced_error runs -- SEAL/evaluator.cpp:312-362), one batch
// norm (cnn_seal.cpp:531-576) and one ReLU polynomial (comp/SEALcomp.cpp:3-60 with one component:
// comp/SEALfunc.cpp:59-260, then x (1 + sgn x) / 2) through the seal:: surface on the GPU with
// MHE_EVAL_TRACE=<dir>, so every evaluator operation of the sequence is written out (seal/trace.h),
// with seeded keys (Blake2xbPRNGFactory {1..8}) and seeded data.  The evaluation keys the sequence
// used are written next to the trace: key_relin.bin, key_gal_<elt>.bin (u64 header: digits, limbs,
// n; then [digits][2][limbs][n] in SEAL's layout, the special prime last).
//   trace_caller_test <log N: 12 | 16> <dir> <comp_dir>
//   trace_caller_test <log N> <dir> <comp_dir> boot <logn>
//   trace_caller_test <log N> <dir> <comp_dir> layers
// The boot mode traces one sparse bootstrap_real_3 instead (Bootstrapper.cpp:3166-3236 with
// ModularReducer.cpp:61-80 and Polynomial.cpp:256-560): the ResNet chain {51} + 16 x {46} + 14 x
// {51} + {51}, loge 10, K 25, cosine degree 59, 2 double-angle steps, inverse_deg 1, logn slots;
// modraise, subsum, CoeffToSlot BSGS, EvalMod and SlotToCoeff all land in the trace.
// The layers mode traces the remaining ResNet layers in network order (cnn/infer_seal.cpp:
// 520-560): a stride-2 downsampling (cnn_seal.cpp:610-679), the residual add with a second tensor of
// the downsampled shape (:593-609), the average pooling (:680-746) and the fully connected layer
// (:747-787).
#include "mhe_boot.h"
#include "mhe_cnn.h"
#include "mhe_comp.h"

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <random>
#include <string>

using namespace seal;

static void write_key(const std::string &path, const PolyStore &key, std::size_t limbs, std::size_t n)
{
    const std::uint64_t hdr[3] = { limbs - 1, limbs, n };
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char *>(hdr), sizeof hdr);
    f.write(reinterpret_cast<const char *>(key.host()), (std::streamsize)(key.words() * 8));
}

static void write_meta(const std::string &dir, const SEALContext &ctx, int logN)
{
    std::ofstream meta(dir + "/meta.json");
    meta << "{\"log_n\": " << logN << ", \"moduli\": [";
    const auto &q = ctx.key_context_data()->parms().coeff_modulus();
    for (std::size_t i = 0; i < q.size(); i++) meta << (i ? ", " : "") << q[i].value();
    meta << "], \"first_limbs\": " << ctx.first_context_data()->parms().coeff_modulus().size() << "}\n";
}

static void write_keys(const std::string &dir, const RelinKeys &rlk, const GaloisKeys &glk, std::size_t N)
{
    write_key(dir + "/key_relin.bin", rlk.key(0), rlk.limbs_of(0), N);
    std::size_t gal = 0;
    for (const auto &kv : glk.usage())
    {
        write_key(dir + "/key_gal_" + std::to_string(2 * kv.first + 1) + ".bin", glk.key(kv.first), kv.second, N);
        gal++;
    }
    std::printf("trace written to %s (%zu Galois keys used)\n", dir.c_str(), gal);
}

// one sparse bootstrap under the trace (see the header)
static int run_boot(int logN, const std::string &dir, long logn)
{
    const std::size_t N = (std::size_t)1 << logN;
    const long loge = 10, boundary_K = 25, boot_deg = 59, scale_factor = 2, inverse_deg = 1;
    const int logp = 46, logq = 51, remaining_level = 16, boot_level = 14, total_level = remaining_level + boot_level;
    std::vector<int> bits{ logq };
    for (int i = 0; i < remaining_level; i++) bits.push_back(logp);
    for (int i = 0; i < boot_level; i++) bits.push_back(logq);
    bits.push_back(51);
    EncryptionParameters parms(scheme_type::ckks);
    parms.set_poly_modulus_degree(N);
    parms.set_coeff_modulus(CoeffModulus::Create(N, bits));
    parms.set_secret_key_hamming_weight(logN >= 16 ? 192 : 64);
    parms.set_random_generator(
        std::make_shared<Blake2xbPRNGFactory>(std::array<std::uint64_t, 8>{ 1, 2, 3, 4, 5, 6, 7, 8 }));
    SEALContext ctx(parms, true, sec_level_type::none);
    KeyGenerator keygen(ctx);
    PublicKey pk;
    keygen.create_public_key(pk);
    RelinKeys rlk;
    keygen.create_relin_keys(rlk);
    GaloisKeys glk;
    CKKSEncoder encoder(ctx);
    Encryptor encryptor(ctx, pk);
    Decryptor decryptor(ctx, keygen.secret_key());
    Evaluator evaluator(ctx, encoder);
    const double scale = std::pow(2.0, logp);
    Bootstrapper bt(loge, logn, logN - 1, total_level, scale, boundary_K, boot_deg, scale_factor, inverse_deg, ctx, keygen,
                    encoder, encryptor, decryptor, evaluator, rlk, glk);
    bt.prepare_mod_polynomial();
    std::vector<int> steps{ 0 };
    for (int i = 0; i < logN - 1; i++) steps.push_back(1 << i);
    bt.addLeftRotKeys_Linear_to_vector_3(steps);
    keygen.create_deferred_galois_keys(steps, glk); // materialised (and grown) at the levels of use
    bt.slot_vec.push_back(logn);
    bt.generate_LT_coefficient_3();

    const long n = 1L << logn, Nh = (long)N / 2;
    std::mt19937_64 g(20261018);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    std::vector<double> z(n), msg(Nh);
    for (auto &x : z) x = U(g);
    for (long i = 0; i < Nh; i++) msg[i] = z[i % n];
    Plaintext pt;
    encoder.encode(msg, scale, pt);
    Ciphertext ct, out;
    encryptor.encrypt(pt, ct);
    evaluator.mod_switch_to_inplace(ct, ctx.last_parms_id());
    bt.bootstrap_real_3(out, ct);
    Plaintext dp;
    decryptor.decrypt(out, dp);
    std::vector<double> got;
    encoder.decode(dp, got);
    double err = 0;
    for (long i = 0; i < Nh; i++) err = std::max(err, std::fabs(got[i] - msg[i]));
    std::printf("bootstrap_real_3 (N 2^%d, logn %ld): %zu -> %zu limbs, max error %.3g\n", logN, logn, (std::size_t)1,
                out.coeff_modulus_size(), err);
    write_keys(dir, rlk, glk, N);
    write_meta(dir, ctx, logN);
    return err < 1e-2 ? 0 : 1;
}

// downsampling -> residual add -> average pooling -> FC under the trace (see the header)
static int run_layers(int logN, const std::string &dir)
{
    const std::size_t N = (std::size_t)1 << logN;
    std::vector<int> bits{ 51 };
    for (int i = 0; i < 8; i++) bits.push_back(46);
    bits.push_back(51);
    EncryptionParameters parms(scheme_type::ckks);
    parms.set_poly_modulus_degree(N);
    parms.set_coeff_modulus(CoeffModulus::Create(N, bits));
    parms.set_secret_key_hamming_weight(logN >= 16 ? 192 : 64);
    parms.set_random_generator(
        std::make_shared<Blake2xbPRNGFactory>(std::array<std::uint64_t, 8>{ 1, 2, 3, 4, 5, 6, 7, 8 }));
    SEALContext ctx(parms, true, sec_level_type::none);
    KeyGenerator keygen(ctx);
    PublicKey pk;
    keygen.create_public_key(pk);
    RelinKeys rlk;
    keygen.create_relin_keys(rlk);
    GaloisKeys glk;
    keygen.create_deferred_galois_keys(glk);
    CKKSEncoder encoder(ctx);
    Encryptor encryptor(ctx, pk);
    Decryptor decryptor(ctx, keygen.secret_key());
    Evaluator evaluator(ctx, encoder);
    const int logn = logN - 1;
    const long n = 1L << logn;
    // ResNet-20's first downsampling at N = 2^16 (k 1, h = w = 32, c = t = 16, p = 2), scaled down to
    // h = w = 8, c = t = 8 at N = 2^12; downsampled to k 2, h / 2, 2c, t / 2
    const int h = logN >= 16 ? 32 : 8, c = logN >= 16 ? 16 : 8, t = c, p = (int)(n / (h * h * t));
    std::mt19937_64 g(20261019);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    std::vector<double> img(n, 0.0);
    for (int r = 0; r < p; r++)
        for (int i = 0; i < c * h * h; i++) img[(std::size_t)r * (n / p) + i] = 0.5 * U(g);
    TensorCipher in(logn, 1, h, h, c, t, p, img, encryptor, encoder, 46);
    Ciphertext ct = in.cipher();
    while (ct.coeff_modulus_size() > 6) evaluator.mod_switch_to_next_inplace(ct);
    in.set_ciphertext(ct);
    TensorCipher ds;
    multiplexed_parallel_downsampling_seal(in, ds, evaluator, glk);
    // the residual branch: a fresh tensor of the downsampled shape at its level
    std::vector<double> img2(n, 0.0);
    const long blk = (long)ds.k() * ds.k() * ds.h() * ds.w() * ds.t();
    for (int r = 0; r < ds.p(); r++)
        for (long i = 0; i < blk; i++) img2[(std::size_t)r * (n / ds.p()) + i] = 0.25 * U(g);
    // (the data constructor takes k = 1 only, as the reference's: encrypt the k = 2 layout directly)
    Plaintext p2;
    encoder.encode(img2, std::pow(2.0, 46), p2);
    Ciphertext rc;
    encryptor.encrypt(p2, rc);
    evaluator.mod_switch_to_inplace(rc, ds.cipher().parms_id());
    TensorCipher res(logn, ds.k(), ds.h(), ds.w(), ds.c(), ds.t(), ds.p(), rc);
    TensorCipher sum;
    cnn_add_seal(ds, res, sum, evaluator);
    TensorCipher pooled, logits;
    std::ofstream devnull;
    averagepooling_seal_scale(sum, pooled, evaluator, glk, 1.0, encoder, decryptor, devnull);
    const int q = 10, r = pooled.c();
    std::vector<double> fc(q * r), bias(q);
    for (auto &v : fc) v = 0.5 * U(g);
    for (auto &v : bias) v = 0.1 * U(g);
    matrix_multiplication_seal(pooled, logits, fc, bias, q, r, evaluator, glk);
    Plaintext dp;
    decryptor.decrypt(logits.cipher(), dp);
    std::vector<double> got;
    encoder.decode(dp, got);
    // the layers' semantics are checked end to end by the ResNet runner against the plain network
    // (resnet_test / test_resnet.py); here only that the logits decrypt to bounded values
    double mag = 0;
    for (int i = 0; i < q; i++) mag = std::max(mag, std::fabs(got[i]));
    std::printf("layers (N 2^%d): downsample %dx%dx%d -> %dx%dx%d, add, avgpool, fc %dx%d: %zu limbs left, "
                "max |logit| %.3g\n",
                logN, h, h, c, ds.h(), ds.w(), ds.c(), q, r, logits.cipher().coeff_modulus_size(), mag);
    if (!(mag < 100.0)) return 1;
    write_keys(dir, rlk, glk, N);
    write_meta(dir, ctx, logN);
    return 0;
}

int main(int argc, char **argv)
{
    if (argc < 4)
    {
        std::fprintf(stderr, "usage: trace_caller_test <log N> <dir> <comp_dir> [boot <logn> | layers]\n");
        return 2;
    }
    const int logN = std::atoi(argv[1]);
    const std::string dir = argv[2];
    setenv("MHE_EVAL_TRACE", dir.c_str(), 1); // before the first evaluator operation
    setenv("MHE_COMP_DIR", argv[3], 1);
    if (argc > 5 && std::string(argv[4]) == "boot") return run_boot(logN, dir, std::atol(argv[5]));
    if (argc > 4 && std::string(argv[4]) == "layers") return run_layers(logN, dir);
    const std::size_t N = (std::size_t)1 << logN;
    // {51} + 8 x {46} + {51}: the ResNet chain's shape (cnn/infer_seal.cpp:288-316), shortened; 2^46 scale
    std::vector<int> bits{ 51 };
    for (int i = 0; i < 8; i++) bits.push_back(46);
    bits.push_back(51);
    EncryptionParameters parms(scheme_type::ckks);
    parms.set_poly_modulus_degree(N);
    parms.set_coeff_modulus(CoeffModulus::Create(N, bits));
    parms.set_secret_key_hamming_weight(logN >= 16 ? 192 : 64);
    parms.set_random_generator(
        std::make_shared<Blake2xbPRNGFactory>(std::array<std::uint64_t, 8>{ 1, 2, 3, 4, 5, 6, 7, 8 }));
    SEALContext ctx(parms, true, sec_level_type::none);
    KeyGenerator keygen(ctx);
    PublicKey pk;
    keygen.create_public_key(pk);
    RelinKeys rlk;
    keygen.create_relin_keys(rlk);
    GaloisKeys glk;
    keygen.create_deferred_galois_keys(glk); // materialised at the level of first use
    CKKSEncoder encoder(ctx);
    Encryptor encryptor(ctx, pk);
    Decryptor decryptor(ctx, keygen.secret_key());
    Evaluator evaluator(ctx, encoder);
    const double scale = std::pow(2.0, 46);
    const int logn = logN - 1;
    const long n = 1L << logn;

    std::mt19937_64 g(20261017);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    // 1. conv: k = 1, h = w = 8 (N = 2^12) or 16 (N = 2^16), ci = co = 4, t = 4, p = n / (h w t)
    const int h = logN >= 16 ? 16 : 8, ci = 4, co = 4, t = 4, p = (int)(n / (h * h * t));
    std::vector<double> img(n, 0.0), wt(9 * ci * co), var(co), gamma(co), bias(co), mean(co);
    for (int r = 0; r < p; r++)
        for (int i = 0; i < ci * h * h; i++) img[(std::size_t)r * (n / p) + i] = 0.5 * U(g);
    for (auto &v : wt) v = 0.3 * U(g);
    for (int b = 0; b < co; b++)
    {
        var[b] = 1.25 + 0.75 * U(g);
        gamma[b] = 1.0 + 0.5 * U(g);
        bias[b] = 0.1 * U(g);
        mean[b] = 0.1 * U(g);
    }
    TensorCipher in(logn, 1, h, h, ci, t, p, img, encryptor, encoder, 46);
    Ciphertext c = in.cipher();
    evaluator.mod_switch_to_inplace(c, ctx.get_context_data(ctx.first_parms_id())->next_context_data()->parms_id());
    while (c.coeff_modulus_size() > 3) evaluator.mod_switch_to_next_inplace(c);
    in.set_ciphertext(c);
    std::vector<Ciphertext> pool(16);
    TensorCipher out;
    multiplexed_parallel_convolution_seal(in, out, co, 1, 3, 3, wt, var, gamma, 1e-5, encoder, encryptor, evaluator, glk,
                                          pool);
    // 2. batch norm on the conv output
    TensorCipher bn;
    multiplexed_parallel_batch_norm_seal(out, bn, bias, mean, var, gamma, 1e-5, encoder, encryptor, evaluator, 40.0);
    // 3. one ReLU polynomial (the first component of the alpha = 13 composite) on a fresh input
    std::vector<double> x(n);
    for (auto &v : x) v = U(g);
    Plaintext px;
    encoder.encode(x, scale, px);
    Ciphertext cx, cr;
    encryptor.encrypt(px, cx);
    std::vector<Tree> tree(1);
    upgrade_oddbaby(15, tree[0]);
    SecretKey sk = keygen.secret_key();
    minimax_ReLU_seal(1, { 15 }, 13, tree, 1.7, 46, encryptor, evaluator, decryptor, encoder, pk, sk, rlk, cx, cr);

    // keys the sequence used, for the replay
    write_keys(dir, rlk, glk, N);
    write_meta(dir, ctx, logN);
    return 0;
}
