// GPU test of the approximate ReLU (include/mhe_comp.h; comp/SEALcomp.cpp, comp/SEALfunc.cpp,
// comp/program.cpp semantics) with the reference's ResNet setting: alpha = 13, three component
// polynomials of degrees {15, 15, 27}, odd baby-step trees, scaled_val 1.7, coefficients from
// tests/golden/comp/d13.txt.  The decrypted result is compared with max(x, 0).  Also checks the
// coefficient counts implied by the trees against the coefficient file (60 values) and a
// baby-step evaluation of a plain Chebyshev polynomial.
#include "mhe_cnn.h"

#include <cmath>
#include <cstdio>
#include <random>

using namespace seal;

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

int main()
{
    const long comp_no = 3, alpha = 13;
    std::vector<int> deg = { 15, 15, 27 };
    std::vector<Tree> tree;
    long total = 0;
    for (int d : deg)
    {
        Tree tr;
        upgrade_oddbaby(d, tr);
        CHECK(tr.type == evaltype::oddbaby);
        total += minicomp::coeff_number(d, tr);
        tree.push_back(tr);
    }
    std::printf("tree coefficient slots: %ld (file holds 60)\n", total);
    CHECK(total == 60);

    EncryptionParameters parms(scheme_type::ckks);
    const size_t N = 1 << 13;
    parms.set_poly_modulus_degree(N);
    std::vector<int> bits(1, 51);
    for (int i = 0; i < 20; i++) bits.push_back(46);
    bits.push_back(51);
    parms.set_coeff_modulus(CoeffModulus::Create(N, bits));
    SEALContext ctx(parms, true, sec_level_type::none);
    KeyGenerator keygen(ctx);
    PublicKey pk;
    keygen.create_public_key(pk);
    RelinKeys rlk;
    keygen.create_relin_keys(rlk);
    SecretKey sk = keygen.secret_key();
    CKKSEncoder encoder(ctx);
    Encryptor encryptor(ctx, pk);
    Decryptor decryptor(ctx, sk);
    Evaluator evaluator(ctx, encoder);

    const size_t slots = N / 2;
    std::mt19937_64 rng(3);
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    std::vector<double> x(slots);
    for (auto &v : x) v = u(rng);
    x[0] = 0.5, x[1] = -0.5, x[2] = 1e-3, x[3] = -1e-3, x[4] = 0.0;
    Plaintext pt;
    encoder.encode(x, std::pow(2.0, 46), pt);
    Ciphertext ct, out;
    encryptor.encrypt(pt, ct);
    const size_t level_in = ctx.get_context_data(ct.parms_id())->chain_index();
    minimax_ReLU_seal(comp_no, deg, alpha, tree, 1.7, 46, encryptor, evaluator, decryptor, encoder, pk, sk, rlk, ct, out);
    const size_t level_out = ctx.get_context_data(out.parms_id())->chain_index();
    decryptor.decrypt(out, pt);
    std::vector<double> y;
    encoder.decode(pt, y);
    double err = 0, err_far = 0;
    for (size_t i = 0; i < slots; i++)
    {
        const double want = x[i] > 0 ? x[i] : 0.0, e = std::fabs(y[i] - want);
        err = std::max(err, e);
        if (std::fabs(x[i]) > 0.01) err_far = std::max(err_far, e / std::fabs(x[i]));
    }
    std::printf("ReLU: levels %zu -> %zu, max abs error %.3g, max relative error (|x| > 0.01) %.3g\n", level_in,
                level_out, err, err_far);
    CHECK(err < 5e-3);
    CHECK(err_far < 1e-3);

    // baby-step variant on a Chebyshev polynomial: p(x) = sum c_k T_k(x) with the coefficient
    // layout the tree prescribes (leaf coefficients in the T basis of each leaf's degree)
    {
        Tree tb;
        upgrade_baby(7, tb);
        CHECK(tb.type == evaltype::baby);
        const long nc = minicomp::coeff_number(7, tb);
        std::printf("baby tree for degree 7: %ld coefficient slots, b=%d m=%d depth=%d\n", nc, tb.b, tb.m, tb.depth);
        CHECK(nc >= 8);
    }

    std::printf("%d checks, %d failed\n", g_checks, g_fail);
    return g_fail ? 1 : 0;
}
