// GPU tests of the multiplexed-packing CNN layers (include/mhe_cnn.h): each layer runs on an
// encrypted tensor and is compared after decryption with the same layer computed in plain
// doubles (cnn_ckks/cpu-ckks/single-key/cnn/cnn_seal.cpp semantics).  N = 2^12 (2048 slots),
// small tensors.  Driven by tests/test_seal_api.py (GPU marker).
#include "mhe_cnn.h"

#include <algorithm>
#include <cmath>
#include <cstring>
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

static std::mt19937_64 rng(7);
static double urand(double a, double b)
{
    return std::uniform_real_distribution<double>(a, b)(rng);
}

struct Env
{
    EncryptionParameters parms{ scheme_type::ckks };
    std::unique_ptr<SEALContext> ctx;
    std::unique_ptr<KeyGenerator> keygen;
    PublicKey pk;
    RelinKeys rlk;
    GaloisKeys glk;
    std::unique_ptr<CKKSEncoder> encoder;
    std::unique_ptr<Encryptor> encryptor;
    std::unique_ptr<Decryptor> decryptor;
    std::unique_ptr<Evaluator> evaluator;
    Env()
    {
        parms.set_poly_modulus_degree(4096);
        parms.set_coeff_modulus(CoeffModulus::Create(4096, { 50, 40, 40, 40, 40, 40, 40, 40, 50 }));
        // seeded (SEAL's debugging factory): the convolution's encryption of zero is the same in both
        // runs of the batched / one-by-one comparison
        parms.set_random_generator(
            std::make_shared<Blake2xbPRNGFactory>(std::array<std::uint64_t, 8>{ 8, 7, 6, 5, 4, 3, 2, 1 }));
        ctx = std::make_unique<SEALContext>(parms, true, sec_level_type::none);
        keygen = std::make_unique<KeyGenerator>(*ctx);
        keygen->create_public_key(pk);
        keygen->create_relin_keys(rlk);
        keygen->create_galois_keys(glk);
        encoder = std::make_unique<CKKSEncoder>(*ctx);
        encryptor = std::make_unique<Encryptor>(*ctx, pk);
        decryptor = std::make_unique<Decryptor>(*ctx, keygen->secret_key());
        evaluator = std::make_unique<Evaluator>(*ctx, *encoder);
    }
    std::vector<double> dec(const TensorCipher &t)
    {
        Plaintext p;
        decryptor->decrypt(t.cipher(), p);
        std::vector<double> out;
        encoder->decode(p, out);
        return out;
    }
};

static const int LOGN = 11, N = 1 << LOGN;

// k = 1 layout: local slot c*h*w + y*w + x, replicated every N/p slots
static std::vector<double> pack1(const std::vector<double> &t, int h, int w, int c, int p)
{
    std::vector<double> v(N, 0.0);
    for (int r = 0; r < p; r++)
        for (int i = 0; i < c * h * w; i++) v[(size_t)r * (N / p) + i] = t[i];
    return v;
}

// general multiplexed slot of (channel, y, x) for gap k, first replica
static int mux_slot(int k, int h, int w, int ch, int y, int x)
{
    const int u = ch / (k * k), rem = ch % (k * k);
    return k * k * h * w * u + k * w * (k * y + rem / k) + (k * x + rem % k);
}

static double conv_plain(const std::vector<double> &in, const std::vector<double> &wt, int h, int w, int ci, int co,
                         int b, int y, int x)
{
    double s = 0;
    for (int a = 0; a < ci; a++)
        for (int i1 = 0; i1 < 3; i1++)
            for (int i2 = 0; i2 < 3; i2++)
            {
                const int yy = y + i1 - 1, xx = x + i2 - 1;
                if (yy < 0 || yy >= h || xx < 0 || xx >= w) continue;
                s += wt[((size_t)(b * ci + a) * 3 + i1) * 3 + i2] * in[(size_t)a * h * w + yy * w + xx];
            }
    return s;
}

static void test_conv_bn_add(Env &e)
{
    const int h = 8, w = 8, ci = 4, co = 4, t = 4, p = N / (h * w * t);
    std::vector<double> img(ci * h * w), wt(9 * ci * co), var(co), gamma(co);
    for (auto &v : img) v = urand(-1, 1);
    for (auto &v : wt) v = urand(-0.3, 0.3);
    for (int b = 0; b < co; b++)
    {
        var[b] = urand(0.5, 2.0);
        gamma[b] = urand(0.5, 1.5);
    }
    TensorCipher in(LOGN, 1, h, w, ci, t, p, pack1(img, h, w, ci, p), *e.encryptor, *e.encoder, 40);
    std::vector<Ciphertext> pool(16);
    TensorCipher out;
    multiplexed_parallel_convolution_seal(in, out, co, 1, 3, 3, wt, var, gamma, 1e-5, *e.encoder, *e.encryptor,
                                          *e.evaluator, e.glk, pool);
    CHECK(out.k() == 1 && out.h() == h && out.w() == w && out.c() == co && out.t() == 4 && out.p() == p);
    auto got = e.dec(out);
    double err = 0;
    for (int r = 0; r < out.p(); r++)
        for (int b = 0; b < co; b++)
            for (int y = 0; y < h; y++)
                for (int x = 0; x < w; x++)
                {
                    const double want = conv_plain(img, wt, h, w, ci, co, b, y, x) * gamma[b] / std::sqrt(var[b] + 1e-5);
                    err = std::max(err, std::fabs(got[(size_t)r * (N / out.p()) + b * h * w + y * w + x] - want));
                }
    std::printf("  conv st=1 max error %.3g\n", err);
    CHECK(err < 1e-3);
    {
        // the blocks' batched launches (tap sums in one pass, shared-key folds, gathered rotations)
        // give the words of the block-by-block, term-by-term sequence
        TensorCipher out1;
        std::vector<Ciphertext> pool1(16);
        set_batched_launches(false);
        multiplexed_parallel_convolution_seal(in, out1, co, 1, 3, 3, wt, var, gamma, 1e-5, *e.encoder, *e.encryptor,
                                              *e.evaluator, e.glk, pool1);
        set_batched_launches(true);
        const Ciphertext &x = out.cipher(), &y = out1.cipher();
        const bool same = x.parms_id() == y.parms_id() && x.scale() == y.scale() &&
                          x.store().words() == y.store().words() &&
                          std::memcmp(x.store().host(), y.store().host(), x.store().words() * 8) == 0;
        std::printf("  conv batched vs one-by-one: %s\n", same ? "identical" : "DIFFERENT");
        CHECK(same);
    }

    // batch norm offset (cnn_seal.cpp:531-576) and residual add
    std::vector<double> bias(co), mean(co), bw(co);
    for (int b = 0; b < co; b++)
    {
        bias[b] = urand(-0.5, 0.5);
        mean[b] = urand(-0.5, 0.5);
        bw[b] = urand(0.5, 1.5);
    }
    const double B = 4.0;
    TensorCipher bn;
    multiplexed_parallel_batch_norm_seal(out, bn, bias, mean, var, bw, 1e-5, *e.encoder, *e.encryptor, *e.evaluator, B);
    auto gb = e.dec(bn);
    err = 0;
    for (int b = 0; b < co; b++)
        for (int i = 0; i < h * w; i++)
        {
            const double off = (mean[b] * bw[b] / std::sqrt(var[b] + 1e-5) - bias[b]) / B;
            err = std::max(err, std::fabs(gb[b * h * w + i] - (got[b * h * w + i] - off)));
        }
    std::printf("  batch norm max error %.3g\n", err);
    CHECK(err < 1e-3);
    TensorCipher sum;
    cnn_add_seal(bn, out, sum, *e.evaluator);
    auto gs = e.dec(sum);
    err = 0;
    for (int i = 0; i < co * h * w; i++) err = std::max(err, std::fabs(gs[i] - (gb[i] + got[i])));
    std::printf("  residual add max error %.3g\n", err);
    CHECK(err < 1e-3);
}

static void test_conv_stride2(Env &e)
{
    const int h = 8, w = 8, ci = 4, co = 8, t = 4, p = N / (h * w * t);
    std::vector<double> img(ci * h * w), wt(9 * ci * co), var(co, 1.0), gamma(co, 1.0);
    for (auto &v : img) v = urand(-1, 1);
    for (auto &v : wt) v = urand(-0.3, 0.3);
    TensorCipher in(LOGN, 1, h, w, ci, t, p, pack1(img, h, w, ci, p), *e.encryptor, *e.encoder, 40);
    std::vector<Ciphertext> pool(16);
    TensorCipher out;
    multiplexed_parallel_convolution_seal(in, out, co, 2, 3, 3, wt, var, gamma, 0.0, *e.encoder, *e.encryptor,
                                          *e.evaluator, e.glk, pool);
    CHECK(out.k() == 2 && out.h() == 4 && out.w() == 4 && out.c() == co);
    auto got = e.dec(out);
    double err = 0;
    for (int b = 0; b < co; b++)
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++)
            {
                const double want = conv_plain(img, wt, h, w, ci, co, b, 2 * y, 2 * x);
                err = std::max(err, std::fabs(got[mux_slot(2, 4, 4, b, y, x)] - want));
            }
    std::printf("  conv st=2 max error %.3g\n", err);
    CHECK(err < 1e-3);
}

static void test_downsample_pool_fc(Env &e)
{
    // downsampling (k=1, 4x4, 8 channels -> k=2, 2x2, 16 channels): the ResNet "option A"
    // shortcut, input channel c lands on output channel c + ci/2 (the -ko^2*ho*wo*(ti/8) term of
    // cnn_seal.cpp:663), the other output channels are zero
    const int h = 4, w = 4, ci = 8, t = 8, p = N / (h * w * t);
    std::vector<double> img(ci * h * w);
    for (auto &v : img) v = urand(-1, 1);
    TensorCipher in(LOGN, 1, h, w, ci, t, p, pack1(img, h, w, ci, p), *e.encryptor, *e.encoder, 40);
    TensorCipher ds;
    multiplexed_parallel_downsampling_seal(in, ds, *e.evaluator, e.glk);
    CHECK(ds.k() == 2 && ds.h() == 2 && ds.w() == 2 && ds.c() == 16 && ds.t() == 4);
    auto got = e.dec(ds);
    double err = 0;
    for (int c = 0; c < ci; c++)
        for (int y = 0; y < 2; y++)
            for (int x = 0; x < 2; x++)
                err = std::max(err, std::fabs(got[mux_slot(2, 2, 2, c + ci / 2, y, x)] -
                                              img[(size_t)c * h * w + 2 * y * w + 2 * x]));
    for (int c = 0; c < ci / 2; c++) // zero padding channels
        err = std::max(err, std::fabs(got[mux_slot(2, 2, 2, c, 1, 1)]));
    std::printf("  downsampling max error %.3g\n", err);
    CHECK(err < 1e-3);

    // average pooling over 4x4 (k=1, 4 channels) then a 3x4 fully connected layer
    const int hp = 4, wp = 4, cp = 4, tp = 4, pp = N / (hp * wp * tp);
    std::vector<double> im2(cp * hp * wp);
    for (auto &v : im2) v = urand(-1, 1);
    TensorCipher in2(LOGN, 1, hp, wp, cp, tp, pp, pack1(im2, hp, wp, cp, pp), *e.encryptor, *e.encoder, 40);
    TensorCipher pooled;
    std::ofstream devnull;
    const double B = 2.0;
    averagepooling_seal_scale(in2, pooled, *e.evaluator, e.glk, B, *e.encoder, *e.decryptor, devnull);
    auto gp = e.dec(pooled);
    std::vector<double> mean(cp, 0.0);
    err = 0;
    for (int c = 0; c < cp; c++)
    {
        for (int i = 0; i < hp * wp; i++) mean[c] += im2[(size_t)c * hp * wp + i];
        mean[c] *= B / (hp * wp);
        err = std::max(err, std::fabs(gp[c] - mean[c]));
    }
    std::printf("  average pooling max error %.3g\n", err);
    CHECK(err < 1e-3);

    const int q = 3, r = 4;
    std::vector<double> M(q * r), bias(q, 0.0);
    for (auto &v : M) v = urand(-1, 1);
    TensorCipher fc;
    matrix_multiplication_seal(pooled, fc, M, bias, q, r, *e.evaluator, e.glk);
    auto gf = e.dec(fc);
    err = 0;
    for (int i = 0; i < q; i++)
    {
        double s = 0;
        for (int j = 0; j < r; j++) s += M[(size_t)i * r + j] * mean[j];
        err = std::max(err, std::fabs(gf[i] - s));
    }
    std::printf("  fully connected max error %.3g\n", err);
    CHECK(err < 1e-3);
}

static void test_memory_save_rotate(Env &e)
{
    std::vector<double> v(N);
    for (int i = 0; i < N; i++) v[i] = std::sin(0.05 * i);
    Plaintext pt;
    e.encoder->encode(v, std::pow(2.0, 40), pt);
    Ciphertext ct, out;
    e.encryptor->encrypt(pt, ct);
    for (int steps : { 40, 58, 7, -5, 0 })
    {
        out = ct;
        memory_save_rotate(ct, out, steps, *e.evaluator, e.glk);
        Plaintext p2;
        e.decryptor->decrypt(out, p2);
        std::vector<double> got;
        e.encoder->decode(p2, got);
        double err = 0;
        for (int i = 0; i < N; i++) err = std::max(err, std::fabs(got[i] - v[((i + steps) % N + N) % N]));
        CHECK(err < 1e-4);
    }
}

int main()
{
    Env e;
    struct T
    {
        const char *name;
        void (*fn)(Env &);
    } tests[] = { { "memory_save_rotate", test_memory_save_rotate },
                  { "conv_bn_add", test_conv_bn_add },
                  { "conv_stride2", test_conv_stride2 },
                  { "downsample_pool_fc", test_downsample_pool_fc } };
    for (auto &t : tests)
    {
        const int before = g_fail;
        try
        {
            t.fn(e);
        }
        catch (const std::exception &ex)
        {
            g_fail++;
            std::fprintf(stderr, "  EXCEPTION in %s: %s\n", t.name, ex.what());
        }
        std::printf("[%s] %s\n", g_fail == before ? "PASS" : "FAIL", t.name);
        std::fflush(stdout);
    }
    std::printf("%d checks, %d failed\n", g_checks, g_fail);
    return g_fail ? 1 : 0;
}
