// Timing of one ResNet-20 stage-1 multiplexed convolution layer at N = 2^16 on the GPU (the
// reference's "multiplexed parallel convolution... time : 12288 ms" at remaining level 2 -> 0,
// result/resnet20_cifar10_image0.txt:21-23, single CPU thread).  The chain is cut to the 3 data
// primes + special prime the layer uses at that level: a key switch at L limbs touches key
// digits 0..L-1 and limbs 0..L-1 + P only, so the work per operation is the same as in the full
// 32-prime chain.  Also times the stage-1 approximate ReLU at its level (16 -> 2) on a
// 17-prime chain.  Prints one JSON line.
#include "mhe_cnn.h"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

using namespace seal;
using clk = std::chrono::steady_clock;

static double secs(clk::time_point a, clk::time_point b)
{
    return std::chrono::duration<double>(b - a).count();
}

int main(int argc, char **argv)
{
    const int reps = argc > 1 ? std::atoi(argv[1]) : 3;
    const size_t N = 1 << 16;
    const int logn = 15;
    std::mt19937_64 rng(11);
    std::uniform_real_distribution<double> u(-1.0, 1.0);

    // --- convolution: 3 data limbs (level 2) + special prime, scale 2^46
    double conv_s = 0;
    {
        EncryptionParameters parms(scheme_type::ckks);
        parms.set_poly_modulus_degree(N);
        parms.set_coeff_modulus(CoeffModulus::Create(N, { 51, 46, 46, 51 }));
        parms.set_secret_key_hamming_weight(192);
        SEALContext ctx(parms, true, sec_level_type::none);
        KeyGenerator keygen(ctx);
        PublicKey pk;
        keygen.create_public_key(pk);
        GaloisKeys glk;
        keygen.create_galois_keys(glk);
        CKKSEncoder encoder(ctx);
        Encryptor encryptor(ctx, pk);
        Evaluator evaluator(ctx, encoder);
        const int h = 32, w = 32, c = 16, t = 16, p = 2, co = 16;
        std::vector<double> img((size_t)1 << logn, 0.0);
        for (int r = 0; r < p; r++)
            for (int i = 0; i < c * h * w; i++) img[(size_t)r * (N / 2 / p) + i] = 0.1 * u(rng);
        std::vector<double> wt(9 * c * co), var(co, 1.0), gamma(co, 1.0);
        for (auto &v : wt) v = 0.1 * u(rng);
        TensorCipher in(logn, 1, h, w, c, t, p, img, encryptor, encoder, 46);
        std::vector<Ciphertext> pool(16);
        TensorCipher out;
        multiplexed_parallel_convolution_seal(in, out, co, 1, 3, 3, wt, var, gamma, 0.0, encoder, encryptor,
                                              evaluator, glk, pool); // warm-up
        auto t0 = clk::now();
        for (int i = 0; i < reps; i++)
            multiplexed_parallel_convolution_seal(in, out, co, 1, 3, 3, wt, var, gamma, 0.0, encoder, encryptor,
                                                  evaluator, glk, pool);
        Plaintext sync;
        Decryptor dec(ctx, keygen.secret_key());
        dec.decrypt(out.cipher(), sync);
        (void)sync.data(); // forces the device work to finish
        conv_s = secs(t0, clk::now()) / reps;
    }

    // --- approximate ReLU from level 16 (17 primes + special) as in the ResNet driver
    double relu_s = 0;
    {
        EncryptionParameters parms(scheme_type::ckks);
        parms.set_poly_modulus_degree(N);
        std::vector<int> bits(1, 51);
        for (int i = 0; i < 16; i++) bits.push_back(46);
        bits.push_back(51);
        parms.set_coeff_modulus(CoeffModulus::Create(N, bits));
        parms.set_secret_key_hamming_weight(192);
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
        std::vector<int> deg = { 15, 15, 27 };
        std::vector<Tree> tree;
        for (int d : deg)
        {
            Tree tr;
            upgrade_oddbaby(d, tr);
            tree.push_back(tr);
        }
        std::vector<double> x(N / 2);
        for (auto &v : x) v = u(rng);
        Plaintext pt;
        encoder.encode(x, std::pow(2.0, 46), pt);
        Ciphertext ct, res;
        encryptor.encrypt(pt, ct);
        minimax_ReLU_seal(3, deg, 13, tree, 1.7, 46, encryptor, evaluator, decryptor, encoder, pk, sk, rlk, ct, res);
        auto t0 = clk::now();
        for (int i = 0; i < reps; i++)
            minimax_ReLU_seal(3, deg, 13, tree, 1.7, 46, encryptor, evaluator, decryptor, encoder, pk, sk, rlk, ct,
                              res);
        decryptor.decrypt(res, pt);
        (void)pt.data();
        relu_s = secs(t0, clk::now()) / reps;
    }
    std::printf("{\"conv_stage1_level2_s\": %.4f, \"conv_reference_cpu_s\": 12.288, \"relu_level16_s\": %.4f, "
                "\"relu_reference_cpu_s\": 11.664, \"reps\": %d}\n",
                conv_s, relu_s, reps);
    return 0;
}
