// mhe_gpt2.h -- the GPT-2 approximation and packed-matmul layer of the reference
// (gpt2_ckks/gpt2-ckks/single-key/gpt2/: PolyApprox.cpp, IterApprox.cpp, Fold.cpp, MatrixMul.cpp,
// util.cpp, pack.cpp) over the MI355X seal:: surface.  Same names, argument order and operation
// sequence as the reference, so its callers and its doctest cases (gpt2_ckks/run/
// run_approx_test.cpp) read unchanged; every ciphertext operation runs on the GPU.
//
// Deviations, by design:
//  * sign_function / compute_gelu take and return Ciphertext instead of the GPT-2 TensorCipher
//    wrapper (gpt2/tensor.h; the wrapper only carries the ciphertext on this path) and drop the
//    Bootstrapper argument, which the reference accepts but never uses on this path
//    (PolyApprox.cpp:308-334, 443-504);
//  * the debugging printf()s of the reference are not reproduced;
//  * compute_gelu_q rescales its last product before the final add (PolyApprox.cpp:429-431 adds it
//    unrescaled, which loses half the polynomial; see gpt2.cpp).
#pragma once

#include <string>
#include <unordered_map>
#include <vector>

#include "mhe_boot.h"
#include "seal/seal.h"

namespace gpt2
{
using seal::CKKSEncoder;
using seal::Ciphertext;
using seal::Decryptor;
using seal::Encryptor;
using seal::Evaluator;
using seal::GaloisKeys;
using seal::RelinKeys;

constexpr int LOGP = 46, LOGQ = 49, BOOT_LEVEL = 14; // gpt2/util.h:22-25
double encode_scale();                               // ENCODE_SCALE, 2^LOGP by default
// The reference hard-codes ENCODE_SCALE = 2^46, but its *_reduced_error ops overwrite scales and so
// assume the scale tracks the primes being rescaled away; on its own chain ({49} + 21 x {46} +
// 14 x {49}) the top levels rescale by 49-bit primes and a 2^46 scale collapses to ~2^1 within one
// Chebyshev evaluation.  Callers working at scale 2^49 set the plaintexts' scale to match.
void set_encode_scale(double scale);

// util.cpp:258-261: next power of two
int round_to_2(double x);

// PolyApprox.cpp:14-101: [T0, T1, T2, T3, T4, T8, ...] -- T0 an encryption of ones, T2 = 2x^2 - 1,
// T3 = 2x T2 - x, then n-2 doublings T_{2k} = 2 T_k^2 - 1
void build_cheby_basis(Ciphertext &input, std::vector<Ciphertext> &chebyBasis, int n, CKKSEncoder &encoder,
                       Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                       RelinKeys &relin_keys);

// PolyApprox.cpp:103-305: the two composite-sign polynomials f and g in the Chebyshev basis
void compute_sign_f(Ciphertext &input, Ciphertext &output, CKKSEncoder &encoder, Encryptor &encryptor,
                    Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);
void compute_sign_g(Ciphertext &input, Ciphertext &output, CKKSEncoder &encoder, Encryptor &encryptor,
                    Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);

// PolyApprox.cpp:308-334: sign(x) ~ f^(df) o g^(dg) (x), applied in pairs
void sign_function(const Ciphertext &input, Ciphertext &output, int df, int dg, CKKSEncoder &encoder,
                   Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                   RelinKeys &relin_keys);

// PolyApprox.cpp:336-433: the two GELU pieces
void compute_gelu_p(Ciphertext &input, Ciphertext &output, CKKSEncoder &encoder, Encryptor &encryptor,
                    Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);
void compute_gelu_q(Ciphertext &input, Ciphertext &output, CKKSEncoder &encoder, Encryptor &encryptor,
                    Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);

// PolyApprox.cpp:443-504: piecewise GELU = b1 p(x) + b2 q(x) + b3 x with b from three signs
void compute_gelu(Ciphertext &inputs, Ciphertext &outputs, CKKSEncoder &encoder, Encryptor &encryptor,
                  Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);

// PolyApprox.cpp:511-531: exp(x) ~ (1 + x/2^r)^(2^r)
void compute_exp(Ciphertext &input, Ciphertext &output, int r, CKKSEncoder &encoder, Encryptor &encryptor,
                 Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);

// IterApprox.cpp:15-68: Goldschmidt 1/x (inputs normalised by 0.001)
void compute_inverse(Ciphertext &input, Ciphertext &output, int iters, CKKSEncoder &encoder, Encryptor &encryptor,
                     Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);

// util.cpp:266-275 (decrypt + re-encrypt at the top level; the reference's bootstrapping stand-in)
void fakeBootstrap(Ciphertext &input, Ciphertext &output, CKKSEncoder &encoder, Encryptor &encryptor,
                   Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);
// IterApprox.cpp:69-120 / :128-166 / :168-246
void taylor_expand(Ciphertext &input, Ciphertext &output, int iters, double guess, CKKSEncoder &encoder,
                   Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                   RelinKeys &relin_keys);
void compute_inv_sqrt(Ciphertext &input, Ciphertext &output, int iters, double guess, CKKSEncoder &encoder,
                      Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                      RelinKeys &relin_keys);
void compute_layernorm(Ciphertext &input, Ciphertext &output, std::vector<double> gamma, std::vector<double> beta,
                       int row_size, CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor,
                       Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);

// PolyApprox.cpp:595-649: softmax over rows of 128 packed at slot i*256 with a fixed shift gamma in
// place of the row max (exp, masked fold + quickSum, Goldschmidt inverse); in place on `input`.
// (compute_softmax, with the bootstrapped row max, is declared below.)
void compute_smax(Ciphertext &input, int r, int gamma, CKKSEncoder &encoder, Encryptor &encryptor,
                  Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);

// Fold.cpp:20-45: out = sum of input rotated by 0, 1, 2, ..., n/2 (log2(n) rotate+add steps)
void quickSum(Ciphertext &input, Ciphertext &output, int n, CKKSEncoder &encoder, Encryptor &encryptor,
              Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);

// util.cpp:292-301: keep slots [start, start+length), rescaled
void mask_out(Ciphertext &cipher, Ciphertext &out, int start, int length, CKKSEncoder &encoder, Evaluator &evaluator,
              RelinKeys &relin_keys);

// util.cpp:303-316: row i of v at slot i * 2 * round_to_2(row_size) (32768-slot ciphertexts)
void pack_plain_row(std::vector<std::vector<double>> &v, int rows, int row_size,
                    std::vector<std::vector<double>> &out);

// pack.cpp:153-178: pack_plain_row + encode at ENCODE_SCALE + encrypt
void pack_from_row(std::vector<std::vector<double>> &input, std::vector<Ciphertext> &output, CKKSEncoder &encoder,
                   Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                   RelinKeys &relin_keys);

// util.cpp:277-290: num_ciphers encryptions of zero at ENCODE_SCALE
void init_output(int num_ciphers, std::vector<Ciphertext> &output, CKKSEncoder &encoder, Encryptor &encryptor,
                 Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);

// MatrixMul.cpp:118-188: A x W^T for row-packed A (A_rows x A_cols) and W (W_rows x W_cols), both
// encrypted; per (input, weight, chunk rotation): rotate, multiply, fold, quickSum, then every chunk
// is masked and rotated into its output position; bias added at the end
void row_matrix_multiplication_seal(std::vector<Ciphertext> &left_inputs, std::vector<Ciphertext> &weights,
                                    Ciphertext bias, std::vector<Ciphertext> &outputs, int A_rows, int A_cols,
                                    int W_rows, int W_cols, CKKSEncoder &encoder, Encryptor &encryptor,
                                    Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                                    RelinKeys &relin_keys);

// The rotation steps of the reference's INIT() (gpt2/util.h:36-74): powers of two below N/2, the
// listed rotation_kinds and the multiples of 2048
// util.cpp:344-356: rotate right by shift_amt with a Galois key generated for that one step
void surefire_rotate(Ciphertext &cipher, int shift_amt, seal::KeyGenerator &keygen, Evaluator &evaluator);

// MatrixMul.cpp:244-358 / :360-478: attention projections into 12 heads (outputs[0..11]), as
// written in the reference (weights-only working ciphertexts, placement rotations by 0 steps)
void attn_proj_row_seal(std::vector<Ciphertext> &left_inputs, std::vector<Ciphertext> &weights, Ciphertext bias,
                        std::vector<Ciphertext> &outputs, int A_rows, int A_cols, int W_rows, int W_cols,
                        seal::KeyGenerator &keygen, CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor,
                        Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);
void attn_proj_col_seal(std::vector<Ciphertext> &left_inputs, std::vector<Ciphertext> &weights, Ciphertext bias,
                        std::vector<Ciphertext> &outputs, int A_rows, int A_cols, int W_rows, int W_cols,
                        seal::KeyGenerator &keygen, CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor,
                        Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);

// MatrixMul.cpp:480-533 / :535-584: Q.K^T scores into rows of 256 slots, and S.V back into the
// 2048-slot row layout (outputs[0..127]); every placement uses surefire_rotate
void qk_matmul(std::vector<Ciphertext> &Q, std::vector<Ciphertext> &K, std::vector<Ciphertext> &outputs, int A_rows,
               int A_cols, int W_rows, int W_cols, seal::KeyGenerator &keygen, CKKSEncoder &encoder,
               Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
               RelinKeys &relin_keys);
void sv_matmul(std::vector<Ciphertext> &S, std::vector<Ciphertext> &V, std::vector<Ciphertext> &outputs, int A_rows,
               int A_cols, int W_rows, int W_cols, seal::KeyGenerator &keygen, CKKSEncoder &encoder,
               Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
               RelinKeys &relin_keys);

// MatrixMul.cpp:586-628 / :630-649 / :651-725: the reference's benchmark-shaped kernels over
// weights["test"] (cipher_plain_128_128 writes no output, as in the reference)
void cipher_plain_128_128(Ciphertext &left_input, std::unordered_map<std::string, std::vector<double>> &weights,
                          Ciphertext bias, std::vector<Ciphertext> &outputs, int A_rows, int A_cols, int W_rows,
                          int W_cols, seal::KeyGenerator &keygen, CKKSEncoder &encoder, Encryptor &encryptor,
                          Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);
void batch_matmul(std::vector<Ciphertext> &left_inputs, std::unordered_map<std::string, std::vector<double>> &weights,
                  Ciphertext bias, std::vector<Ciphertext> &outputs, int A_rows, int A_cols, int W_rows, int W_cols,
                  seal::KeyGenerator &keygen, CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor,
                  Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);
void qk_matmul_col(std::vector<Ciphertext> &left_input, std::vector<Ciphertext> &right_input,
                   std::unordered_map<std::string, std::vector<double>> &weights, Ciphertext bias,
                   std::vector<Ciphertext> &outputs, int A_rows, int A_cols, int W_rows, int W_cols,
                   seal::KeyGenerator &keygen, CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor,
                   Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);

std::vector<int> gpt2_rotation_steps(int logN);

// ---- bootstrapped pieces (full-slot Bootstrapper, logn = logN - 1, as the reference's GPT-2 tests)
// util.cpp:317-326: mod-switch to the last level, then bootstrap_3.  With >= 2 limbs the message is
// first divided by kappa (one rescale, input scale reinterpreted as Delta / kappa) so that the sine
// step of the modular reduction works on x / (8 kappa) instead of x / 8 (gpt2.cpp); kappa = 32 by
// default, 1 reproduces the reference exactly
void bootstrap(Ciphertext &ctxt, Ciphertext &rtn, Bootstrapper &bootstrapper, Evaluator &evaluator);
void set_bootstrap_prescale(double kappa);
double bootstrap_prescale();
// util.cpp:328-339
void init_bootstrap(Bootstrapper &bootstrapper, std::vector<int> &gal_steps_vector, int logn);
// Fold.cpp:47-88: max(a, b) = 0.5 ((a + b) + (a - b) sign(0.1 (a - b)))
void computeMax(Ciphertext &input1, Ciphertext &input2, Ciphertext &output, Bootstrapper &bootstrapper,
                CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator,
                GaloisKeys &gal_keys, RelinKeys &relin_keys);
// Fold.cpp:91-110: max over n consecutive slots (rotate by 1, 2, 4, ...), bootstrapping below 18 limbs
void quickMax(Ciphertext &input, Ciphertext &output, int n, Bootstrapper &bootstrapper, CKKSEncoder &encoder,
              Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
              RelinKeys &relin_keys);
// PolyApprox.cpp:533-593: softmax over rows of 128 at slot i*256 with the bootstrapped row max
void compute_softmax(Ciphertext &input, int r, Bootstrapper &bootstrapper, CKKSEncoder &encoder,
                     Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                     RelinKeys &relin_keys);

// ============================================================================ gpt2_block.cpp
// The transformer block (layers.cpp:3-72, which does not compile as written; the plain pipeline
// plain_approx/full_gpt2.py:94-147) over the packed layouts, for any rows / d_model / heads / d_ff
// whose heads fit one ciphertext.  Layouts and deviations: gpt2_block.cpp, DESIGN.md.
struct BlockDims
{
    int rows = 128, d_model = 768, heads = 12, d_ff = 3072;
};
// The weight of GELU's last piece (x for x >= 3): `reference` is b3 = 0.5 s2 as PolyApprox.cpp:484-485
// and plain_approx/poly.py:33 write it (+-x/4 outside the middle pieces); `indicator` (the block's
// default, a deliberate departure) is s2 + 1/2, the indicator of x >= 3 that GELU needs.
enum class GeluLastPiece
{
    indicator,
    reference
};
struct AttentionParams
{
    double masked_score = -5.0; // masked scores pinned here before the row max
    double inv_norm = 0.0;      // Goldschmidt normalisation of the row sums (0: 1 / rows)
    int inv_iters = 8;          // Goldschmidt steps
    int newton_iters = 3;       // layer-norm Newton steps
    double gelu_alpha = 0.1;    // GELU signs taken of alpha (x + shift)
    GeluLastPiece gelu_last = GeluLastPiece::indicator; // the block's GELU x piece (reference: poly.py's 0.5 s2)
};
struct PlainBlockWeights
{
    // row-major [in][out] as GPT-2's Conv1D (x W + b)
    std::vector<double> ln1_g, ln1_b, qw, qb, kw, kb, vw, vb, ow, ob, ln2_g, ln2_b, fc_w, fc_b, pj_w, pj_b;
};
// The FFN hidden state is held in d_model-wide column chunks, each row-packed like the block's input
// (FeedForwardLayer): fc_b holds one bias ciphertext per chunk, pj_w the packed W2 rows of chunk 0,
// then chunk 1, ...
struct BlockWeights
{
    std::vector<Ciphertext> qw, qb, kw, kb, vw, vb, ow, fc_w, fc_b, pj_w;
    Ciphertext ob, pj_b;
    std::vector<double> ln1_g, ln1_b, ln2_g, ln2_b;
};
struct BlockTrace
{
    std::vector<Ciphertext> ln1, attn, x1, ln2, ffn;
};

// pack.cpp / pack.py
std::vector<double> repeat(const std::vector<double> &input, int times);
void expand_bias(std::vector<double> &input, Ciphertext &output, CKKSEncoder &encoder, Encryptor &encryptor,
                 Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys,
                 int rows = -1);
void expand_bias_head_row(std::vector<double> &input, std::vector<Ciphertext> &output, int heads,
                          CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator,
                          GaloisKeys &gal_keys, RelinKeys &relin_keys, int rows = -1);
void expand_bias_head_col(std::vector<double> &input, std::vector<Ciphertext> &output, int heads, int rows, int cols,
                          CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator,
                          GaloisKeys &gal_keys, RelinKeys &relin_keys);
std::vector<std::vector<std::vector<double>>> unpack_heads(const std::vector<std::vector<double>> &heads, int num_ciphers,
                                                           int num_rows, int row_size);
void pack_heads(std::vector<Ciphertext> &input, std::vector<std::vector<double>> &output, int heads, int num_ciphers,
                int num_rows, int row_size, CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor,
                Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);
void pack_tight(std::vector<Ciphertext> &input, std::vector<Ciphertext> &output, CKKSEncoder &encoder,
                Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                RelinKeys &relin_keys);
void pack_tight(std::vector<Ciphertext> &input, std::vector<Ciphertext> &output, int rows, int row_size, int stride,
                CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator,
                GaloisKeys &gal_keys, RelinKeys &relin_keys);
void unpack_tight(std::vector<Ciphertext> &input, std::vector<Ciphertext> &output, CKKSEncoder &encoder,
                  Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                  RelinKeys &relin_keys);
void unpack_tight(std::vector<Ciphertext> &input, std::vector<Ciphertext> &output, int rows, int row_size, int stride,
                  CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator,
                  GaloisKeys &gal_keys, RelinKeys &relin_keys);
// optimize.cpp:4-40 (KV cache)
void augment_value_row(std::vector<Ciphertext> &A, std::vector<Ciphertext> &cached_val, int padded_row_size, int idx,
                       CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator,
                       GaloisKeys &gal_keys, RelinKeys &relin_keys);
void augment_value_col(std::vector<Ciphertext> &A, std::vector<Ciphertext> &cached_val, int padded_row_size, int idx,
                       CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator,
                       GaloisKeys &gal_keys, RelinKeys &relin_keys);

// block pieces
void row_matmul(std::vector<Ciphertext> &A, std::vector<Ciphertext> &W, std::vector<Ciphertext> bias,
                std::vector<Ciphertext> &outputs, int A_rows, int A_cols, int W_cols, CKKSEncoder &encoder,
                Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                RelinKeys &relin_keys);
void attn_proj_heads(std::vector<Ciphertext> &A, std::vector<Ciphertext> &W, std::vector<Ciphertext> &bias,
                     std::vector<Ciphertext> &outputs, int rows, int d_model, int heads, bool column_layout,
                     CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator,
                     GaloisKeys &gal_keys, RelinKeys &relin_keys);
void qk_heads(std::vector<Ciphertext> &Q, std::vector<Ciphertext> &K, std::vector<Ciphertext> &outputs, int rows,
              int head_dim, CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator,
              GaloisKeys &gal_keys, RelinKeys &relin_keys);
void sv_heads(std::vector<Ciphertext> &S, std::vector<Ciphertext> &V, std::vector<Ciphertext> &outputs, int rows,
              int head_dim, int d_model, CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor,
              Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);
void compute_inverse_norm(Ciphertext &input, Ciphertext &output, int iters, double normalize_factor,
                          CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator,
                          GaloisKeys &gal_keys, RelinKeys &relin_keys);
void compute_softmax_rows(Ciphertext &input, int n, const std::vector<double> &keep_mask, double inv_norm,
                          int inv_iters, Bootstrapper &bootstrapper, CKKSEncoder &encoder, Encryptor &encryptor,
                          Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);
void layer_norm_rows(Ciphertext &input, Ciphertext &output, const std::vector<double> &gamma,
                     const std::vector<double> &beta, int rows, int row_size, int newton_iters,
                     Bootstrapper &bootstrapper, CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor,
                     Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys);
void compute_gelu_block(Ciphertext &inputs, Ciphertext &outputs, double alpha, CKKSEncoder &encoder,
                        Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                        RelinKeys &relin_keys, GeluLastPiece last = GeluLastPiece::indicator);
// layers.cpp
void attentionLayer(std::vector<Ciphertext> &A, std::vector<Ciphertext> &qw, std::vector<Ciphertext> &qb,
                    std::vector<Ciphertext> &kw, std::vector<Ciphertext> &kb, std::vector<Ciphertext> &vw,
                    std::vector<Ciphertext> &vb, std::vector<Ciphertext> &w_out, Ciphertext &b_out,
                    const std::vector<std::vector<double>> &keep, std::vector<std::vector<Ciphertext>> &kv_cache,
                    std::vector<Ciphertext> &outputs, int rows, int cols, int heads, int idx,
                    const AttentionParams &params, Bootstrapper &bootstrapper, seal::KeyGenerator &keygen,
                    CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator,
                    GaloisKeys &gal_keys, RelinKeys &relin_keys);
void FeedForwardLayer(std::vector<Ciphertext> &A, std::vector<Ciphertext> &W1, std::vector<Ciphertext> &b1,
                      std::vector<Ciphertext> &W2, Ciphertext b2, std::vector<Ciphertext> &outputs, int rows, int cols,
                      int d_ff, double gelu_alpha, Bootstrapper &bootstrapper, CKKSEncoder &encoder,
                      Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                      RelinKeys &relin_keys, GeluLastPiece gelu_last = GeluLastPiece::indicator);
void transformer_block(std::vector<Ciphertext> &x, BlockWeights &w, const std::vector<std::vector<double>> &keep,
                       std::vector<Ciphertext> &y, const BlockDims &dims, const AttentionParams &params,
                       Bootstrapper &bootstrapper, seal::KeyGenerator &keygen, CKKSEncoder &encoder,
                       Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                       RelinKeys &relin_keys, BlockTrace *trace = nullptr);
// full_gpt2.py:17-78 for one block; ciphertexts dropped to `limbs` (<= 0: kept at the top level)
void encrypt_block_weights(const PlainBlockWeights &p, BlockWeights &w, const BlockDims &dims, CKKSEncoder &encoder,
                           Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                           RelinKeys &relin_keys, int limbs);
// the +-2^i steps every block rotation is composed from
std::vector<int> block_rotation_steps(int logN);
} // namespace gpt2
