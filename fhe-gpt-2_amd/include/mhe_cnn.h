// mhe_cnn.h -- the reference's multiplexed-packing CNN layers (TensorCipher and the linear
// layers of cnn_ckks/cpu-ckks/single-key/cnn/cnn_seal.h, plus the approximate ReLU) over the
// MI355X seal:: surface.
//
// Same class, function names, signatures and operation sequences as the reference
// (cnn_seal.cpp:3-100, 284-809), so a caller that builds against these gets the same
// ciphertext-operation trace, run on the GPU.  Bootstrapping (Bootstrapper) is not part of this
// header yet.
#pragma once

#include <fstream>
#include <vector>

#include "mhe_comp.h"
#include "seal/seal.h"

class TensorCipher
{
public:
    TensorCipher();
    // data: h*w*c values in the multiplexed layout (replicated p times by the caller); k must be 1
    TensorCipher(int logn, int k, int h, int w, int c, int t, int p, std::vector<double> data,
                 seal::Encryptor &encryptor, seal::CKKSEncoder &encoder, int logp);
    TensorCipher(int logn, int k, int h, int w, int c, int t, int p, seal::Ciphertext cipher);
    int k() const { return k_; }
    int h() const { return h_; }
    int w() const { return w_; }
    int c() const { return c_; }
    int t() const { return t_; }
    int p() const { return p_; }
    int logn() const { return logn_; }
    seal::Ciphertext cipher() const { return cipher_; }
    void set_ciphertext(seal::Ciphertext cipher) { cipher_ = std::move(cipher); }
    void print_parms();

private:
    int k_ = 0, h_ = 0, w_ = 0, c_ = 0, t_ = 0, p_ = 0, logn_ = 0;
    seal::Ciphertext cipher_;
};

void multiplexed_parallel_convolution_seal(const TensorCipher &cnn_in, TensorCipher &cnn_out, int co, int st, int fh,
                                           int fw, const std::vector<double> &data, std::vector<double> running_var,
                                           std::vector<double> constant_weight, double epsilon,
                                           seal::CKKSEncoder &encoder, seal::Encryptor &encryptor,
                                           seal::Evaluator &evaluator, seal::GaloisKeys &gal_keys,
                                           std::vector<seal::Ciphertext> &cipher_pool, bool end = false);
void multiplexed_parallel_batch_norm_seal(const TensorCipher &cnn_in, TensorCipher &cnn_out, std::vector<double> bias,
                                          std::vector<double> running_mean, std::vector<double> running_var,
                                          std::vector<double> weight, double epsilon, seal::CKKSEncoder &encoder,
                                          seal::Encryptor &encryptor, seal::Evaluator &evaluator, double B,
                                          bool end = false);
// cnn_seal.cpp:577-592: approximate ReLU (minimax composite polynomial, mhe_comp.h) of the tensor
void ReLU_seal(const TensorCipher &cnn_in, TensorCipher &cnn_out, long comp_no, std::vector<int> deg, long alpha,
               std::vector<Tree> &tree, double scaled_val, long scalingfactor, seal::Encryptor &encryptor,
               seal::Evaluator &evaluator, seal::Decryptor &decryptor, seal::CKKSEncoder &encoder,
               seal::PublicKey &public_key, seal::SecretKey &secret_key, seal::RelinKeys &relin_keys,
               double scale = 1.0);
void cnn_add_seal(const TensorCipher &cnn1, const TensorCipher &cnn2, TensorCipher &destination,
                  seal::Evaluator &evaluator);
void multiplexed_parallel_downsampling_seal(const TensorCipher &cnn_in, TensorCipher &cnn_out,
                                            seal::Evaluator &evaluator, seal::GaloisKeys &gal_keys);
void averagepooling_seal_scale(const TensorCipher &cnn_in, TensorCipher &cnn_out, seal::Evaluator &evaluator,
                               seal::GaloisKeys &gal_keys, double B, seal::CKKSEncoder &encoder,
                               seal::Decryptor &decryptor, std::ofstream &output);
void matrix_multiplication_seal(const TensorCipher &cnn_in, TensorCipher &cnn_out, std::vector<double> matrix,
                                std::vector<double> bias, int q, int r, seal::Evaluator &evaluator,
                                seal::GaloisKeys &gal_keys);
void memory_save_rotate(const seal::Ciphertext &cipher_in, seal::Ciphertext &cipher_out, int steps,
                        seal::Evaluator &evaluator, seal::GaloisKeys &gal_keys);

// helpers of the reference's common/MinicompFunc.cpp:15-46 used by the layer code
long pow2(long n);
int floor_to_int(double x);
long log2_long(long n);
