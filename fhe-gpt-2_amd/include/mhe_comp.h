// mhe_comp.h -- homomorphic comparison / approximate ReLU of the reference
// (cnn_ckks/cpu-ckks/single-key/comp/{SEALcomp,SEALfunc,program}.cpp and the Tree of
// common/PolyUpdate.cpp) over the MI355X seal:: surface.
//
// A minimax composite polynomial p_k o ... o p_1 approximates sgn(x); ReLU(x) = x (1 + sgn x) / 2.
// Each component is evaluated in the Chebyshev basis with the "odd baby-step giant-step" (or
// "baby") evaluation tree found by a small dynamic program (upgrade_oddbaby / upgrade_baby); the
// tree's leaf coefficients come from an offline Remez step and are read from text
// (result/d<alpha>.txt in the reference).  Same names, signatures and operation sequence as the
// reference, so the ciphertext-operation trace is the reference's, run on the GPU.
#pragma once

#include <string>
#include <vector>

#include "seal/seal.h"

enum class evaltype : int
{
    none = 0,
    oddbaby = 1,
    baby = 2,
};

namespace minicomp
{
// Evaluation tree (common/PolyUpdate.h:29-45): tree[1] is the root's split degree g, tree[2i] /
// tree[2i+1] its children; 0 marks a leaf, -1 an absent node.
class Tree
{
public:
    int depth = 0;
    evaltype type = evaltype::none;
    std::vector<int> tree{ -1, 0 };
    int m = 0, l = 0, b = 0;

    Tree() = default;
    explicit Tree(evaltype ty) : type(ty) {}
    Tree(const Tree &a, const Tree &b, int g) { merge(a, b, g); }
    void clear();
    void merge(const Tree &a, const Tree &b, int g);
    void print() const;
};

long num_one(long n);
long coeff_number(long deg, Tree &tree);
} // namespace minicomp

using minicomp::Tree;

// Optimal evaluation trees for an odd-degree (oddbaby) or any-degree (baby) polynomial
// (comp/program.cpp:3-157).
void upgrade_oddbaby(long n, Tree &tree);
void upgrade_baby(long n, Tree &tree);

namespace seal
{
void eval_polynomial_integrate(Encryptor &encryptor, Evaluator &evaluator, Decryptor &decryptor, CKKSEncoder &encoder,
                               PublicKey &public_key, SecretKey &secret_key, RelinKeys &relin_keys, Ciphertext &res,
                               Ciphertext &cipher, long deg, const std::vector<double> &decomp_coeff, Tree &tree);
} // namespace seal

// comp/SEALcomp.cpp:3-60.  Coefficients are read from <dir>/d<alpha>.txt, dir = $MHE_COMP_DIR or
// "../result" (the reference's relative path).
void minimax_ReLU_seal(long comp_no, std::vector<int> deg, long alpha, std::vector<Tree> &tree, double scaled_val,
                       long scalingfactor, seal::Encryptor &encryptor, seal::Evaluator &evaluator,
                       seal::Decryptor &decryptor, seal::CKKSEncoder &encoder, seal::PublicKey &public_key,
                       seal::SecretKey &secret_key, seal::RelinKeys &relin_keys, seal::Ciphertext &cipher_in,
                       seal::Ciphertext &cipher_res);

// minimax_ReLU_seal restated on plain doubles (same coefficients, scalings and evaluation trees), for
// checking a decrypted network against its plain twin: u -> u (1 + sgn~(u)) / 2.
class MinimaxReluPlain
{
public:
    MinimaxReluPlain(long comp_no, std::vector<int> deg, long alpha, std::vector<Tree> tree, double scaled_val);
    double operator()(double u) const;

private:
    double eval_component(long c, double x) const;
    long comp_no_;
    std::vector<int> deg_;
    std::vector<Tree> tree_;
    std::vector<std::vector<double>> coeff_;
};
