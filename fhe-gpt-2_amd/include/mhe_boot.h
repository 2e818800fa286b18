// mhe_boot.h -- CKKS bootstrapping of the reference (cnn_ckks/cpu-ckks/single-key/ckks_bootstrapping/
// {Bootstrapper,ModularReducer}.{h,cpp} and the Chebyshev-heap evaluator of cnn_ckks/common/
// Polynomial.cpp) over the MI355X seal:: surface.
//
// Same class names, constructor arguments, public methods and ciphertext-operation sequences as
// the reference for the paths its CNN driver uses (cnn/infer_seal.cpp:287-388, 514-530):
// addLeftRotKeys_Linear_to_vector_3, addBootKeys_3, generate_LT_coefficient_3,
// prepare_mod_polynomial, bootstrap_real_3 / bootstrap_inplace_real_3 (sparse slots), with the
// three-level BSGS CoeffToSlot / SlotToCoeff (sflinv_3 / sfl_half_3), modraise, the Chebyshev
// cosine + double-angle modular reduction and the scaled linear arcsine (inverse_deg = 1).
//
// Host-side coefficient generation restates the reference's: the cosine and arcsine polynomials
// come from its multi-interval Remez exchange (common/Remez.cpp, NTL RR there) run in __float128
// (pinned by the reference's cosine.txt to every printed digit), and the linear-transform
// diagonals from genorigcoeff / genfftcoeff_3 / geninvfftcoeff_3 (Bootstrapper.cpp:512-592,
// 1116-1383, 1516-1776) with the reference's loops and operation order (lt_coefficients_3), so the
// encoded diagonals are the reference's doubles.  lt_coefficients_3_merged derives the same
// diagonals independently (products of sparse stage matrices) as the check.
// The evaluation trees, rotation steps, levels and scales are the reference's.
#pragma once

#include <complex>
#include <iosfwd>
#include <map>
#include <memory>
#include <functional>
#include <vector>

#include "seal/seal.h"

namespace boot
{
// A real polynomial in the Chebyshev basis on [-1, 1] (common/Polynomial.h).  `coeff` is the
// power-basis form, kept for the degree <= 3 evaluation branch; heaps are built by dividing by
// Chebyshev polynomials directly in the Chebyshev basis (exact identity, no power-basis round trip).
class Polynomial
{
public:
    std::vector<double> coeff;     // power basis
    std::vector<double> chebcoeff; // Chebyshev basis
    long deg = 0, heap_k = 0, heap_m = 0, heaplen = 0;
    std::vector<std::shared_ptr<Polynomial>> poly_heap;

    Polynomial() = default;
    explicit Polynomial(long deg);
    void set_chebyshev(const std::vector<double> &cheb); // deg = size - 1
    void set_zero_polynomial(long deg);
    void cheb_to_power();
    void constmul(double c);
    double evaluate(double x) const; // Chebyshev evaluation at x in [-1, 1]

    void generate_poly_heap_manual(long k, long m);
    void generate_poly_heap();     // babycount
    void generate_poly_heap_odd(); // oddbabycount
    void write_heap_to_file(std::ostream &out) const;
    void read_heap_from_file(std::istream &in);

    // Polynomial.cpp:256-560: deg <= 3 directly, else baby steps T_1..T_{k-1}, giant steps
    // T_k, T_2k, ..., leaves by multiply_const + add, combined up the heap.
    void homomorphic_poly_evaluation(seal::SEALContext &context, seal::CKKSEncoder &encoder,
                                     seal::Encryptor &encryptor, seal::Evaluator &evaluator,
                                     seal::RelinKeys &relin_keys, seal::Ciphertext &rtn, seal::Ciphertext &cipher,
                                     seal::Decryptor &decryptor);
};

// Merged special-FFT diagonals in the BSGS layout of the reference's *_3 transforms for n = 2^logn
// sparse slots: f1..f3 (SlotToCoeff, sfl_half_3) and i1..i3 (CoeffToSlot, sflinv_3), each a list
// of diagonals indexed as bsgs_linear_transform / rotated_bsgs_linear_transform expect.
using LTDiags = std::vector<std::vector<std::complex<double>>>;
void lt_coefficients_3(int logn, long logNh, long boundary_K, LTDiags &f1, LTDiags &f2, LTDiags &f3, LTDiags &i1,
                       LTDiags &i2, LTDiags &i3);
void lt_coefficients_3_merged(int logn, long logNh, long boundary_K, LTDiags &f1, LTDiags &f2, LTDiags &f3,
                              LTDiags &i1, LTDiags &i2, LTDiags &i3);

// target = quotient * T_chebdeg + remainder, all in the Chebyshev basis (Polynomial.cpp:890-916).
void divide_poly(Polynomial &quotient, Polynomial &remainder, const Polynomial &target, long chebdeg);
} // namespace boot

// common/func.cpp:90-213 (tree-shape searches and the BSGS giant-step size)
void oddbabycount(long &mink, long &minm, long deg);
void babycount(long &mink, long &minm, long deg);
int giantstep(int M);
// common/func.cpp:215-224: vec (length 2^logslot) rotated by shiftcount, repeated to Nh slots
void rotation(int logslot, int Nh, int shiftcount, const std::vector<std::complex<double>> &vec,
              std::vector<std::complex<double>> &rtnvec);

// common/Remez.cpp's exchange for any target (the reference's Remez::function_value), in binary128:
// the minimax polynomial sum_j c_j T_j(x / K) of f on the union of [i - 2^-log_width,
// i + 2^-log_width], |i| < K.  RemezCos / RemezArcsin below are this with their targets.
std::vector<double> remez_chebyshev(long K, double log_width, long deg, const std::function<__float128(__float128)> &f,
                                    double log_scan_step_diff = 9.5, int *iterations = nullptr,
                                    double *spread = nullptr);

// ckks_bootstrapping/RemezCos.h: cos(2 pi (x - 1/4) / scale_factor) (even scale_factor) or
// sin(2 pi x / scale_factor), approximated on the union of [i - 2^-log_width, i + 2^-log_width],
// |i| < boundary_K, in Chebyshev polynomials of x / boundary_K.
class RemezCos
{
public:
    long boundary_K, deg, scale_factor;
    double log_width;
    RemezCos(long boundary_K, double log_width, long deg, long scale_factor);
    void generate_optimal_poly(boot::Polynomial &poly) const;
    // the minimax Chebyshev coefficients by the Remez exchange (common/Remez.cpp), cached per
    // parameter set; optionally the iterations and the final relative spread of the alternation
    std::vector<double> chebyshev_coefficients(int *iterations = nullptr, double *spread = nullptr) const;
    double max_error(const boot::Polynomial &poly) const; // over the intervals (dense scan)
};

// ckks_bootstrapping/RemezArcsin.h: arcsin(x) / (2 pi) on [-2^-log_width, 2^-log_width].
class RemezArcsin
{
public:
    double log_width;
    long deg;
    RemezArcsin(double log_width, long deg);
    void generate_optimal_poly(boot::Polynomial &poly) const;
};

class ModularReducer
{
public:
    long boundary_K;
    double log_width;
    long deg;
    long num_double_formula;
    double inverse_log_width;
    long inverse_deg;
    double scale_inverse_coeff = 1.0;

    seal::SEALContext &context;
    seal::CKKSEncoder &encoder;
    seal::Encryptor &encryptor;
    seal::Evaluator &evaluator;
    seal::RelinKeys &relin_keys;
    seal::Decryptor &decryptor;

    RemezCos poly_generator;
    RemezArcsin inverse_poly_generator;
    boot::Polynomial sin_cos_polynomial;
    boot::Polynomial inverse_sin_polynomial;

    ModularReducer(long boundary_K, double log_width, long deg, long num_double_formula, long inverse_deg,
                   seal::SEALContext &context, seal::CKKSEncoder &encoder, seal::Encryptor &encryptor,
                   seal::Evaluator &evaluator, seal::RelinKeys &relin_keys, seal::Decryptor &decryptor);
    void double_angle_formula(seal::Ciphertext &cipher);
    void double_angle_formula_scaled(seal::Ciphertext &cipher, double scale_coeff);
    void generate_sin_cos_polynomial();
    void generate_inverse_sine_polynomial();
    void write_polynomials();
    void modular_reduction(seal::Ciphertext &rtn, seal::Ciphertext &cipher);
};

class Bootstrapper
{
public:
    long loge, logn, n, logNh, Nh, L;
    double initial_scale = 1.0, final_scale;
    long boundary_K, sin_cos_deg, scale_factor, inverse_deg;

    seal::SEALContext &context;
    seal::KeyGenerator &keygen;
    seal::CKKSEncoder &encoder;
    seal::Encryptor &encryptor;
    seal::Decryptor &decryptor;
    seal::Evaluator &evaluator;
    seal::RelinKeys &relin_keys;
    seal::GaloisKeys &gal_keys;

    std::vector<long> slot_vec;
    long slot_index = 0;
    // merged LT diagonals per slot_vec entry: [u][diagonal][slot]
    std::vector<std::vector<std::vector<std::complex<double>>>> fftcoeff1, fftcoeff2, fftcoeff3;
    std::vector<std::vector<std::vector<std::complex<double>>>> invfftcoeff1, invfftcoeff2, invfftcoeff3;

    std::unique_ptr<ModularReducer> mod_reducer;

    Bootstrapper(long loge, long logn, long logNh, long L, double final_scale, long boundary_K, long sin_cos_deg,
                 long scale_factor, long inverse_deg, seal::SEALContext &context, seal::KeyGenerator &keygen,
                 seal::CKKSEncoder &encoder, seal::Encryptor &encryptor, seal::Decryptor &decryptor,
                 seal::Evaluator &evaluator, seal::RelinKeys &relin_keys, seal::GaloisKeys &gal_keys);

    void addLeftRotKeys_Linear_to_vector_3(std::vector<int> &gal_steps_vector);
    void addBootKeys_3(seal::GaloisKeys &gal_keys);
    void change_logn(long new_logn);

    void generate_LT_coefficient_3();
    void prepare_mod_polynomial();

    void bsgs_linear_transform(seal::Ciphertext &rtncipher, seal::Ciphertext &cipher, int totlen, int basicstep,
                               int coeff_logn, const std::vector<std::vector<std::complex<double>>> &fftcoeff,
                               double coeff_scale = 1.0);
    void rotated_bsgs_linear_transform(seal::Ciphertext &rtncipher, seal::Ciphertext &cipher, int totlen,
                                       int basicstep, int coeff_logn,
                                       const std::vector<std::vector<std::complex<double>>> &fftcoeff,
                                       double coeff_scale = 1.0);

    void sfl_half_3(seal::Ciphertext &rtncipher, seal::Ciphertext &cipher);
    void sflinv_3(seal::Ciphertext &rtncipher, seal::Ciphertext &cipher);
    void coefftoslot_3(seal::Ciphertext &rtncipher, seal::Ciphertext &cipher);
    void slottocoeff_half_3(seal::Ciphertext &rtncipher, seal::Ciphertext &cipher);
    void modraise_inplace(seal::Ciphertext &cipher);

    void bootstrap_sparse_real_3(seal::Ciphertext &rtncipher, seal::Ciphertext &cipher);
    // full slots (logn == logNh; the GPT-2 path's bootstrap_3): Bootstrapper.cpp:2499-2760, 3250-3274
    void sfl_full_half_3(seal::Ciphertext &rtncipher, seal::Ciphertext &cipher);
    void sfl_full_3(seal::Ciphertext &rtncipher, seal::Ciphertext &cipher);
    void slottocoeff_full_3(seal::Ciphertext &rtncipher, seal::Ciphertext &cipher1, seal::Ciphertext &cipher2);
    void bootstrap_full_3(seal::Ciphertext &rtncipher, seal::Ciphertext &cipher);
    // Bootstrapper.cpp:3421-3431: complex bootstrapping (full slots)
    void bootstrap_3(seal::Ciphertext &rtncipher, seal::Ciphertext &cipher);
    void bootstrap_inplace_3(seal::Ciphertext &cipher);
    void sflinv_full_3(seal::Ciphertext &rtncipher, seal::Ciphertext &cipher);
    void coefftoslot_full_3(seal::Ciphertext &rtncipher1, seal::Ciphertext &rtncipher2, seal::Ciphertext &cipher);
    void slottocoeff_full_half_3(seal::Ciphertext &rtncipher, seal::Ciphertext &cipher1, seal::Ciphertext &cipher2);
    void bootstrap_full_real_3(seal::Ciphertext &rtncipher, seal::Ciphertext &cipher);

private:
    void sfl_full_common(seal::Ciphertext &rtncipher, seal::Ciphertext &cipher, bool half);

public:
    void bootstrap_real_3(seal::Ciphertext &rtncipher, seal::Ciphertext &cipher);
    void bootstrap_inplace_real_3(seal::Ciphertext &cipher);

    // plaintext cache of the LT diagonals (diagonal pointer, shift, level, scale) -> NTT plaintext;
    // the reference re-encodes every diagonal on every bootstrap
    std::size_t cached_plaintexts() const { return pt_cache_.size(); }
    std::size_t verify_cache(); // debugging aid: re-encode and compare every cached plaintext

private:
    // the giant-step rotations of a BSGS transform in batched launches, then the outer sum
    void giant_rotate_sum(std::vector<seal::Ciphertext> &giantct, std::vector<seal::Ciphertext> &rotct, int first,
                          int gs, int basicstep, seal::Ciphertext &rtncipher);
    void multiply_diag(seal::Ciphertext &ct, const std::vector<std::complex<double>> &diag, int coeff_logn,
                       int shift, seal::Ciphertext &dest, double coeff_scale = 1.0, bool accumulate = false);
    // the encoded, rotated diagonal multiply_diag multiplies by (cached, or built into `local`)
    const seal::Plaintext &diag_plain(seal::Ciphertext &ct, const std::vector<std::complex<double>> &diag, int coeff_logn,
                                      int shift, double coeff_scale, seal::Plaintext &local);
    // one giant step's inner sum: sum_j diag_j(babyct[j]) * babyct[j] into dest (multiply_plain_sum)
    void diag_sum(const std::vector<seal::Ciphertext *> &cts, const std::vector<const std::vector<std::complex<double>> *> &diags,
                  int coeff_logn, int shift, double coeff_scale, seal::Ciphertext &dest);
    struct PtKey
    {
        const void *diag;
        int shift;
        std::size_t limbs;
        double scale, coeff_scale;
        int coeff_logn;
        bool operator<(const PtKey &o) const;
    };
    std::map<PtKey, seal::Plaintext> pt_cache_;
};
