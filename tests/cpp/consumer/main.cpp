// Minimal reference-style caller (cnn/infer_seal.cpp shape): parameters, keys, encode,
// encrypt, one HMult, decrypt.  Built on CPU by tests/test_seal_api.py; runs on a GPU.
#include "seal/seal.h"

#include <cmath>
#include <cstdio>
#include <vector>

int main()
{
    using namespace seal;
    EncryptionParameters parms(scheme_type::ckks);
    parms.set_poly_modulus_degree(4096);
    parms.set_coeff_modulus(CoeffModulus::Create(4096, { 60, 40, 40, 60 }));
    SEALContext context(parms, true, sec_level_type::none);
    KeyGenerator keygen(context);
    PublicKey pk;
    keygen.create_public_key(pk);
    RelinKeys rlk;
    keygen.create_relin_keys(rlk);
    CKKSEncoder encoder(context);
    Encryptor encryptor(context, pk);
    Decryptor decryptor(context, keygen.secret_key());
    Evaluator evaluator(context, encoder);
    std::vector<double> x(encoder.slot_count());
    for (std::size_t i = 0; i < x.size(); i++) x[i] = 0.5 * std::cos(0.01 * i);
    Plaintext pt;
    encoder.encode(x, std::pow(2.0, 40), pt);
    Ciphertext ct;
    encryptor.encrypt(pt, ct);
    evaluator.square_inplace(ct);
    evaluator.relinearize_inplace(ct, rlk);
    evaluator.rescale_to_next_inplace(ct);
    decryptor.decrypt(ct, pt);
    std::vector<double> y;
    encoder.decode(pt, y);
    double err = 0;
    for (std::size_t i = 0; i < x.size(); i++) err = std::fmax(err, std::fabs(y[i] - x[i] * x[i]));
    std::printf("max error %.3g\n", err);
    return err < 1e-5 ? 0 : 1;
}
