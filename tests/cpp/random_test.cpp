// random_test: keys and encryptions from SEAL's randomness on the GPU, written out for the
// oracle comparison in tests/test_gpu_random.py.  The parameters carry a seeded
// Blake2xbPRNGFactory (SEAL's debug seed {1..8}), so every PRNG the library creates has that seed
// (randomgen.h:405-470), exactly as SEAL with the same factory.
//   random_test <out_dir> <log_n> <hamming_weight> <bits...>
#include "seal/seal.h"

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

using namespace seal;

static void dump(const std::string &path, const std::uint64_t *p, std::size_t words)
{
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char *>(p), (std::streamsize)(words * 8));
}

int main(int argc, char **argv)
{
    if (argc < 5)
    {
        std::fprintf(stderr, "usage: random_test out_dir log_n hw bits...\n");
        return 2;
    }
    const std::string dir = argv[1];
    const int log_n = std::atoi(argv[2]);
    const std::size_t hw = (std::size_t)std::atoi(argv[3]);
    std::vector<int> bits;
    for (int i = 4; i < argc; i++) bits.push_back(std::atoi(argv[i]));
    const std::size_t n = (std::size_t)1 << log_n, K = bits.size();

    EncryptionParameters parms(scheme_type::ckks);
    parms.set_poly_modulus_degree(n);
    parms.set_coeff_modulus(CoeffModulus::Create(n, bits));
    parms.set_secret_key_hamming_weight(hw);
    parms.set_random_generator(std::make_shared<Blake2xbPRNGFactory>(prng_seed_type{ 1, 2, 3, 4, 5, 6, 7, 8 }));
    SEALContext ctx(parms, true, sec_level_type::none);
    KeyGenerator keygen(ctx);
    dump(dir + "/sk.bin", keygen.secret_key().data().data(), K * n);
    PublicKey pk;
    keygen.create_public_key(pk);
    dump(dir + "/pk.bin", pk.data().data(), 2 * K * n);
    RelinKeys rk;
    keygen.create_relin_keys(rk);
    dump(dir + "/relin.bin", rk.key(0).host(), (K - 1) * 2 * K * n);
    GaloisKeys gk;
    keygen.create_galois_keys(std::vector<int>{ 1 }, gk);
    const std::uint32_t elt = 5; // step 1 (galois.cpp:53-76, generator 5)
    dump(dir + "/galois1.bin", gk.key(GaloisKeys::get_index(elt)).host(), (K - 1) * 2 * K * n);
    // the same key truncated to 2-limb ciphertexts: digits 0,1 over primes q_0, q_1, P
    GaloisKeys gt;
    keygen.create_galois_keys(std::vector<std::pair<std::uint32_t, std::size_t>>{ { elt, 2 } }, gt);
    dump(dir + "/galois1_trunc2.bin", gt.key(GaloisKeys::get_index(elt)).host(), 2 * 2 * 3 * n);
    if (gt.limbs_of(GaloisKeys::get_index(elt)) != 3) return 3;

    Encryptor enc(ctx, pk);
    Ciphertext ct;
    enc.encrypt_zero(ct); // first level: drawn at the key level, divided and rounded by P
    dump(dir + "/asym_first.bin", ct.data(), 2 * (K - 1) * n);
    auto cd = ctx.first_context_data();
    while (cd->parms().coeff_modulus().size() > 2) cd = cd->next_context_data();
    Ciphertext ct2;
    enc.encrypt_zero(cd->parms_id(), ct2); // 2 limbs: drawn at 3, rounded by q_2
    dump(dir + "/asym_l2.bin", ct2.data(), 2 * 2 * n);
    Encryptor sym(ctx, keygen.secret_key());
    Ciphertext ct3;
    sym.encrypt_zero_symmetric(ct3);
    dump(dir + "/sym_first.bin", ct3.data(), 2 * (K - 1) * n);
    std::printf("random_test ok: n=%zu K=%zu hw=%zu\n", n, K, hw);
    return 0;
}
