// Serialization of the SEAL surface (fhe-gpt-2_amd/seal/serialize.cpp): SEAL 3.6's byte format for
// Ciphertext / Plaintext and SEAL's BLAKE2b parms_id.
//   serialize_test parms            -- host only: prints the parms_id of the CNN chain (checked
//                                      against hashlib.blake2b by tests/test_serialize.py)
//   serialize_test roundtrip <dir>  -- GPU: save/load round trips (stream and buffer), decrypts after
//                                      load, rejects corrupt streams; writes ct.bin / pt.bin into
//                                      <dir> for the independent Python parser of the format
// Follows the reference's SEAL tests CiphertextTest.SaveLoadCiphertext and
// PlaintextTest.SaveLoadPlaintext (native/tests/seal/ciphertext.cpp, plaintext.cpp).
#include "seal/seal.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

using namespace seal;

static int g_fail = 0;
#define CHECK(cond)                                                                  \
    do                                                                               \
    {                                                                                \
        if (!(cond))                                                                 \
        {                                                                            \
            g_fail++;                                                                \
            std::fprintf(stderr, "  FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond); \
        }                                                                            \
    } while (0)

template <typename F>
static bool throws(F f)
{
    try
    {
        f();
    }
    catch (const std::exception &)
    {
        return true;
    }
    return false;
}

static EncryptionParameters cnn_parms(std::size_t n)
{
    // cnn/infer_seal.cpp:306-310 chain: {51} + 30 x {46} + {51 special}
    EncryptionParameters parms(scheme_type::ckks);
    parms.set_poly_modulus_degree(n);
    std::vector<int> bits{ 51 };
    for (int i = 0; i < 30; i++) bits.push_back(46);
    bits.push_back(51);
    parms.set_coeff_modulus(CoeffModulus::Create(n, bits));
    return parms;
}

static void print_id(const char *tag, const parms_id_type &id)
{
    std::printf("%s", tag);
    for (auto w : id) std::printf(" %016llx", (unsigned long long)w);
    std::printf("\n");
}

int main(int argc, char **argv)
{
    const std::string mode = argc > 1 ? argv[1] : "parms";
    if (mode == "parms")
    {
        for (std::size_t n : { 1u << 12, 1u << 16 })
        {
            auto p = cnn_parms(n);
            std::printf("moduli %zu", n);
            for (auto &m : p.coeff_modulus()) std::printf(" %llu", (unsigned long long)m.value());
            std::printf("\n");
            print_id("parms_id", p.parms_id());
        }
        return 0;
    }
    const std::string dir = argc > 2 ? argv[2] : ".";
    const std::size_t n = 1 << 13;
    EncryptionParameters parms(scheme_type::ckks);
    parms.set_poly_modulus_degree(n);
    parms.set_coeff_modulus(CoeffModulus::Create(n, { 51, 46, 46, 51 }));
    SEALContext ctx(parms, true, sec_level_type::none);
    KeyGenerator keygen(ctx);
    PublicKey pk;
    keygen.create_public_key(pk);
    CKKSEncoder encoder(ctx);
    Encryptor encryptor(ctx, pk);
    Decryptor decryptor(ctx, keygen.secret_key());
    const double scale = std::pow(2.0, 46);
    std::vector<double> x(encoder.slot_count());
    for (std::size_t i = 0; i < x.size(); i++) x[i] = 0.5 * std::cos(0.001 * (double)i);
    Plaintext pt;
    encoder.encode(x, scale, pt);
    Ciphertext ct;
    encryptor.encrypt(pt, ct);
    print_id("first_parms_id", ctx.first_parms_id());
    CHECK(ctx.first_parms_id() == parms.parms_id() || ctx.key_parms_id() == parms.parms_id());

    // stream round trip
    std::stringstream ss;
    const auto wrote = ct.save(ss);
    CHECK(wrote == ct.save_size());
    CHECK((std::streamoff)ss.str().size() == wrote);
    Ciphertext ct2;
    const auto read = ct2.load(ctx, ss);
    CHECK(read == wrote);
    CHECK(ct2.parms_id() == ct.parms_id());
    CHECK(ct2.size() == ct.size() && ct2.coeff_modulus_size() == ct.coeff_modulus_size());
    CHECK(ct2.poly_modulus_degree() == n && ct2.is_ntt_form() && ct2.scale() == ct.scale());
    CHECK(std::memcmp(ct2.data(), ct.data(), 8 * ct.dyn_array_size()) == 0);
    Plaintext back;
    decryptor.decrypt(ct2, back);
    std::vector<double> y;
    encoder.decode(back, y);
    double err = 0;
    for (std::size_t i = 0; i < x.size(); i++) err = std::max(err, std::fabs(y[i] - x[i]));
    std::printf("decrypt after load: max error %.3g\n", err);
    CHECK(err < 1e-6);

    // buffer round trip, lower level
    Evaluator evaluator(ctx, encoder);
    Ciphertext low;
    evaluator.mod_switch_to_next(ct, low);
    std::vector<seal_byte> buf((std::size_t)low.save_size());
    CHECK(low.save(buf.data(), buf.size()) == (std::streamoff)buf.size());
    CHECK(throws([&] { low.save(buf.data(), buf.size() - 1); }));
    Ciphertext low2;
    low2.load(ctx, buf.data(), buf.size());
    CHECK(low2.parms_id() == low.parms_id() && low2.coeff_modulus_size() == low.coeff_modulus_size());
    CHECK(std::memcmp(low2.data(), low.data(), 8 * low.dyn_array_size()) == 0);

    // plaintext round trip
    std::stringstream ps;
    CHECK(pt.save(ps) == pt.save_size());
    Plaintext pt2;
    pt2.load(ctx, ps);
    CHECK(pt2.parms_id() == pt.parms_id() && pt2.scale() == pt.scale() && pt2.coeff_count() == pt.coeff_count());
    CHECK(std::memcmp(pt2.data(), pt.data(), 8 * pt.coeff_count()) == 0);

    // corrupt streams are rejected
    std::string good = [&] {
        std::stringstream t;
        ct.save(t);
        return t.str();
    }();
    auto load_str = [&](const std::string &s) {
        std::stringstream t(s);
        Ciphertext c;
        c.load(ctx, t);
    };
    CHECK(!throws([&] { load_str(good); }));
    std::string bad = good;
    bad[0] ^= 1; // magic
    CHECK(throws([&] { load_str(bad); }));
    bad = good;
    bad[5] = 2; // zstd
    CHECK(throws([&] { load_str(bad); }));
    bad = good;
    bad[16] ^= 0x40; // parms_id
    CHECK(throws([&] { load_str(bad); }));
    bad = good;
    std::uint64_t q0 = ctx.first_context_data()->parms().coeff_modulus()[0].value();
    std::memcpy(&bad[16 + 32 + 1 + 32 + 16 + 8], &q0, 8); // first residue = q_0: not canonical
    CHECK(throws([&] { load_str(bad); }));
    CHECK(throws([&] { load_str(good.substr(0, good.size() - 8)); })); // truncated

    // keys: RelinKeys / PublicKey round trips (kswitchkeys.cpp:42-140, publickey.h); relinearizing
    // with the loaded key is bit-identical, encrypting with the loaded public key decrypts
    RelinKeys rlk;
    keygen.create_relin_keys(rlk);
    std::stringstream ks;
    const auto kbytes = rlk.save(ks);
    CHECK(kbytes == rlk.save_size() && (std::streamoff)ks.str().size() == kbytes);
    const std::string kstr = ks.str();
    RelinKeys rlk2;
    CHECK(rlk2.load(ctx, ks) == kbytes);
    CHECK(rlk2.parms_id() == ctx.key_parms_id() && rlk2.has_key(2));
    Ciphertext sq1, sq2;
    evaluator.square(ct, sq1);
    sq2 = sq1;
    evaluator.relinearize_inplace(sq1, rlk);
    evaluator.relinearize_inplace(sq2, rlk2);
    CHECK(std::memcmp(sq1.data(), sq2.data(), 8 * sq1.dyn_array_size()) == 0);
    std::stringstream pks;
    pk.save(pks);
    PublicKey pk2;
    pk2.load(ctx, pks);
    Encryptor enc2(ctx, pk2);
    Ciphertext ct3;
    enc2.encrypt(pt, ct3);
    Plaintext back3;
    decryptor.decrypt(ct3, back3);
    std::vector<double> y3;
    encoder.decode(back3, y3);
    double err3 = 0;
    for (std::size_t i = 0; i < x.size(); i++) err3 = std::max(err3, std::fabs(y3[i] - x[i]));
    CHECK(err3 < 1e-6);
    GaloisKeys dgk;
    keygen.create_deferred_galois_keys(std::vector<int>{ 1 }, dgk); // client-side provider: holds the secret
    CHECK(throws([&] {
        std::stringstream t;
        dgk.save(t);
    }));
    {
        // eager Galois keys (SEAL's, the default) and a level-truncated one round-trip, and the
        // loaded keys rotate bit-identically
        GaloisKeys glk;
        keygen.create_galois_keys(std::vector<int>{ 1 }, glk);
        keygen.create_galois_keys(std::vector<std::pair<std::uint32_t, std::size_t>>{ { 25u, 2 } }, glk); // step 2
        std::stringstream gs;
        const auto gbytes = glk.save(gs);
        CHECK(gbytes == glk.save_size());
        GaloisKeys glk2;
        CHECK(glk2.load(ctx, gs) == gbytes);
        CHECK(glk2.has_key(5) && glk2.has_key(25) && glk2.limbs_of(GaloisKeys::get_index(25)) == 3);
        Ciphertext r1, r2;
        evaluator.rotate_vector(ct, 1, glk, r1);
        evaluator.rotate_vector(ct, 1, glk2, r2);
        CHECK(std::memcmp(r1.data(), r2.data(), 8 * r1.dyn_array_size()) == 0);
        Ciphertext low = ct, l1, l2;
        while (low.coeff_modulus_size() > 2) evaluator.mod_switch_to_next_inplace(low);
        evaluator.rotate_vector(low, 2, glk, l1);
        evaluator.rotate_vector(low, 2, glk2, l2);
        CHECK(std::memcmp(l1.data(), l2.data(), 8 * l1.dyn_array_size()) == 0);
        // a truncated key refuses a ciphertext above its level
        CHECK(throws([&] {
            Ciphertext t;
            evaluator.rotate_vector(ct, 2, glk2, t);
        }));
    }
    {
        std::string badk = kstr;
        badk[16] ^= 1; // parms_id
        std::stringstream t(badk);
        RelinKeys r;
        CHECK(throws([&] { r.load(ctx, t); }));
    }
    {
        std::ofstream kf(dir + "/relin.bin", std::ios::binary);
        kf << kstr;
    }

    // seeded objects (Serializable<T>, SEAL's seeded save: ciphertext.cpp:148-239, keygenerator.h:83-310):
    // the second polynomial of every symmetric encryption is written as its PRNG seed, and load()
    // expands it into the words a twin generation wrote.  A fixed-seed factory gives every
    // generator the same seed, so the Serializable and the plain creators draw identical objects.
    {
        EncryptionParameters sp = parms;
        sp.set_random_generator(
            std::make_shared<Blake2xbPRNGFactory>(prng_seed_type{ 11, 12, 13, 14, 15, 16, 17, 18 }));
        SEALContext sctx(sp, true, sec_level_type::none);
        KeyGenerator kg(sctx);
        CKKSEncoder senc(sctx);
        Plaintext spt;
        senc.encode(x, scale, spt);
        auto bytes_of = [](const auto &ser) {
            std::stringstream t;
            const auto w = ser.save(t);
            CHECK(w == ser.save_size() && (std::streamoff)t.str().size() == w);
            return t.str();
        };
        // ciphertext: encrypt_symmetric / encrypt_zero_symmetric
        Encryptor se(sctx, kg.secret_key());
        Ciphertext full, zfull;
        se.encrypt_symmetric(spt, full);
        const std::string sb = bytes_of(se.encrypt_symmetric(spt));
        const std::size_t Ln = full.coeff_modulus_size() * n;
        CHECK((std::streamoff)sb.size() == full.save_size() - (std::streamoff)(8 * Ln) + 81);
        Ciphertext back_s;
        {
            std::stringstream t(sb);
            CHECK(back_s.load(sctx, t) == (std::streamoff)sb.size());
        }
        CHECK(back_s.size() == 2 && back_s.scale() == full.scale() && back_s.parms_id() == full.parms_id());
        CHECK(std::memcmp(back_s.data(), full.data(), 8 * full.dyn_array_size()) == 0);
        se.encrypt_zero_symmetric(zfull);
        const std::string zb = bytes_of(se.encrypt_zero_symmetric());
        Ciphertext zback;
        {
            std::stringstream t(zb);
            zback.load(sctx, t);
        }
        CHECK(std::memcmp(zback.data(), zfull.data(), 8 * zfull.dyn_array_size()) == 0);
        // a lower level: the seed expands over that level's primes only
        Ciphertext lowfull;
        Plaintext lowpt;
        senc.encode(x, sctx.first_context_data()->next_context_data()->parms_id(), scale, lowpt);
        se.encrypt_symmetric(lowpt, lowfull);
        const std::string lb = bytes_of(se.encrypt_symmetric(lowpt));
        Ciphertext lowback;
        {
            std::stringstream t(lb);
            lowback.load(sctx, t);
        }
        CHECK(lowback.coeff_modulus_size() == lowfull.coeff_modulus_size() &&
              std::memcmp(lowback.data(), lowfull.data(), 8 * lowfull.dyn_array_size()) == 0);
        // decrypts after load
        Decryptor sdec(sctx, kg.secret_key());
        Plaintext sp_back;
        sdec.decrypt(back_s, sp_back);
        std::vector<double> ys;
        senc.decode(sp_back, ys);
        double es = 0;
        for (std::size_t i = 0; i < x.size(); i++) es = std::max(es, std::fabs(ys[i] - x[i]));
        std::printf("seeded ciphertext: %zu bytes (full %lld), decrypt error %.3g\n", sb.size(),
                    (long long)full.save_size(), es);
        CHECK(es < 1e-6);
        // public key, relin keys, Galois keys
        PublicKey pkf;
        kg.create_public_key(pkf);
        const std::string pb = bytes_of(kg.create_public_key());
        PublicKey pkb;
        {
            std::stringstream t(pb);
            pkb.load(sctx, t);
        }
        CHECK(std::memcmp(pkb.data().data(), pkf.data().data(), 8 * pkf.data().dyn_array_size()) == 0);
        RelinKeys rkf;
        kg.create_relin_keys(rkf);
        const std::string rb = bytes_of(kg.create_relin_keys());
        RelinKeys rkb;
        {
            std::stringstream t(rb);
            CHECK(rkb.load(sctx, t) == (std::streamoff)rb.size());
        }
        const std::size_t ri = RelinKeys::get_index(2);
        CHECK(rkb.has_key(2) && rkb.key(ri).words() == rkf.key(ri).words() &&
              std::memcmp(rkb.key(ri).host(), rkf.key(ri).host(), 8 * rkf.key(ri).words()) == 0);
        std::printf("seeded relin keys: %zu bytes (full %lld)\n", rb.size(), (long long)rkf.save_size());
        CHECK((std::streamoff)rb.size() < rkf.save_size() * 6 / 10);
        GaloisKeys gkf;
        kg.create_galois_keys(std::vector<int>{ 1, -1 }, gkf);
        const std::string gb = bytes_of(kg.create_galois_keys(std::vector<int>{ 1, -1 }));
        GaloisKeys gkb;
        {
            std::stringstream t(gb);
            gkb.load(sctx, t);
        }
        bool gsame = gkb.size() == gkf.size() && gkf.size() == 2;
        for (std::size_t i = 0; i < 2 * n && gsame; i++)
            if (gkf.has_index(i))
                gsame = gkb.has_index(i) && gkb.key(i).words() == gkf.key(i).words() &&
                        std::memcmp(gkb.key(i).host(), gkf.key(i).host(), 8 * gkf.key(i).words()) == 0;
        CHECK(gsame);
        // a public-key encryption has no seed: Serializable saves it in full
        Encryptor pe(sctx, pkf);
        Ciphertext pfull;
        pe.encrypt(spt, pfull);
        CHECK(pe.encrypt(spt).save_size() == pfull.save_size());
        CHECK(throws([&] { pe.encrypt_symmetric(spt); }));
        Encryptor both(sctx, pkf, kg.secret_key());
        CHECK(bytes_of(both.encrypt_symmetric(spt)) == sb);
        // corrupt seed records are rejected: PRNG type, info header size, truncation
        auto load_s = [&](const std::string &b) {
            std::stringstream t(b);
            Ciphertext c;
            c.load(sctx, t);
        };
        std::string bad = sb;
        bad[sb.size() - 65] = 2; // shake256 (not supported)
        CHECK(throws([&] { load_s(bad); }));
        bad = sb;
        bad[sb.size() - 65] = 7;
        CHECK(throws([&] { load_s(bad); }));
        bad = sb;
        bad[sb.size() - 81 + 8] ^= 1; // info record size
        CHECK(throws([&] { load_s(bad); }));
        CHECK(throws([&] { load_s(sb.substr(0, sb.size() - 10)); }));
        // for the Python check: the seeded file and its full twin (the oracle expands the seed)
        std::ofstream f1(dir + "/ct_seeded.bin", std::ios::binary), f2(dir + "/ct_twin.bin", std::ios::binary);
        f1 << sb;
        full.save(f2);
        std::ofstream f3(dir + "/relin_seeded.bin", std::ios::binary), f4(dir + "/relin_twin.bin", std::ios::binary);
        f3 << rb;
        rkf.save(f4);
        std::ofstream f5(dir + "/key_moduli.txt");
        for (auto &q : sctx.key_context_data()->parms().coeff_modulus()) f5 << q.value() << "\n";
    }

    // files for the Python-side format check
    {
        std::ofstream f(dir + "/ct.bin", std::ios::binary);
        ct.save(f);
        std::ofstream g(dir + "/pt.bin", std::ios::binary);
        pt.save(g);
        std::ofstream m(dir + "/moduli.txt");
        for (auto &q : ctx.first_context_data()->parms().coeff_modulus()) m << q.value() << "\n";
    }
    std::printf("%s\n", g_fail ? "FAILED" : "ok");
    return g_fail ? 1 : 0;
}
