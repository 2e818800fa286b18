// End-to-end tests of the SEAL-compatible surface (libmhe_seal.so) on the GPU, written as a
// reference caller would use it.  They follow the reference GoogleTest cases
// (seal-modified-3.6.6/native/tests/seal/evaluator.cpp: CKKSEncryptAddDecrypt :183,
// AddPlain :346, SubPlain :564, MultiplyByNumber :1703, MultiplyRelin :1936, SquareRelin :2136,
// MultiplyRelinRescale :2315, SquareRelinRescale :2582, ModSwitch :2708,
// MultiplyRelinRescaleModSwitchAdd :2931, Rotate :3101, RescaleRotate :3255;
// encryptor.cpp CKKSEncryptZeroDecrypt :421, CKKSEncryptDecrypt :564; ckks.cpp encoder tests)
// at N = 2^12..2^13 (the engine's smallest rings), plus the modified-SEAL entry points
// (add/multiply_const, multiply_vector, *_reduced_error) and a multi-threaded case.
// Driven by tests/test_seal_api.py (GPU marker).
#include "seal/seal.h"

#include <cmath>
#include <complex>
#include <cstdio>
#include <functional>
#include <random>
#include <string>
#include <thread>
#include <vector>

using namespace seal;
using cplx = std::complex<double>;

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

template <typename E, typename F>
static bool throws(F f)
{
    try
    {
        f();
    }
    catch (const E &)
    {
        return true;
    }
    catch (...)
    {
        return false;
    }
    return false;
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

    Env(std::size_t n, std::vector<int> bits, bool galois = false, bool expand = true, std::size_t hw = 0)
    {
        parms.set_poly_modulus_degree(n);
        parms.set_coeff_modulus(CoeffModulus::Create(n, bits));
        if (hw) parms.set_secret_key_hamming_weight(hw);
        ctx = std::make_unique<SEALContext>(parms, expand, sec_level_type::none);
        keygen = std::make_unique<KeyGenerator>(*ctx);
        keygen->create_public_key(pk);
        if (ctx->using_keyswitching()) keygen->create_relin_keys(rlk);
        if (galois) keygen->create_galois_keys(glk);
        encoder = std::make_unique<CKKSEncoder>(*ctx);
        encryptor = std::make_unique<Encryptor>(*ctx, pk);
        decryptor = std::make_unique<Decryptor>(*ctx, keygen->secret_key());
        evaluator = std::make_unique<Evaluator>(*ctx, *encoder);
    }

    Ciphertext enc(const std::vector<cplx> &v, double scale, parms_id_type id)
    {
        Plaintext p;
        encoder->encode(v, id, scale, p);
        Ciphertext c;
        encryptor->encrypt(p, c);
        return c;
    }
    Ciphertext enc(const std::vector<cplx> &v, double scale) { return enc(v, scale, ctx->first_parms_id()); }
    std::vector<cplx> dec(const Ciphertext &c)
    {
        Plaintext p;
        decryptor->decrypt(c, p);
        std::vector<cplx> out;
        encoder->decode(p, out);
        return out;
    }
};

static std::vector<cplx> rand_vec(std::mt19937_64 &g, std::size_t n, double bound, bool complex = true)
{
    std::uniform_real_distribution<double> d(-bound, bound);
    std::vector<cplx> v(n);
    for (auto &x : v) x = cplx(d(g), complex ? d(g) : 0.0);
    return v;
}

static double max_err(const std::vector<cplx> &a, const std::vector<cplx> &b)
{
    double e = 0;
    for (std::size_t i = 0; i < std::min(a.size(), b.size()); i++) e = std::max(e, std::abs(a[i] - b[i]));
    return e;
}

static std::mt19937_64 rng(20261015);
static const std::vector<int> BITS = { 60, 40, 40, 40, 40, 60 };

static void test_encoder_roundtrip()
{
    EncryptionParameters parms(scheme_type::ckks);
    parms.set_poly_modulus_degree(4096);
    parms.set_coeff_modulus(CoeffModulus::Create(4096, { 60, 40, 40, 60 }));
    SEALContext ctx(parms, true, sec_level_type::none);
    CKKSEncoder encoder(ctx);
    CHECK(encoder.slot_count() == 2048);
    auto v = rand_vec(rng, 2048, 10.0);
    Plaintext p;
    encoder.encode(v, std::pow(2.0, 40), p);
    CHECK(p.parms_id() == ctx.first_parms_id());
    std::vector<cplx> out;
    encoder.decode(p, out);
    CHECK(out.size() == 2048);
    CHECK(max_err(v, out) < 1e-6);
    // single value: every slot holds it
    encoder.encode(-1.25, std::pow(2.0, 40), p);
    std::vector<double> re;
    encoder.decode(p, re);
    bool all = true;
    for (double x : re) all = all && std::fabs(x + 1.25) < 1e-6;
    CHECK(all);
    CHECK(throws<std::invalid_argument>([&] { encoder.encode(v, std::pow(2.0, 200), p); }));
    CHECK(throws<std::invalid_argument>([&] { encoder.encode(std::vector<cplx>(4096), 1e10, p); }));
}

static void test_encrypt_zero_and_decrypt()
{
    Env e(4096, BITS);
    for (auto id : { e.ctx->first_parms_id(), e.ctx->last_parms_id() })
    {
        Ciphertext c;
        e.encryptor->encrypt_zero(id, c);
        CHECK(c.parms_id() == id);
        c.scale() = std::pow(2.0, 30);
        auto out = e.dec(c);
        double m = 0;
        for (auto &x : out) m = std::max(m, std::abs(x));
        CHECK(m < 1e-3);
    }
    auto v = rand_vec(rng, 2048, 5.0);
    CHECK(max_err(e.dec(e.enc(v, std::pow(2.0, 40))), v) < 1e-4);
    // symmetric encryption
    Encryptor sym(*e.ctx, e.keygen->secret_key());
    Plaintext p;
    e.encoder->encode(v, std::pow(2.0, 40), p);
    Ciphertext c;
    sym.encrypt_symmetric(p, c);
    CHECK(max_err(e.dec(c), v) < 1e-4);
    // encrypt() is a public-key encryption in SEAL and throws without a public key
    bool threw = false;
    try
    {
        sym.encrypt(p, c);
    }
    catch (const std::logic_error &ex)
    {
        threw = std::string(ex.what()) == "public key is not set";
    }
    CHECK(threw);
}

static void test_add_sub_negate()
{
    Env e(4096, BITS);
    const double s = std::pow(2.0, 40);
    auto a = rand_vec(rng, 2048, 8.0), b = rand_vec(rng, 2048, 8.0);
    auto ca = e.enc(a, s), cb = e.enc(b, s);
    Ciphertext r;
    e.evaluator->add(ca, cb, r);
    std::vector<cplx> ex(2048);
    for (int i = 0; i < 2048; i++) ex[i] = a[i] + b[i];
    CHECK(max_err(e.dec(r), ex) < 1e-4);
    e.evaluator->sub(ca, cb, r);
    for (int i = 0; i < 2048; i++) ex[i] = a[i] - b[i];
    CHECK(max_err(e.dec(r), ex) < 1e-4);
    // destination aliasing encrypted2: SEAL computes encrypted1 - encrypted2 then negates
    Ciphertext cb2 = cb;
    e.evaluator->sub(ca, cb2, cb2);
    CHECK(max_err(e.dec(cb2), ex) < 1e-4);
    e.evaluator->negate(ca, r);
    for (int i = 0; i < 2048; i++) ex[i] = -a[i];
    CHECK(max_err(e.dec(r), ex) < 1e-4);
    std::vector<Ciphertext> many{ ca, cb, ca };
    e.evaluator->add_many(many, r);
    for (int i = 0; i < 2048; i++) ex[i] = 2.0 * a[i] + b[i];
    CHECK(max_err(e.dec(r), ex) < 1e-4);
    // plain add/sub (AddPlain :346, SubPlain :564)
    Plaintext pb;
    e.encoder->encode(b, s, pb);
    e.evaluator->add_plain(ca, pb, r);
    for (int i = 0; i < 2048; i++) ex[i] = a[i] + b[i];
    CHECK(max_err(e.dec(r), ex) < 1e-4);
    e.evaluator->sub_plain(ca, pb, r);
    for (int i = 0; i < 2048; i++) ex[i] = a[i] - b[i];
    CHECK(max_err(e.dec(r), ex) < 1e-4);
    // mismatches
    Ciphertext cs = e.enc(b, std::pow(2.0, 30));
    CHECK(throws<std::invalid_argument>([&] { e.evaluator->add_inplace(r, cs); }));
    Ciphertext cl = cb;
    e.evaluator->mod_switch_to_next_inplace(cl);
    CHECK(throws<std::invalid_argument>([&] { e.evaluator->add_inplace(r, cl); }));
}

static void test_multiply_relin_rescale()
{
    Env e(4096, BITS);
    const double s = std::pow(2.0, 40);
    auto next = e.ctx->first_context_data()->next_context_data()->parms_id();
    for (int round = 0; round < 10; round++)
    {
        std::vector<cplx> a(2048), b(2048), ex(2048);
        for (int i = 0; i < 2048; i++)
        {
            a[i] = (double)(rng() % 128);
            b[i] = (double)(rng() % 128);
            ex[i] = a[i] * b[i];
        }
        auto ca = e.enc(a, s), cb = e.enc(b, s);
        e.evaluator->multiply_inplace(ca, cb);
        CHECK(ca.size() == 3);
        CHECK(max_err(e.dec(ca), ex) < 0.5); // size-3 decryption (MultiplyRelin without relin)
        e.evaluator->relinearize_inplace(ca, e.rlk);
        CHECK(ca.size() == 2);
        CHECK(max_err(e.dec(ca), ex) < 0.5);
        e.evaluator->rescale_to_next_inplace(ca);
        CHECK(ca.parms_id() == next);
        CHECK(std::fabs(ca.scale() - s * s / (double)e.parms.coeff_modulus()[4].value()) < 1e-6 * ca.scale());
        CHECK(max_err(e.dec(ca), ex) < 0.5);
    }
    // square
    auto a = rand_vec(rng, 2048, 4.0);
    auto ca = e.enc(a, s);
    e.evaluator->square_inplace(ca);
    e.evaluator->relinearize_inplace(ca, e.rlk);
    e.evaluator->rescale_to_next_inplace(ca);
    std::vector<cplx> ex(2048);
    for (int i = 0; i < 2048; i++) ex[i] = a[i] * a[i];
    CHECK(max_err(e.dec(ca), ex) < 1e-3);
    // chain to the last level then "end of modulus switching chain reached"
    Ciphertext c = e.enc(rand_vec(rng, 2048, 1.0), s);
    while (c.parms_id() != e.ctx->last_parms_id()) e.evaluator->rescale_to_next_inplace(c), c.scale() = s;
    CHECK(throws<std::invalid_argument>([&] { e.evaluator->rescale_to_next_inplace(c); }));
    CHECK(throws<std::invalid_argument>([&] { e.evaluator->mod_switch_to_next_inplace(c); }));
}

static void test_multiply_by_number_and_consts()
{
    Env e(4096, BITS);
    const double s = std::pow(2.0, 40);
    auto a = rand_vec(rng, 2048, 4.0);
    auto ca = e.enc(a, s);
    // MultiplyByNumber (:1703): plaintext of a single value
    Plaintext p;
    e.encoder->encode(-2.5, s, p);
    Ciphertext r;
    e.evaluator->multiply_plain(ca, p, r);
    e.evaluator->rescale_to_next_inplace(r);
    std::vector<cplx> ex(2048);
    for (int i = 0; i < 2048; i++) ex[i] = -2.5 * a[i];
    CHECK(max_err(e.dec(r), ex) < 1e-3);
    // modified SEAL: multiply_const / add_const / multiply_vector (evaluator.cpp:287-310)
    e.evaluator->multiply_const(ca, 0.75, r);
    CHECK(std::fabs(r.scale() - s * s) < 1);
    e.evaluator->rescale_to_next_inplace(r);
    for (int i = 0; i < 2048; i++) ex[i] = 0.75 * a[i];
    CHECK(max_err(e.dec(r), ex) < 1e-3);
    e.evaluator->add_const_inplace(r, 1.5); // at a lower level: encoded at first, switched down
    for (int i = 0; i < 2048; i++) ex[i] += 1.5;
    CHECK(max_err(e.dec(r), ex) < 1e-3);
    std::vector<double> w(2048);
    for (int i = 0; i < 2048; i++) w[i] = std::sin(0.01 * i);
    Ciphertext rv;
    e.evaluator->multiply_vector(r, w, rv);
    e.evaluator->rescale_to_next_inplace(rv);
    for (int i = 0; i < 2048; i++) ex[i] *= w[i];
    CHECK(max_err(e.dec(rv), ex) < 1e-3);
    std::vector<cplx> wc(2048);
    for (int i = 0; i < 2048; i++) wc[i] = cplx(0.0, 1.0);
    Ciphertext rc;
    e.evaluator->multiply_vector(r, wc, rc);
    e.evaluator->rescale_to_next_inplace(rc);
    auto got = e.dec(rc), base = e.dec(r);
    for (int i = 0; i < 2048; i++) ex[i] = base[i] * cplx(0.0, 1.0);
    CHECK(max_err(got, ex) < 1e-3);
}

static void test_mod_switch()
{
    Env e(4096, BITS);
    const double s = std::pow(2.0, 40);
    auto a = rand_vec(rng, 2048, 4.0), b = rand_vec(rng, 2048, 4.0);
    auto ca = e.enc(a, s);
    Ciphertext c = ca;
    e.evaluator->mod_switch_to_next_inplace(c);
    CHECK(c.coeff_modulus_size() == 4);
    CHECK(max_err(e.dec(c), a) < 1e-4);
    e.evaluator->mod_switch_to_inplace(c, e.ctx->last_parms_id());
    CHECK(c.coeff_modulus_size() == 1);
    CHECK(max_err(e.dec(c), a) < 1e-3);
    CHECK(throws<std::invalid_argument>([&] { e.evaluator->mod_switch_to_inplace(c, e.ctx->first_parms_id()); }));
    Plaintext pb;
    e.encoder->encode(b, s, pb);
    e.evaluator->mod_switch_to_inplace(pb, e.ctx->last_parms_id());
    e.evaluator->add_plain_inplace(c, pb);
    std::vector<cplx> ex(2048);
    for (int i = 0; i < 2048; i++) ex[i] = a[i] + b[i];
    CHECK(max_err(e.dec(c), ex) < 1e-3);
    // MultiplyRelinRescaleModSwitchAdd (:2931)
    auto c1 = e.enc(a, s), c2 = e.enc(b, s), c3 = e.enc(b, s * s / (double)e.parms.coeff_modulus()[4].value());
    e.evaluator->multiply_inplace(c1, c2);
    e.evaluator->relinearize_inplace(c1, e.rlk);
    e.evaluator->rescale_to_next_inplace(c1);
    e.evaluator->mod_switch_to_next_inplace(c3);
    c3.scale() = c1.scale();
    e.evaluator->add_inplace(c1, c3);
    for (int i = 0; i < 2048; i++) ex[i] = a[i] * b[i] + b[i];
    CHECK(max_err(e.dec(c1), ex) < 1e-3);
    // NTT form round trip
    Ciphertext t = ca;
    e.evaluator->transform_from_ntt_inplace(t);
    CHECK(!t.is_ntt_form());
    CHECK(throws<std::invalid_argument>([&] { e.evaluator->transform_from_ntt_inplace(t); }));
    e.evaluator->transform_to_ntt_inplace(t);
    CHECK(max_err(e.dec(t), a) < 1e-4);
}

static void test_rotate()
{
    Env e(4096, BITS, true);
    const double s = std::pow(2.0, 40);
    const int slots = 2048;
    auto a = rand_vec(rng, slots, 4.0);
    for (int shift : { 1, 2, 3, 5, 64, 1023, -1, -7, 2047 })
    {
        Ciphertext c = e.enc(a, s), r;
        e.evaluator->rotate_vector(c, shift, e.glk, r);
        std::vector<cplx> ex(slots);
        for (int i = 0; i < slots; i++) ex[i] = a[((i + shift) % slots + slots) % slots];
        CHECK(max_err(e.dec(r), ex) < 1e-3);
    }
    Ciphertext c = e.enc(a, s);
    e.evaluator->complex_conjugate_inplace(c, e.glk);
    std::vector<cplx> ex(slots);
    for (int i = 0; i < slots; i++) ex[i] = std::conj(a[i]);
    CHECK(max_err(e.dec(c), ex) < 1e-4);
    // RescaleRotate (:3255): rotation at a lower level
    Ciphertext d = e.enc(a, s * (double)e.parms.coeff_modulus()[4].value());
    e.evaluator->rescale_to_next_inplace(d);
    e.evaluator->rotate_vector_inplace(d, 3, e.glk);
    for (int i = 0; i < slots; i++) ex[i] = a[(i + 3) % slots];
    CHECK(max_err(e.dec(d), ex) < 1e-3);
    CHECK(throws<std::invalid_argument>([&] { e.evaluator->rotate_vector_inplace(d, slots, e.glk); }));
    // keys for selected steps only: 3 = 4 - 1 through NAF
    GaloisKeys few;
    e.keygen->create_galois_keys(std::vector<int>{ 1, -1, 4 }, few);
    CHECK(few.size() == 3);
    Ciphertext f = e.enc(a, s);
    e.evaluator->rotate_vector_inplace(f, 3, few);
    for (int i = 0; i < slots; i++) ex[i] = a[(i + 3) % slots];
    CHECK(max_err(e.dec(f), ex) < 1e-3);
    CHECK(throws<std::invalid_argument>([&] { e.evaluator->rotate_vector_inplace(f, 2, few); }));
}

static void test_reduced_error_ops()
{
    Env e(8192, { 60, 50, 50, 50, 50, 50, 60 });
    const double s = std::pow(2.0, 50);
    auto a = rand_vec(rng, 4096, 2.0, false), b = rand_vec(rng, 4096, 2.0, false);
    auto ca = e.enc(a, s), cb = e.enc(b, s);
    // ca at a lower level than cb
    e.evaluator->multiply_const_inplace(ca, 1.0);
    e.evaluator->rescale_to_next_inplace(ca);
    std::vector<cplx> ex(4096);
    Ciphertext r;
    e.evaluator->add_reduced_error(ca, cb, r);
    CHECK(r.parms_id() == ca.parms_id());
    for (int i = 0; i < 4096; i++) ex[i] = a[i] + b[i];
    CHECK(max_err(e.dec(r), ex) < 1e-5);
    e.evaluator->add_reduced_error(cb, ca, r); // other branch (encrypted1 above encrypted2)
    CHECK(max_err(e.dec(r), ex) < 1e-5);
    e.evaluator->sub_reduced_error(ca, cb, r);
    for (int i = 0; i < 4096; i++) ex[i] = a[i] - b[i];
    CHECK(max_err(e.dec(r), ex) < 1e-5);
    e.evaluator->multiply_reduced_error(ca, cb, e.rlk, r);
    CHECK(r.size() == 2);
    e.evaluator->rescale_to_next_inplace(r);
    for (int i = 0; i < 4096; i++) ex[i] = a[i] * b[i];
    CHECK(max_err(e.dec(r), ex) < 1e-4);
    // same level: scale copied across
    Ciphertext x = e.enc(a, s), y = e.enc(b, s * 1.0000001);
    e.evaluator->add_inplace_reduced_error(x, y);
    CHECK(x.scale() == y.scale());
    // modified SEAL quirk kept: sub_reduced_error(e1, e2, e2) yields e2 - e1
    Ciphertext p = e.enc(a, s), q = e.enc(b, s);
    e.evaluator->sub_reduced_error(p, q, q);
    for (int i = 0; i < 4096; i++) ex[i] = b[i] - a[i];
    CHECK(max_err(e.dec(q), ex) < 1e-5);
    Ciphertext v = e.enc(a, s);
    std::vector<double> w(4096, 0.5);
    Ciphertext vr;
    e.evaluator->multiply_vector_reduced_error(v, w, vr);
    e.evaluator->rescale_to_next_inplace(vr);
    for (int i = 0; i < 4096; i++) ex[i] = 0.5 * a[i];
    CHECK(max_err(e.dec(vr), ex) < 1e-5);
    // fused multiply_plain + add_inplace_reduced_error: the same words as the two separate ops
    {
        Ciphertext acc1 = e.enc(a, s), acc2 = acc1, c = e.enc(b, s), t;
        Plaintext pw;
        e.evaluator->encode_vector_for(c, w, pw);
        e.evaluator->multiply_plain(c, pw, t);
        e.evaluator->add_inplace_reduced_error(acc1, t);
        e.evaluator->multiply_plain_add_reduced_error(acc2, c, pw);
        const std::uint64_t *p1 = acc1.data(), *p2 = acc2.data();
        std::size_t diff = 0;
        for (std::size_t k = 0; k < acc1.dyn_array_size(); k++) diff += p1[k] != p2[k];
        CHECK(diff == 0 && acc1.scale() == acc2.scale() && acc1.dyn_array_size() == acc2.dyn_array_size());
    }
    // cached static-vector encodings: bit-identical to encode_vector_for, built once per
    // (id, level, scale), and the builder is not called on a hit
    {
        Ciphertext c = e.enc(b, s), low = e.enc(b, s);
        e.evaluator->mod_switch_to_next_inplace(low);
        Plaintext fresh, scratch;
        e.evaluator->encode_vector_for(c, w, fresh);
        int built = 0;
        auto make = [&] {
            built++;
            return w;
        };
        const std::size_t before = e.evaluator->vector_cache_entries();
        const Plaintext &p1 = e.evaluator->cached_vector_plain(c, 7, 11, make, scratch);
        const Plaintext &p2 = e.evaluator->cached_vector_plain(c, 7, 11, make, scratch);
        CHECK(&p1 == &p2 && built == 1 && e.evaluator->vector_cache_entries() == before + 1);
        std::size_t diff = fresh.store().words() != p1.store().words();
        for (std::size_t k = 0; !diff && k < fresh.store().words(); k++)
            diff += fresh.store().host()[k] != p1.store().host()[k];
        CHECK(diff == 0 && p1.scale() == fresh.scale() && p1.parms_id() == fresh.parms_id());
        // another level (and another scale) is another entry
        const Plaintext &p3 = e.evaluator->cached_vector_plain(low, 7, 11, make, scratch);
        CHECK(&p3 != &p1 && built == 2 && p3.parms_id() == low.parms_id());
        c.scale() *= 2;
        const Plaintext &p4 = e.evaluator->cached_vector_plain(c, 7, 11, make, scratch);
        CHECK(&p4 != &p1 && built == 3 && p4.scale() == c.scale());
        // and a product through the cached plaintext equals multiply_vector_inplace
        Ciphertext m1 = e.enc(a, s), m2 = m1;
        e.evaluator->multiply_vector_inplace(m1, w);
        e.evaluator->multiply_plain_inplace(m2, e.evaluator->cached_vector_plain(m2, 7, 12, make, scratch));
        diff = 0;
        for (std::size_t k = 0; k < m1.dyn_array_size(); k++) diff += m1.data()[k] != m2.data()[k];
        CHECK(diff == 0);
    }
}

static void test_security_level()
{
    // context.cpp:207-220: a chain above CoeffModulus::MaxBitCount for the requested level is
    // flagged and refused by key generation; sec_level_type::none accepts it
    CHECK(CoeffModulus::MaxBitCount(4096) == 109 && CoeffModulus::MaxBitCount(65536) == 1792);
    CHECK(CoeffModulus::MaxBitCount(4096, sec_level_type::tc256) == 58);
    EncryptionParameters parms(scheme_type::ckks);
    parms.set_poly_modulus_degree(4096);
    parms.set_coeff_modulus(CoeffModulus::Create(4096, BITS)); // 280 bits > 109
    SEALContext strict(parms);
    CHECK(!strict.parameters_set() && strict.sec_level() == sec_level_type::none);
    CHECK(throws<std::invalid_argument>([&] { KeyGenerator k(strict); }));
    SEALContext lax(parms, true, sec_level_type::none);
    CHECK(lax.parameters_set());
    parms.set_coeff_modulus(CoeffModulus::Create(4096, { 36, 36, 36 })); // 108 bits
    SEALContext ok(parms);
    CHECK(ok.parameters_set() && ok.sec_level() == sec_level_type::tc128);
}

static void test_sparse_secret_and_slots()
{
    EncryptionParameters parms(scheme_type::ckks);
    parms.set_poly_modulus_degree(4096);
    parms.set_coeff_modulus(CoeffModulus::Create(4096, BITS));
    parms.set_secret_key_hamming_weight(64);
    parms.set_sparse_slots(256);
    SEALContext ctx(parms, true, sec_level_type::none);
    KeyGenerator keygen(ctx);
    PublicKey pk;
    keygen.create_public_key(pk);
    CKKSEncoder encoder(ctx);
    Encryptor enc(ctx, pk);
    Decryptor dec(ctx, keygen.secret_key());
    std::vector<cplx> base = rand_vec(rng, 256, 3.0), v(2048);
    for (int i = 0; i < 2048; i++) v[i] = base[i % 256];
    Plaintext p;
    encoder.encode(v, std::pow(2.0, 40), p);
    Ciphertext c;
    enc.encrypt(p, c);
    dec.decrypt(c, p);
    std::vector<cplx> out;
    encoder.decode(p, out);
    CHECK(out.size() == 256);
    CHECK(max_err(out, base) < 1e-4);
}

static void test_threads()
{
    // one Evaluator shared by several host threads (cnn/infer_seal.cpp:404 pattern): the input
    // is produced on the main thread's stream and consumed on the workers' streams.
    Env e(4096, BITS, true);
    const double s = std::pow(2.0, 40);
    auto a = rand_vec(rng, 2048, 2.0);
    Ciphertext shared = e.enc(a, s);
    e.evaluator->multiply_const_inplace(shared, 1.0);
    e.evaluator->rescale_to_next_inplace(shared);
    const int T = 6;
    std::vector<Ciphertext> outs(T);
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
            Ciphertext c;
            e.evaluator->rotate_vector(shared, t + 1, e.glk, c);
            e.evaluator->multiply_inplace(c, shared);
            e.evaluator->relinearize_inplace(c, e.rlk);
            e.evaluator->rescale_to_next_inplace(c);
            outs[t] = c;
        });
    for (auto &x : th) x.join();
    for (int t = 0; t < T; t++)
    {
        std::vector<cplx> ex(2048);
        for (int i = 0; i < 2048; i++) ex[i] = a[(i + t + 1) % 2048] * a[i];
        CHECK(max_err(e.dec(outs[t]), ex) < 1e-3);
    }
}

// without an explicit seed every KeyGenerator / Encryptor draws a fresh
// 512-bit Blake2xb seed from the OS (getrandom, seal/random.cpp): two of them never collide
static void test_fresh_seeds_differ()
{
    Env e(4096, BITS);
    KeyGenerator kg2(*e.ctx);
    const SecretKey &s1 = e.keygen->secret_key(), &s2 = kg2.secret_key();
    std::size_t same = 0, words = s1.data().coeff_count();
    for (std::size_t k = 0; k < words; k++) same += s1.data().data()[k] == s2.data().data()[k];
    CHECK(words > 0 && same < words); // sparse keys share zeros, never every word
    Plaintext p;
    e.encoder->encode(rand_vec(rng, 2048, 1.0), std::pow(2.0, 40), p);
    Ciphertext c1, c2;
    e.encryptor->encrypt(p, c1);
    Encryptor enc2(*e.ctx, e.pk);
    enc2.encrypt(p, c2);
    std::size_t eq = 0;
    for (std::size_t k = 0; k < c1.dyn_array_size(); k++) eq += c1.data()[k] == c2.data()[k];
    CHECK(eq * 1000 < c1.dyn_array_size()); // fresh u, e0, e1: essentially every residue differs
    prng_seed_type a = UniformRandomGeneratorFactory::DefaultFactory()->next_seed();
    prng_seed_type b = UniformRandomGeneratorFactory::DefaultFactory()->next_seed();
    CHECK(a != b);
}

int main()
{
    struct T
    {
        const char *name;
        void (*fn)();
    } tests[] = { { "encoder_roundtrip", test_encoder_roundtrip },
                  { "encrypt_zero_and_decrypt", test_encrypt_zero_and_decrypt },
                  { "add_sub_negate", test_add_sub_negate },
                  { "multiply_relin_rescale", test_multiply_relin_rescale },
                  { "multiply_by_number_and_consts", test_multiply_by_number_and_consts },
                  { "mod_switch", test_mod_switch },
                  { "rotate", test_rotate },
                  { "reduced_error_ops", test_reduced_error_ops },
                  { "sparse_secret_and_slots", test_sparse_secret_and_slots },
                  { "security_level", test_security_level },
                  { "threads", test_threads },
                  { "fresh_seeds_differ", test_fresh_seeds_differ } };
    for (auto &t : tests)
    {
        const int before = g_fail;
        try
        {
            t.fn();
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
