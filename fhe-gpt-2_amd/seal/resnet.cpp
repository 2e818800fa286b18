// resnet.cpp -- encrypted ResNet CIFAR-10 inference (include/mhe_resnet.h), restating
// cnn_ckks/cpu-ckks/single-key/cnn/infer_seal.cpp over the seal:: surface.
#include "mhe_resnet.h"

#include "../../include/mhe.h"

#include <atomic>
#include <chrono>
#include <exception>
#include <mutex>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <random>
#include <stdexcept>

#include "../../include/mhe.h"

using namespace seal;

namespace
{
std::size_t end_num_of(std::size_t layer_num)
{
    // infer_seal.cpp:393-400
    switch (layer_num)
    {
    case 20: return 2;
    case 32: return 4;
    case 44: return 6;
    case 56: return 8;
    case 110: return 17;
    default: throw std::invalid_argument("layer_num is not correct");
    }
}

// conv / bn channel counts in import order (infer_seal.cpp:31-99)
void shapes(std::size_t layer_num, std::vector<std::size_t> &conv_sizes, std::vector<std::size_t> &bn_sizes)
{
    const std::size_t end_num = end_num_of(layer_num);
    conv_sizes = { 9 * 3 * 16 };
    for (int j = 1; j <= 3; j++)
        for (std::size_t k = 0; k <= end_num; k++)
        {
            const int co = j == 1 ? 16 : j == 2 ? 32 : 64;
            int ci;
            if (j == 1 || (j == 2 && k == 0))
                ci = 16;
            else if ((j == 2 && k != 0) || (j == 3 && k == 0))
                ci = 32;
            else
                ci = 64;
            conv_sizes.push_back((std::size_t)9 * ci * co);
            conv_sizes.push_back((std::size_t)9 * co * co);
        }
    bn_sizes = { 16 };
    for (int j = 1; j <= 3; j++)
        for (std::size_t k = 0; k <= end_num; k++)
        {
            const std::size_t ci = j == 1 ? 16 : j == 2 ? 32 : 64;
            bn_sizes.push_back(ci);
            bn_sizes.push_back(ci);
        }
}

void read_text(const std::string &path, std::size_t count, std::vector<double> &out)
{
    std::ifstream in(path);
    if (!in.is_open()) throw std::runtime_error("file is not open");
    double v;
    for (std::size_t i = 0; i < count; i++)
    {
        in >> v;
        out.emplace_back(v);
    }
}
} // namespace

void import_parameters_cifar10(std::vector<double> &linear_weight, std::vector<double> &linear_bias,
                               std::vector<std::vector<double>> &conv_weight, std::vector<std::vector<double>> &bn_bias,
                               std::vector<std::vector<double>> &bn_running_mean,
                               std::vector<std::vector<double>> &bn_running_var,
                               std::vector<std::vector<double>> &bn_weight, std::size_t layer_num, std::size_t end_num,
                               const std::string &root)
{
    // infer_seal.cpp:3-100
    if (layer_num != 20 && layer_num != 32 && layer_num != 44 && layer_num != 56 && layer_num != 110)
        throw std::invalid_argument("layer number is not valid");
    const std::string dir = root + "/resnet" + std::to_string(layer_num) + "_new/";
    std::vector<std::size_t> cs, bs;
    shapes(layer_num, cs, bs);
    (void)end_num;
    conv_weight.assign(layer_num - 1, {});
    bn_bias.assign(layer_num - 1, {});
    bn_running_mean.assign(layer_num - 1, {});
    bn_running_var.assign(layer_num - 1, {});
    bn_weight.assign(layer_num - 1, {});
    const std::size_t E = end_num_of(layer_num);
    std::size_t c = 0;
    read_text(dir + "conv1_weight.txt", cs[c], conv_weight[c]);
    c++;
    for (int j = 1; j <= 3; j++)
        for (std::size_t k = 0; k <= E; k++)
            for (int i = 1; i <= 2; i++, c++)
                read_text(dir + "layer" + std::to_string(j) + "_" + std::to_string(k) + "_conv" + std::to_string(i) +
                              "_weight.txt",
                          cs[c], conv_weight[c]);
    std::size_t b = 0;
    auto bn = [&](const std::string &prefix) {
        read_text(dir + prefix + "_bias.txt", bs[b], bn_bias[b]);
        read_text(dir + prefix + "_running_mean.txt", bs[b], bn_running_mean[b]);
        read_text(dir + prefix + "_running_var.txt", bs[b], bn_running_var[b]);
        read_text(dir + prefix + "_weight.txt", bs[b], bn_weight[b]);
        b++;
    };
    bn("bn1");
    for (int j = 1; j <= 3; j++)
        for (std::size_t k = 0; k <= E; k++)
            for (int i = 1; i <= 2; i++)
                bn("layer" + std::to_string(j) + "_" + std::to_string(k) + "_bn" + std::to_string(i));
    read_text(dir + "linear_weight.txt", 10 * 64, linear_weight);
    read_text(dir + "linear_bias.txt", 10, linear_bias);
}

ResNetParams load_resnet_params_bin(const std::string &path, std::size_t layer_num)
{
    std::vector<std::size_t> cs, bs;
    shapes(layer_num, cs, bs);
    std::ifstream in(path, std::ios::binary);
    if (!in.is_open()) throw std::runtime_error("parameter file is not open: " + path);
    // ".d7": 4-byte words sign | (exp + 64) << 24 | 7-digit mantissa, the reference's "%e" text
    // losslessly (tests/golden/make_resnet_params.py); the decimal is re-formed and parsed with
    // strtod, as the reference's `>>` parses its text
    const bool d7 = path.size() > 3 && path.compare(path.size() - 3, 3, ".d7") == 0;
    auto take = [&](std::size_t count) {
        std::vector<double> v(count);
        if (d7)
        {
            std::vector<std::uint32_t> w(count);
            in.read(reinterpret_cast<char *>(w.data()), (std::streamsize)(count * sizeof(std::uint32_t)));
            if (!in) throw std::runtime_error("parameter file is truncated: " + path);
            char buf[32];
            for (std::size_t i = 0; i < count; i++)
            {
                std::snprintf(buf, sizeof buf, "%s%ue%d", (w[i] >> 31) ? "-" : "", w[i] & 0xFFFFFFu,
                              (int)((w[i] >> 24) & 0x7F) - 64 - 6);
                v[i] = std::strtod(buf, nullptr);
            }
            return v;
        }
        in.read(reinterpret_cast<char *>(v.data()), (std::streamsize)(count * sizeof(double)));
        if (!in) throw std::runtime_error("parameter file is truncated: " + path);
        return v;
    };
    ResNetParams p;
    for (std::size_t c : cs) p.conv_weight.push_back(take(c));
    for (std::size_t b : bs)
    {
        p.bn_bias.push_back(take(b));
        p.bn_running_mean.push_back(take(b));
        p.bn_running_var.push_back(take(b));
        p.bn_weight.push_back(take(b));
    }
    p.linear_weight = take(10 * 64);
    p.linear_bias = take(10);
    return p;
}

// ------------------------------------------------------------------------------ plain network
namespace
{
std::vector<double> plain_conv(const std::vector<double> &in, const std::vector<double> &wt, int h, int ci, int co,
                               int st)
{
    // 3 x 3, zero padding 1, stride st; weights [co][ci][3][3] (the reference's import layout)
    const int ho = h / st;
    std::vector<double> out((std::size_t)co * ho * ho, 0.0);
    for (int b = 0; b < co; b++)
        for (int y = 0; y < ho; y++)
            for (int x = 0; x < ho; x++)
            {
                double s = 0;
                for (int a = 0; a < ci; a++)
                    for (int i1 = 0; i1 < 3; i1++)
                        for (int i2 = 0; i2 < 3; i2++)
                        {
                            const int yy = st * y + i1 - 1, xx = st * x + i2 - 1;
                            if (yy < 0 || yy >= h || xx < 0 || xx >= h) continue;
                            s += wt[((std::size_t)(b * ci + a) * 3 + i1) * 3 + i2] * in[(std::size_t)a * h * h + yy * h + xx];
                        }
                out[(std::size_t)b * ho * ho + y * ho + x] = s;
            }
    return out;
}

void plain_bn(std::vector<double> &v, const ResNetParams &p, int s, int c, int hw)
{
    for (int b = 0; b < c; b++)
    {
        const double g = p.bn_weight[s][b] / std::sqrt(p.bn_running_var[s][b] + 1e-5);
        for (int i = 0; i < hw; i++)
            v[(std::size_t)b * hw + i] = (v[(std::size_t)b * hw + i] - p.bn_running_mean[s][b]) * g + p.bn_bias[s][b];
    }
}

void plain_relu(std::vector<double> &v)
{
    for (auto &x : v) x = x > 0 ? x : 0.0;
}
} // namespace

std::vector<double> resnet_plain_logits(const ResNetParams &p, const std::vector<double> &img, std::size_t layer_num,
                                        const std::function<void(std::vector<double> &)> &relu)
{
    // the block structure of infer_seal.cpp:445-540 (conv, BN, ReLU; option-A shortcut with a
    // stride-2 subsample for the first block of stages 2 and 3), then average pooling and FC
    const int end_num = (int)end_num_of(layer_num);
    std::vector<double> x = plain_conv(img, p.conv_weight[0], 32, 3, 16, 1);
    int h = 32, c = 16;
    plain_bn(x, p, 0, c, h * h);
    relu(x);
    for (int j = 0; j < 3; j++)
        for (int k = 0; k <= end_num; k++)
        {
            const int s1 = 2 * ((end_num + 1) * j + k) + 1, s2 = s1 + 1;
            const int co = j == 0 ? 16 : j == 1 ? 32 : 64, st = (j >= 1 && k == 0) ? 2 : 1;
            std::vector<double> temp = x;
            std::vector<double> y = plain_conv(x, p.conv_weight[s1], h, c, co, st);
            const int ho = h / st;
            plain_bn(y, p, s1, co, ho * ho);
            relu(y);
            y = plain_conv(y, p.conv_weight[s2], ho, co, co, 1);
            plain_bn(y, p, s2, co, ho * ho);
            if (st == 2)
            {
                // input channel a -> output channel a + c/2, even pixels
                std::vector<double> ds((std::size_t)co * ho * ho, 0.0);
                for (int a = 0; a < c; a++)
                    for (int yy = 0; yy < ho; yy++)
                        for (int xx = 0; xx < ho; xx++)
                            ds[(std::size_t)(a + c / 2) * ho * ho + yy * ho + xx] = temp[(std::size_t)a * h * h + 2 * yy * h + 2 * xx];
                temp = ds;
            }
            for (std::size_t i = 0; i < y.size(); i++) y[i] += temp[i];
            relu(y);
            x = y;
            h = ho;
            c = co;
        }
    std::vector<double> f(64, 0.0), logits(10, 0.0);
    for (int b = 0; b < 64; b++)
    {
        for (int i = 0; i < h * h; i++) f[b] += x[(std::size_t)b * h * h + i];
        f[b] /= h * h;
    }
    for (int i = 0; i < 10; i++)
    {
        logits[i] = p.linear_bias[i];
        for (int b = 0; b < 64; b++) logits[i] += p.linear_weight[(std::size_t)i * 64 + b] * f[b];
    }
    return logits;
}

// ------------------------------------------------------------------------------------ runner
struct ResNetRunner::Impl
{
    std::size_t layer_num, end_num;
    ResNetParams prm;
    // infer_seal.cpp:236-310
    const double B = 40.0;
    const long alpha = 13, comp_no = 3;
    std::vector<int> deg{ 15, 15, 27 };
    const double scaled_val = 1.7;
    std::vector<Tree> tree;
    const long boundary_K = 25, boot_deg = 59, scale_factor = 2, inverse_deg = 1;
    const long logN = 16, loge = 10, logn = 15, logn_1 = 14, logn_2 = 13, logn_3 = 12;
    const int logp = 46, logq = 51, log_special_prime = 51;
    const int remaining_level = 16, boot_level = 14, total_level = remaining_level + boot_level;

    EncryptionParameters parms{ scheme_type::ckks };
    std::unique_ptr<SEALContext> context;
    std::unique_ptr<KeyGenerator> keygen;
    PublicKey public_key;
    SecretKey secret_key;
    RelinKeys relin_keys;
    GaloisKeys gal_keys;
    std::unique_ptr<CKKSEncoder> encoder;
    std::unique_ptr<Encryptor> encryptor;
    std::unique_ptr<Evaluator> evaluator;
    std::unique_ptr<Decryptor> decryptor;
    std::unique_ptr<Bootstrapper> boot[3];
};

ResNetRunner::ResNetRunner(std::size_t layer_num, const ResNetParams &params, const std::string &comp_dir,
                           KeySource keys, std::uint64_t rng_seed)
    : impl_(std::make_unique<Impl>())
{
    t0_ = std::chrono::steady_clock::now();
    Impl &m = *impl_;
    m.layer_num = layer_num;
    m.end_num = end_num_of(layer_num);
    m.prm = params;
    if (!comp_dir.empty()) setenv("MHE_COMP_DIR", comp_dir.c_str(), 1);
    for (int i = 0; i < m.comp_no; i++)
    {
        Tree tr;
        upgrade_oddbaby(m.deg[i], tr); // ev_type oddbaby (infer_seal.cpp:245-276)
        m.tree.emplace_back(tr);
    }
    std::vector<int> coeff_bit_vec{ m.logq };
    for (int i = 0; i < m.remaining_level; i++) coeff_bit_vec.push_back(m.logp);
    for (int i = 0; i < m.boot_level; i++) coeff_bit_vec.push_back(m.logq);
    coeff_bit_vec.push_back(m.log_special_prime);
    const std::size_t poly_modulus_degree = (std::size_t)1 << m.logN;
    m.parms.set_poly_modulus_degree(poly_modulus_degree);
    m.parms.set_coeff_modulus(CoeffModulus::Create(poly_modulus_degree, coeff_bit_vec));
    m.parms.set_secret_key_hamming_weight(192);
    std::shared_ptr<Blake2xbSeedSequence> seeds;
    if (rng_seed)
    {
        // reproducible keys, each from its own seed; frozen after setup (seal.h Blake2xbSeedSequence)
        prng_seed_type seed{};
        seed[0] = rng_seed;
        seeds = std::make_shared<Blake2xbSeedSequence>(seed);
        m.parms.set_random_generator(seeds);
    }
    m.context = std::make_unique<SEALContext>(m.parms);
    m.encoder = std::make_unique<CKKSEncoder>(*m.context);
    m.evaluator = std::make_unique<Evaluator>(*m.context, *m.encoder);
    if (keys == KeySource::generate)
    {
        m.keygen = std::make_unique<KeyGenerator>(*m.context);
        m.keygen->create_public_key(m.public_key);
        m.secret_key = m.keygen->secret_key();
        m.keygen->create_relin_keys(m.relin_keys);
        finish_setup(true);
    }
    if (seeds) seeds->freeze();
}

void ResNetRunner::finish_setup(bool plan_galois_keys)
{
    Impl &m = *impl_;
    if (!m.keygen) m.keygen = std::make_unique<KeyGenerator>(*m.context, m.secret_key);
    m.encryptor = std::make_unique<Encryptor>(*m.context, m.public_key);
    m.decryptor = std::make_unique<Decryptor>(*m.context, m.secret_key);
    const double scale = std::pow(2.0, m.logp);
    const long logns[3] = { m.logn_1, m.logn_2, m.logn_3 };
    for (int i = 0; i < 3; i++)
        m.boot[i] = std::make_unique<Bootstrapper>(m.loge, logns[i], m.logN - 1, m.total_level, scale, m.boundary_K,
                                                   m.boot_deg, m.scale_factor, m.inverse_deg, *m.context, *m.keygen,
                                                   *m.encoder, *m.encryptor, *m.decryptor, *m.evaluator, m.relin_keys,
                                                   m.gal_keys);
    for (auto &b : m.boot) b->prepare_mod_polynomial();
    for (int i = 0; i < 3; i++)
    {
        m.boot[i]->slot_vec.push_back(logns[i]);
        m.boot[i]->generate_LT_coefficient_3();
    }
    if (plan_galois_keys)
    {
        // Galois keys.  The reference's driver asks for its rotation steps at the key level
        // (infer_seal.cpp:345-379, 284 keys = 295 GB), more than one GPU holds.  Client side, a
        // deferred key provider over every step runs one planning inference on a zero image and
        // records the level each key is used at (the network's control flow does not depend on
        // the data); the server's set is then SEAL's keys truncated to those levels, made eagerly,
        // with no secret in them (seal.h KSwitchKeys).
        std::vector<int> gal_steps_vector{ 0 };
        for (long i = 1; i < (1L << (m.logN - 1)); i++) gal_steps_vector.push_back((int)i);
        m.keygen->create_deferred_galois_keys(gal_steps_vector, m.gal_keys);
        const auto t1 = std::chrono::steady_clock::now();
        (void)infer(std::vector<double>(3 * 32 * 32, 0.0));
        std::vector<std::pair<std::uint32_t, std::size_t>> plan;
        for (const auto &kv : m.gal_keys.usage()) plan.emplace_back((std::uint32_t)(2 * kv.first + 1), kv.second - 1);
        const auto t2 = std::chrono::steady_clock::now();
        {
            GaloisKeys eager;
            m.keygen->create_galois_keys(plan, eager);
            m.gal_keys = std::move(eager); // the deferred provider (and its secret key copy) goes away
        }
        mhe_stream_sync(m.context->engine(), m.context->stream());
        const auto t3 = std::chrono::steady_clock::now();
        plan_s_ = std::chrono::duration<double>(t2 - t1).count();
        keygen_s_ = std::chrono::duration<double>(t3 - t2).count();
    }
    galois_keys_ = m.gal_keys.usage().size();
    prepare_keys();
    // the planning inference's deferred keys and temporaries are freed by now; the allocator keeps
    // them cached at their sizes, which the steady state (ciphertexts, scratch) never reuses
    if (mhe_trim(m.context->engine()) != 0) throw std::runtime_error(mhe_last_error());
    setup_s_ = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0_).count();
}

// ---------------------------------------------------------------- key export / import
// kind 0 secret key [K][n], 1 public key [2][K][n], 2 relinearization key [K-1][2][K][n],
// 3 Galois key `index` truncated to `limbs` stored primes ([limbs-1][2][limbs][n])
std::vector<ResNetRunner::KeyBlob> ResNetRunner::export_keys() const
{
    const Impl &m = *impl_;
    void *s = m.context->stream();
    const std::size_t K = m.context->key_size();
    std::vector<KeyBlob> out;
    out.push_back({ 0, 0, K, m.secret_key.data().store().words(), m.secret_key.data().store().dev_read(s) });
    out.push_back({ 1, 0, K, m.public_key.data().store().words(), m.public_key.data().store().dev_read(s) });
    out.push_back({ 2, 0, K, m.relin_keys.key(0).words(), m.relin_keys.key(0).dev_read(s) });
    for (const auto &kv : m.gal_keys.usage())
        out.push_back({ 3, kv.first, kv.second, m.gal_keys.key(kv.first).words(), m.gal_keys.key(kv.first).dev_read(s) });
    mhe_stream_sync(m.context->engine(), s);
    return out;
}

void ResNetRunner::import_key(const KeyBlob &b)
{
    Impl &m = *impl_;
    SEALContext &ctx = *m.context;
    void *s = ctx.stream();
    const std::size_t K = ctx.key_size(), n = (std::size_t)1 << m.logN;
    auto copy_in = [&](PolyStore &ps, std::size_t words) {
        if (words != b.words) throw std::invalid_argument("imported key has the wrong size");
        ps.bind(ctx);
        ps.resize_words(words, false);
        if (mhe_memcpy_d2d(ctx.engine(), ps.dev_write(s, true), b.dev, words * 8, s) != MHE_OK)
            throw std::runtime_error(mhe_last_error());
    };
    switch (b.kind)
    {
    case 0:
        m.secret_key.data().set_level(ctx, ctx.key_parms_id(), K);
        copy_in(m.secret_key.data().store(), K * n);
        break;
    case 1:
        m.public_key.data().resize(ctx, ctx.key_parms_id(), 2);
        m.public_key.data().is_ntt_form() = true;
        m.public_key.data().scale() = 1.0;
        copy_in(m.public_key.data().store(), 2 * K * n);
        break;
    case 2:
    {
        PolyStore key;
        copy_in(key, (K - 1) * 2 * K * n);
        m.relin_keys.insert(RelinKeys::get_index(2), std::move(key), K);
        m.relin_keys.parms_id() = ctx.key_parms_id();
        m.relin_keys.set_key_limbs(K);
        break;
    }
    case 3:
    {
        if (b.limbs < 2 || b.limbs > K) throw std::invalid_argument("imported Galois key has invalid limbs");
        PolyStore key;
        copy_in(key, (b.limbs - 1) * 2 * b.limbs * n);
        m.gal_keys.insert(b.index, std::move(key), b.limbs);
        m.gal_keys.parms_id() = ctx.key_parms_id();
        m.gal_keys.set_key_limbs(K);
        break;
    }
    default: throw std::invalid_argument("unknown key kind");
    }
    mhe_stream_sync(ctx.engine(), s);
}

void ResNetRunner::copy_key(const KeyBlob &b, void *dst) const
{
    const Impl &m = *impl_;
    void *s = m.context->stream();
    if (mhe_memcpy_d2d(m.context->engine(), dst, b.dev, b.words * 8, s) != MHE_OK ||
        mhe_stream_sync(m.context->engine(), s) != MHE_OK)
        throw std::runtime_error(mhe_last_error());
    if (b.kind == 2 || b.kind == 3)
    {
        int prepared = 0;
        if (mhe_key_is_prepared(m.context->engine(), b.dev, (int)b.limbs, &prepared, s) != MHE_OK)
            throw std::runtime_error(mhe_last_error());
        if (prepared && mhe_key_unprepare(m.context->engine(), static_cast<std::uint64_t *>(dst), (int)b.limbs - 1,
                                          (int)b.limbs, s) != MHE_OK)
            throw std::runtime_error(mhe_last_error());
    }
}

void ResNetRunner::prepare_keys()
{
    // The server's evaluation keys in the engine's prepared format (mhe_key_prepare): the key MAC
    // streams 6 instead of 8 bytes per residue for the 46-bit primes; results are bit-identical.
    // MHE_KEY_PREPARE=0 keeps SEAL's layout.
    const char *e = getenv("MHE_KEY_PREPARE");
    if (e && atoi(e) == 0) return;
    Impl &m = *impl_;
    mhe_ctx *eng = m.context->engine();
    void *s = m.context->stream();
    auto prep = [&](PolyStore &ps, std::size_t limbs) {
        int prepared = 0;
        std::uint64_t *p = ps.dev_write(s);
        if (mhe_key_is_prepared(eng, p, (int)limbs, &prepared, s) != MHE_OK) throw std::runtime_error(mhe_last_error());
        if (!prepared && mhe_key_prepare(eng, p, (int)limbs - 1, (int)limbs, s) != MHE_OK)
            throw std::runtime_error(mhe_last_error());
    };
    if (m.relin_keys.has_index(0)) prep(m.relin_keys.key_mut(0), m.relin_keys.limbs_of(0));
    for (const auto &kv : m.gal_keys.usage()) prep(m.gal_keys.key_mut(kv.first), kv.second);
    mhe_stream_sync(eng, s);
    keys_prepared_ = true;
}

void ResNetRunner::finish_import()
{
    finish_setup(false);
}

ResNetRunner::~ResNetRunner() = default;

double ResNetRunner::galois_key_gb() const
{
    return impl_->gal_keys.device_bytes() / 1e9;
}

double ResNetRunner::key_traffic_bytes(bool reset)
{
    std::uint64_t b = 0;
    // SURVEY 8(d)'s algorithmic figure: every slice counted in SEAL's u64 layout, prepared or not
    // (a prepared key streams 6 of those 8 bytes for the 46-bit primes: mhe_key_traffic_prepared)
    std::uint64_t other = 0;
    mhe_ctx *eng = impl_->context->engine();
    const int rc = mhe_key_traffic(eng, &b, reset ? 1 : 0) | mhe_key_traffic_prepared(eng, &other, reset ? 1 : 0);
    if (rc != 0) throw std::runtime_error(mhe_last_error());
    return (double)b;
}

void ResNetRunner::set_hoist(bool on, bool check)
{
    if (mhe_ctx_set_hoist(impl_->context->engine(), on ? 1 : 0, check ? 1 : 0) != 0)
        throw std::runtime_error(mhe_last_error());
}

std::vector<std::uint64_t> ResNetRunner::hoist_stats(bool reset)
{
    std::vector<std::uint64_t> v(3, 0);
    if (mhe_hoist_stats(impl_->context->engine(), &v[0], &v[1], &v[2], reset ? 1 : 0) != 0)
        throw std::runtime_error(mhe_last_error());
    return v;
}

std::size_t ResNetRunner::scratch_bytes() const
{
    std::uint64_t w = 0, h = 0, m = 0;
    int st = 0;
    if (mhe_scratch_bytes(impl_->context->engine(), &w, &h, &m, &st) != 0) throw std::runtime_error(mhe_last_error());
    return (std::size_t)(w + h + m);
}

std::vector<std::uint64_t> ResNetRunner::op_counts(int kind, bool reset)
{
    std::vector<std::uint64_t> c(64, 0);
    if (mhe_op_counts(impl_->context->engine(), kind, c.data(), (int)c.size(), reset ? 1 : 0) != 0)
        throw std::runtime_error(mhe_last_error());
    return c;
}

std::vector<double> resnet_plain_logits(const ResNetParams &p, const std::vector<double> &img, std::size_t layer_num)
{
    return resnet_plain_logits(p, img, layer_num, plain_relu);
}

std::vector<double> ResNetRunner::plain_logits(const std::vector<double> &image) const
{
    return resnet_plain_logits(impl_->prm, image, impl_->layer_num, plain_relu);
}

std::vector<double> ResNetRunner::plain_logits_approx(const std::vector<double> &image) const
{
    const Impl &m = *impl_;
    const MinimaxReluPlain r(m.comp_no, m.deg, m.alpha, m.tree, m.scaled_val);
    const double B = m.B; // the encrypted network runs on x / B (infer_seal.cpp:444)
    return resnet_plain_logits(m.prm, image, m.layer_num, [&](std::vector<double> &v) {
        for (double &x : v) x = B * r(x / B);
    });
}

ResNetResult ResNetRunner::infer(const std::vector<double> &img)
{
    return infer(img, nullptr);
}

ResNetResult ResNetRunner::infer(const std::vector<double> &img, std::ostream *log)
{
    return infer(img, log, true);
}

ResNetResult ResNetRunner::infer(const std::vector<double> &img, std::ostream *log, bool stage_syncs)
{
    // infer_seal.cpp:404-577 (one image).  With `log`, every stage is written as the reference's
    // *_print wrappers write it to result/resnet{L}_cifar10_image{id}.txt (cnn_seal.cpp:106-123,
    // infer_seal.cpp:408-577): "<op>...", "time : <ms> ms", "remaining level : <chain index>",
    // "scale: <scale>", then a blank line; ReLU outputs are followed by a few decrypted values.
    Impl &m = *impl_;
    Evaluator &evaluator = *m.evaluator;
    CKKSEncoder &encoder = *m.encoder;
    Encryptor &encryptor = *m.encryptor;
    Decryptor &decryptor = *m.decryptor;
    ResNetResult res;
    using clk = std::chrono::steady_clock;
    auto sync = [&] { mhe_stream_sync(m.context->engine(), m.context->stream()); };
    auto stage_sync = [&] {
        if (stage_syncs || log) sync();
    };
    std::vector<Ciphertext> cipher_pool(14);
    TensorCipher cnn, temp;
    int co = 0, st = 0;
    const int fh = 3, fw = 3;
    const long init_p = 8, n = 1L << m.logn;
    int stage = 0;
    const double epsilon = 0.00001;
    const auto &prm = m.prm;
    auto t_op = clk::now();
    auto op_begin = [&] {
        if (!log) return;
        sync();
        t_op = clk::now();
    };
    auto op_end = [&](const char *what, const Ciphertext &c, bool timed = true, const char *extra = nullptr) {
        if (!log) return;
        sync();
        *log << what << "..." << std::endl;
        if (timed)
            *log << "time : " << (long)(std::chrono::duration<double>(clk::now() - t_op).count() * 1000) << " ms"
                 << std::endl;
        if (extra) *log << extra << std::endl;
        *log << "remaining level : " << m.context->get_context_data(c.parms_id())->chain_index() << std::endl;
        *log << "scale: " << c.scale() << std::endl << std::endl;
    };
    auto print_values = [&] {
        if (!log) return;
        // decrypt_and_print_part (func.cpp:262-333): four leading slots and the last
        Plaintext pt;
        decryptor.decrypt(cnn.cipher(), pt);
        std::vector<std::complex<double>> v;
        encoder.decode(pt, v);
        *log << "intermediate decrypted values: " << std::endl << "( ";
        for (int i = 0; i < 4; i++) *log << v[i] << ", ";
        *log << "... " << v.back() << ")" << std::endl << std::endl;
    };

    std::vector<double> image(n, 0.0);
    for (long i = 0; i < 32 * 32 * 3 && i < (long)img.size(); i++) image[i] = img[i];
    for (long i = n / init_p; i < n; i++) image[i] = image[i % (n / init_p)];
    for (long i = 0; i < n; i++) image[i] /= m.B; // for boundary [-1,1]

    cnn = TensorCipher((int)m.logn, 1, 32, 32, 3, 3, (int)init_p, image, encryptor, encoder, m.logq);
    stage_sync();
    const auto total_start = clk::now();
    double t_boot = 0, t_relu = 0;

    Ciphertext ctxt = cnn.cipher();
    for (int i = 0; i < m.boot_level - 3; i++) evaluator.mod_switch_to_next_inplace(ctxt);
    cnn.set_ciphertext(std::move(ctxt));

    // layer 0
    if (log) *log << "layer 0" << std::endl;
    op_begin();
    multiplexed_parallel_convolution_seal(cnn, cnn, 16, 1, fh, fw, prm.conv_weight[stage], prm.bn_running_var[stage],
                                          prm.bn_weight[stage], epsilon, encoder, encryptor, evaluator, m.gal_keys,
                                          cipher_pool);
    op_end("multiplexed parallel convolution", cnn.cipher());
    // scaling factor ~2^51 -> 2^46
    op_begin();
    {
        const auto &modulus = m.context->first_context_data()->parms().coeff_modulus();
        ctxt = cnn.cipher();
        const std::size_t cur_level = ctxt.coeff_modulus_size();
        Plaintext scaler;
        const double scale_change = std::pow(2.0, 46) * ((double)modulus[cur_level - 1].value()) / ctxt.scale();
        encoder.encode(1, scale_change, scaler);
        evaluator.mod_switch_to_inplace(scaler, ctxt.parms_id());
        evaluator.multiply_plain_inplace(ctxt, scaler);
        evaluator.rescale_to_next_inplace(ctxt);
        ctxt.scale() = std::pow(2.0, 46);
        cnn.set_ciphertext(std::move(ctxt));
    }
    multiplexed_parallel_batch_norm_seal(cnn, cnn, prm.bn_bias[stage], prm.bn_running_mean[stage],
                                         prm.bn_running_var[stage], prm.bn_weight[stage], epsilon, encoder, encryptor,
                                         evaluator, m.B);
    op_end("multiplexed parallel batch normalization", cnn.cipher());
    auto relu = [&] {
        stage_sync();
        const auto a = clk::now();
        op_begin();
        ReLU_seal(cnn, cnn, m.comp_no, m.deg, m.alpha, m.tree, m.scaled_val, m.logp, encryptor, evaluator, decryptor,
                  encoder, m.public_key, m.secret_key, m.relin_keys, m.B);
        stage_sync();
        t_relu += std::chrono::duration<double>(clk::now() - a).count();
        op_end("approximate ReLU", cnn.cipher());
        print_values();
    };
    auto bootstrap = [&](int j) {
        stage_sync();
        const auto a = clk::now();
        op_begin();
        Ciphertext c = cnn.cipher(), rtn;
        {
            seal::Lockstep::Active merge; // MHE_RESNET_LOCKSTEP=2 (a no-op outside a group)
            m.boot[j]->bootstrap_real_3(rtn, c);
        }
        cnn.set_ciphertext(std::move(rtn));
        stage_sync();
        t_boot += std::chrono::duration<double>(clk::now() - a).count();
        res.bootstraps++;
        const std::string tag = "bootstrapping " + std::to_string(res.bootstraps) + " result";
        op_end("bootstrapping", cnn.cipher(), true, tag.c_str());
    };
    relu();

    int layer = 1;
    for (int j = 0; j < 3; j++) // layer 1_x, 2_x, 3_x
    {
        co = j == 0 ? 16 : j == 1 ? 32 : 64;
        for (std::size_t k = 0; k <= m.end_num; k++)
        {
            stage = (int)(2 * ((m.end_num + 1) * j + k) + 1);
            if (log) *log << "layer " << layer++ << std::endl;
            temp = cnn;
            st = (j >= 1 && k == 0) ? 2 : 1;
            op_begin();
            multiplexed_parallel_convolution_seal(cnn, cnn, co, st, fh, fw, prm.conv_weight[stage],
                                                  prm.bn_running_var[stage], prm.bn_weight[stage], epsilon, encoder,
                                                  encryptor, evaluator, m.gal_keys, cipher_pool);
            op_end("multiplexed parallel convolution", cnn.cipher());
            op_begin();
            multiplexed_parallel_batch_norm_seal(cnn, cnn, prm.bn_bias[stage], prm.bn_running_mean[stage],
                                                 prm.bn_running_var[stage], prm.bn_weight[stage], epsilon, encoder,
                                                 encryptor, evaluator, m.B);
            op_end("multiplexed parallel batch normalization", cnn.cipher());
            bootstrap(j);
            relu();

            stage = (int)(2 * ((m.end_num + 1) * j + k) + 2);
            if (log) *log << "layer " << layer++ << std::endl;
            st = 1;
            op_begin();
            multiplexed_parallel_convolution_seal(cnn, cnn, co, st, fh, fw, prm.conv_weight[stage],
                                                  prm.bn_running_var[stage], prm.bn_weight[stage], epsilon, encoder,
                                                  encryptor, evaluator, m.gal_keys, cipher_pool);
            op_end("multiplexed parallel convolution", cnn.cipher());
            op_begin();
            multiplexed_parallel_batch_norm_seal(cnn, cnn, prm.bn_bias[stage], prm.bn_running_mean[stage],
                                                 prm.bn_running_var[stage], prm.bn_weight[stage], epsilon, encoder,
                                                 encryptor, evaluator, m.B);
            op_end("multiplexed parallel batch normalization", cnn.cipher());
            if (j >= 1 && k == 0)
            {
                op_begin();
                multiplexed_parallel_downsampling_seal(temp, temp, evaluator, m.gal_keys);
                op_end("multiplexed parallel downsampling", temp.cipher());
            }
            cnn_add_seal(temp, cnn, cnn, evaluator);
            op_end("cipher add", cnn.cipher(), false);
            bootstrap(j);
            relu();
        }
    }
    if (log) *log << "layer " << layer << std::endl;
    std::ofstream devnull;
    op_begin();
    averagepooling_seal_scale(cnn, cnn, evaluator, m.gal_keys, m.B, encoder, decryptor, devnull);
    op_end("average pooling", cnn.cipher());
    op_begin();
    matrix_multiplication_seal(cnn, cnn, prm.linear_weight, prm.linear_bias, 10, 64, evaluator, m.gal_keys);
    op_end("fully connected layer", cnn.cipher());
    sync();
    res.seconds = std::chrono::duration<double>(clk::now() - total_start).count();
    res.boot_seconds = t_boot;
    res.relu_seconds = t_relu;
    res.linear_seconds = res.seconds - t_boot - t_relu;

    {
        // FNV-1a over the output ciphertext's words, its size, level and scale bits
        const Ciphertext &out = cnn.cipher();
        std::uint64_t h = 0xcbf29ce484222325ull;
        auto mix = [&](std::uint64_t v) {
            for (int b = 0; b < 8; b++)
            {
                h ^= (v >> (8 * b)) & 0xff;
                h *= 0x100000001b3ull;
            }
        };
        const std::uint64_t *w = out.store().host();
        for (std::size_t i = 0; i < out.store().words(); i++) mix(w[i]);
        double sc = out.scale();
        std::uint64_t sb;
        std::memcpy(&sb, &sc, sizeof sb);
        mix(out.size());
        mix(out.coeff_modulus_size());
        mix(sb);
        res.digest = h;
    }
    Plaintext plain;
    decryptor.decrypt(cnn.cipher(), plain);
    std::vector<std::complex<double>> rtn_vec;
    encoder.decode(plain, rtn_vec);
    double max_score = -100.0;
    for (std::size_t i = 0; i < 10; i++)
    {
        res.logits.push_back(rtn_vec[i].real());
        res.slots.push_back(rtn_vec[i]);
        if (max_score < rtn_vec[i].real())
        {
            res.label = i;
            max_score = rtn_vec[i].real();
        }
    }
    return res;
}

std::vector<ResNetResult> ResNetRunner::infer_batch(const std::vector<std::vector<double>> &images, int threads,
                                                    int fibers)
{
    std::vector<ResNetResult> out(images.size());
    std::atomic<std::size_t> next{ 0 };
    std::exception_ptr err;
    std::mutex err_mu;
    // MHE_RESNET_LOCKSTEP=1: the images in flight run their key switches and rescales as one
    // batched launch per operation (seal::Lockstep); 2: only inside bootstrapping, where the
    // rotations run at high levels with one key per step shared by all images
    static const int lockstep = [] {
        const char *e = std::getenv("MHE_RESNET_LOCKSTEP");
        return e ? std::atoi(e) : 0;
    }();
    if (fibers <= 0)
    {
        const char *e = std::getenv("MHE_RESNET_FIBERS");
        fibers = e ? std::max(1, std::atoi(e)) : 1;
    }
    const int nthreads = std::max(1, threads);
    std::unique_ptr<seal::Lockstep> group;
    if (lockstep && nthreads > 1 && fibers <= 1) group = std::make_unique<seal::Lockstep>((std::size_t)nthreads);
    std::atomic<std::size_t> fb_rounds{ 0 }, fb_merged{ 0 };
    auto work = [&] {
        std::unique_ptr<seal::Lockstep::Member> member;
        if (group) member = std::make_unique<seal::Lockstep::Member>(*group, lockstep == 1);
        try
        {
            if (fibers > 1)
            {
                // `fibers` images at a time on this thread as one FiberBatch
                for (;;)
                {
                    const std::size_t i0 = next.fetch_add((std::size_t)fibers);
                    if (i0 >= images.size()) break;
                    const std::size_t cnt = std::min<std::size_t>((std::size_t)fibers, images.size() - i0);
                    seal::FiberBatch::run(cnt, [&](std::size_t k) { out[i0 + k] = infer(images[i0 + k], nullptr, false); });
                    fb_rounds += seal::FiberBatch::last_rounds();
                    fb_merged += seal::FiberBatch::last_merged();
                }
            }
            else
                for (std::size_t i; (i = next.fetch_add(1)) < images.size();) out[i] = infer(images[i]);
        }
        catch (...)
        {
            std::lock_guard<std::mutex> g(err_mu);
            if (!err) err = std::current_exception();
        }
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < nthreads; t++) pool.emplace_back(work);
    for (auto &t : pool) t.join();
    if (group && std::getenv("MHE_RESNET_LOCKSTEP_STATS"))
        std::fprintf(stderr, "lockstep: %zu rounds, %zu member calls merged\n", group->rounds(), group->merged_calls());
    if (fibers > 1 && std::getenv("MHE_RESNET_LOCKSTEP_STATS"))
        std::fprintf(stderr, "fibers: %d per thread, %zu rounds, %zu member calls merged\n", fibers, fb_rounds.load(),
                     fb_merged.load());
    if (err) std::rethrow_exception(err);
    return out;
}

void ResNet_cifar10_seal_sparse(std::size_t layer_num, std::size_t start_image_id, std::size_t end_image_id)
{
    // infer_seal.cpp:234-582: parameters, the shared label file ../../result/resnet{L}_cifar10_label_{s}_{e}
    // and per image ../../result/resnet{L}_cifar10_image{id}.txt with the per-stage log
    if (layer_num != 20 && layer_num != 32 && layer_num != 44 && layer_num != 56 && layer_num != 110)
        throw std::invalid_argument("layer_num is not correct");
    ResNetParams prm;
    if (const char *bin = std::getenv("MHE_RESNET_PARAMS"))
        prm = load_resnet_params_bin(bin, layer_num);
    else
        import_parameters_cifar10(prm.linear_weight, prm.linear_bias, prm.conv_weight, prm.bn_bias,
                                  prm.bn_running_mean, prm.bn_running_var, prm.bn_weight, layer_num,
                                  end_num_of(layer_num));
    const std::string net = "resnet" + std::to_string(layer_num) + "_cifar10_";
    std::ofstream out_share("../../result/" + net + "label_" + std::to_string(start_image_id) + "_" +
                            std::to_string(end_image_id));
    const char *cd = std::getenv("MHE_COMP_DIR");
    ResNetRunner runner(layer_num, prm, cd ? cd : "../../result");
    std::ifstream values("../../../testFile/test_values.txt"), labels("../../../testFile/test_label.txt");
    const bool have_images = values.is_open();
    const auto all_start = std::chrono::steady_clock::now();
    for (std::size_t image_id = start_image_id; image_id <= end_image_id; image_id++)
    {
        std::vector<double> img(32 * 32 * 3);
        int image_label = -1;
        if (have_images)
        {
            double v;
            values.clear();
            values.seekg(0);
            for (std::size_t i = 0; i < 32 * 32 * 3 * image_id; i++) values >> v;
            for (auto &x : img) values >> x;
            labels.clear();
            labels.seekg(0);
            for (std::size_t i = 0; i <= image_id; i++) labels >> image_label;
        }
        else
        {
            // test_values.txt is not in the reference tree: seeded synthetic pixels
            std::mt19937_64 g(image_id);
            std::uniform_real_distribution<double> U(-2.5, 2.5);
            for (auto &x : img) x = U(g);
        }
        std::ofstream output("../../result/" + net + "image" + std::to_string(image_id) + ".txt");
        ResNetResult r = runner.infer(img, &output);
        for (std::ostream *o : { (std::ostream *)&std::cout, (std::ostream *)&output })
        {
            *o << "( ";
            for (std::size_t i = 0; i < 9; i++) *o << r.slots[i] << ", ";
            *o << r.slots[9] << ")" << std::endl;
            *o << "total time : " << (long)(r.seconds * 1000) << " ms" << std::endl;
            *o << "image label: " << image_label << std::endl;
            *o << "inferred label: " << r.label << std::endl;
            *o << "max score: " << r.logits[r.label] << std::endl;
        }
        out_share << "image_id: " << image_id << ", "
                  << "image label: " << image_label << ", inferred label: " << r.label << std::endl;
    }
    const long all_ms = (long)(std::chrono::duration<double>(std::chrono::steady_clock::now() - all_start).count() * 1000);
    std::cout << "all threads time : " << all_ms << " ms" << std::endl;
    out_share << std::endl << "all threads time : " << all_ms << " ms" << std::endl;
}
