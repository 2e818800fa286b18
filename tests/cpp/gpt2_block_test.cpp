// GPU test of the GPT-2 block (fhe-gpt-2_amd/seal/gpt2_block.cpp) against the committed plain
// restatement tests/golden/gpt2_block/{block.bin,block.txt} (made by make_fixture.py there): the
// packing helpers and KV-cache augmentation against their plain definitions, each block piece on
// encrypted fixture inputs, then the whole block (LN1 -> attention -> residual -> LN2 -> MLP ->
// residual) with real bootstrapping, every stage decrypted and compared.  Pass: every compared
// value within 1e-3.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <thread>
#include <fstream>
#include <map>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "mhe_boot.h"
#include "mhe_gpt2.h"

using namespace seal;
using namespace gpt2;

static int g_fail = 0;
static void report(const std::string &name, bool ok, double err, double secs)
{
    std::printf("[%s] %s  max err %.3g  (%.2f s)\n", ok ? "PASS" : "FAIL", name.c_str(), err, secs);
    if (!ok) g_fail++;
}

struct Mat
{
    int rows = 0, cols = 0;
    std::vector<double> v;
    double at(int r, int c) const { return v[(std::size_t)r * cols + c]; }
};

static std::map<std::string, Mat> load_fixture(const std::string &dir, const std::string &stem = "block")
{
    std::ifstream txt(dir + "/" + stem + ".txt"), bin(dir + "/" + stem + ".bin", std::ios::binary);
    if (!txt || !bin) throw std::runtime_error("fixture not found under " + dir);
    std::vector<char> raw((std::istreambuf_iterator<char>(bin)), std::istreambuf_iterator<char>());
    std::map<std::string, Mat> out;
    std::string line;
    while (std::getline(txt, line))
    {
        if (line.empty() || line[0] == '#') continue;
        std::istringstream is(line);
        std::string name;
        long r, c, off;
        is >> name >> r >> c >> off;
        Mat m;
        m.rows = (int)r;
        m.cols = (int)c;
        m.v.resize((std::size_t)r * c);
        if ((std::size_t)(off + r * c) * 8 > raw.size()) throw std::runtime_error("fixture truncated at " + name);
        std::memcpy(m.v.data(), raw.data() + off * 8, m.v.size() * 8);
        out[name] = m;
    }
    return out;
}

static std::vector<double> vec(const Mat &m) { return m.v; }

// "key value" pairs of the fixture's header line (make_fixture.py header())
static std::map<std::string, double> fixture_header(const std::string &dir)
{
    std::ifstream txt(dir + "/block.txt");
    std::string line, tok;
    std::getline(txt, line);
    std::istringstream is(line);
    std::vector<std::string> w;
    while (is >> tok) w.push_back(tok);
    std::map<std::string, double> out;
    for (std::size_t i = 0; i + 1 < w.size(); i++)
    {
        char *end = nullptr;
        const double v = std::strtod(w[i + 1].c_str(), &end);
        if (end && *end == 0 && !w[i + 1].empty()) out[w[i]] = v;
    }
    return out;
}

int main(int argc, char **argv)
{
    std::setvbuf(stdout, nullptr, _IONBF, 0);
    // heartbeat: a line every 30 s so a long block run is never mistaken for a hang
    const auto t_start = std::chrono::steady_clock::now();
    std::atomic<bool> done{ false };
    std::thread beat([&] {
        int k = 0;
        while (!done.load())
        {
            std::this_thread::sleep_for(std::chrono::milliseconds(200));
            if (++k % 150 == 0)
                std::printf("  ... %.0f s\n",
                            std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count());
        }
    });
    struct Join
    {
        std::atomic<bool> &d;
        std::thread &t;
        ~Join()
        {
            d = true;
            t.join();
        }
    } join{ done, beat };
    const std::string dir = argc > 1 ? argv[1] : "tests/golden/gpt2_block";
    // "block": the whole block only (the GPT-2-width fixture, make_fixture.py --full)
    const bool block_only = argc > 2 && std::string(argv[2]) == "block";
    try
    {
        const auto fx = load_fixture(dir);
        const auto hdr = fixture_header(dir);
        const Mat &X = fx.at("x");
        const int T = X.rows, d = X.cols, F = fx.at("fc_w").cols, H = hdr.count("heads") ? (int)hdr.at("heads") : 4,
                  dh = d / H;
        const double kTol = 1e-3;

        // INIT() of gpt2/util.h:36-74: {49} + 21 x {46} + 14 x {49} + {60}, h = 192, scale 2^46
        const long logN = 16;
        const int remaining_level = 21, boot_level = BOOT_LEVEL;
        std::vector<int> bits{ LOGQ };
        for (int i = 0; i < remaining_level; i++) bits.push_back(LOGP);
        for (int i = 0; i < boot_level; i++) bits.push_back(LOGQ);
        bits.push_back(60);
        EncryptionParameters params(scheme_type::ckks);
        params.set_poly_modulus_degree((std::size_t)1 << logN);
        params.set_coeff_modulus(CoeffModulus::Create((std::size_t)1 << logN, bits));
        params.set_secret_key_hamming_weight(192);
        const auto t0 = std::chrono::steady_clock::now();
        SEALContext context(params);
        KeyGenerator keygen(context);
        PublicKey pk;
        RelinKeys rk;
        GaloisKeys gk;
        keygen.create_public_key(pk);
        keygen.create_relin_keys(rk);
        const double scale = std::pow(2.0, LOGP);
        set_encode_scale(scale);
        set_bootstrap_prescale(8.0);
        CKKSEncoder encoder(context);
        Encryptor encryptor(context, pk);
        Evaluator evaluator(context, encoder);
        Decryptor decryptor(context, keygen.secret_key());
        Bootstrapper bt(10, logN - 1, logN - 1, remaining_level + boot_level, scale, 25, 59, 2, 1, context, keygen,
                        encoder, encryptor, decryptor, evaluator, rk, gk);
        std::vector<int> steps = block_rotation_steps((int)logN);
        init_bootstrap(bt, steps, (int)logN - 1);
        keygen.create_galois_keys(steps, gk);
        std::printf("setup: %zu Galois keys, %.1f s\n", steps.size(),
                    std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());

        const int S = 32768;
        const int Rd = round_to_2(d), Sd = 2 * Rd;
        auto enc_slots = [&](const std::vector<double> &v) {
            Plaintext p;
            Ciphertext c;
            encoder.encode(v, scale, p);
            encryptor.encrypt(p, c);
            while ((int)c.coeff_modulus_size() > remaining_level + 1) evaluator.mod_switch_to_next_inplace(c);
            return c;
        };
        auto dec_slots = [&](const Ciphertext &c) {
            Plaintext p;
            std::vector<double> v;
            decryptor.decrypt(c, p);
            encoder.decode(p, v);
            return v;
        };
        // row-packed (rows x cols) <-> ciphertexts
        auto enc_rows = [&](const Mat &m) {
            const int st = 2 * round_to_2(m.cols), c = S / st;
            std::vector<Ciphertext> out;
            for (int i0 = 0; i0 < m.rows; i0 += c)
            {
                std::vector<double> v(S, 0.0);
                for (int r = i0; r < std::min(m.rows, i0 + c); r++)
                    for (int j = 0; j < m.cols; j++) v[(std::size_t)(r - i0) * st + j] = m.at(r, j);
                out.push_back(enc_slots(v));
            }
            return out;
        };
        auto err_rows = [&](const std::vector<Ciphertext> &cts, const Mat &want) {
            const int st = 2 * round_to_2(want.cols), c = S / st;
            double e = 0;
            for (std::size_t i = 0; i < cts.size(); i++)
            {
                const auto v = dec_slots(cts[i]);
                for (int r = (int)i * c; r < std::min(want.rows, (int)(i + 1) * c); r++)
                    for (int j = 0; j < want.cols; j++) e = std::max(e, std::fabs(v[(std::size_t)(r % c) * st + j] - want.at(r, j)));
            }
            return e;
        };
        auto since = [](std::chrono::steady_clock::time_point t) {
            return std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
        };
        std::mt19937_64 rng(7);
        std::uniform_real_distribution<double> U(-1, 1);

        // ------------------------------------------------------------ packing helpers (pack.py)
        if (!block_only)
        {
            // pack_tight / unpack_tight with rows straddling the ciphertext boundary
            const int rows = 1400, rs = 24, st = 64, c = S / st;
            std::vector<std::vector<double>> M(rows, std::vector<double>(rs));
            for (auto &r : M)
                for (auto &x : r) x = U(rng);
            std::vector<Ciphertext> in;
            for (int i0 = 0; i0 < rows; i0 += c)
            {
                std::vector<double> v(S, 0.0);
                for (int r = i0; r < std::min(rows, i0 + c); r++)
                    for (int j = 0; j < rs; j++) v[(std::size_t)(r - i0) * st + j] = M[r][j];
                in.push_back(enc_slots(v));
            }
            auto t = std::chrono::steady_clock::now();
            std::vector<Ciphertext> tight, back;
            pack_tight(in, tight, rows, rs, st, encoder, encryptor, decryptor, evaluator, gk, rk);
            double e = 0;
            for (std::size_t k = 0; k < tight.size(); k++)
            {
                const auto v = dec_slots(tight[k]);
                for (int s = 0; s < S; s++)
                {
                    const long g = (long)k * S + s;
                    const double want = g < (long)rows * rs ? M[g / rs][g % rs] : 0.0;
                    e = std::max(e, std::fabs(v[s] - want));
                }
            }
            report("pack_tight 1400 rows of 24 at stride 64 (3 -> 2 ciphertexts, boundary rows split)",
                   e < kTol && tight.size() == 2, e, since(t));
            t = std::chrono::steady_clock::now();
            unpack_tight(tight, back, rows, rs, st, encoder, encryptor, decryptor, evaluator, gk, rk);
            e = 0;
            for (std::size_t k = 0; k < back.size(); k++)
            {
                const auto v = dec_slots(back[k]);
                for (int s = 0; s < S; s++)
                {
                    const int r = (int)k * c + s / st, j = s % st;
                    const double want = (r < rows && j < rs) ? M[r][j] : 0.0;
                    e = std::max(e, std::fabs(v[s] - want));
                }
            }
            report("unpack_tight restores the stride-64 layout", e < kTol && back.size() == in.size(), e, since(t));
        }
        if (!block_only)
        {
            // expand_bias / expand_bias_head_row / expand_bias_head_col (pack.py:78-113)
            auto t = std::chrono::steady_clock::now();
            std::vector<double> b(d);
            for (auto &x : b) x = U(rng);
            Ciphertext eb;
            expand_bias(b, eb, encoder, encryptor, decryptor, evaluator, gk, rk);
            std::vector<Ciphertext> hr, hc;
            expand_bias_head_row(b, hr, H, encoder, encryptor, decryptor, evaluator, gk, rk, T);
            expand_bias_head_col(b, hc, H, T, dh, encoder, encryptor, decryptor, evaluator, gk, rk);
            double e = 0;
            auto v = dec_slots(eb);
            for (int s = 0; s < S; s++) e = std::max(e, std::fabs(v[s] - ((s % Sd) < d ? b[s % Sd] : 0.0)));
            for (int h = 0; h < H; h++)
            {
                v = dec_slots(hr[h]);
                for (int s = 0; s < S; s++)
                {
                    const int r = s / (2 * dh), j = s % (2 * dh);
                    e = std::max(e, std::fabs(v[s] - (r < T && j < dh ? b[h * dh + j] : 0.0)));
                }
                v = dec_slots(hc[h]);
                for (int s = 0; s < S; s++)
                {
                    const int j = s / (2 * T), r = s % (2 * T);
                    e = std::max(e, std::fabs(v[s] - (j < dh && r < T ? b[h * dh + j] : 0.0)));
                }
            }
            report("expand_bias / expand_bias_head_row / expand_bias_head_col vs pack.py", e < kTol, e, since(t));
        }
        if (!block_only)
        {
            // KV cache (optimize.cpp:4-40): augment_value_row keeps row idx of A, the rest from the
            // cache; augment_value_col clears cache column idx and adds A rotated by idx
            auto t = std::chrono::steady_clock::now();
            const int prs = 32, idx = 3;
            std::vector<double> a(S), cache(S);
            for (int s = 0; s < S; s++)
            {
                a[s] = U(rng);
                cache[s] = U(rng);
            }
            std::vector<Ciphertext> A{ enc_slots(a) }, C{ enc_slots(cache) };
            augment_value_row(A, C, prs, idx, encoder, encryptor, decryptor, evaluator, gk, rk);
            double e = 0;
            auto v = dec_slots(A[0]);
            for (int s = 0; s < S; s++)
            {
                const bool in_row = s >= idx * prs && s < (idx + 1) * prs;
                e = std::max(e, std::fabs(v[s] - ((in_row ? 0.0 : a[s]) + cache[s])));
            }
            std::vector<Ciphertext> A2{ enc_slots(a) }, C2{ enc_slots(cache) };
            augment_value_col(A2, C2, prs, idx, encoder, encryptor, decryptor, evaluator, gk, rk);
            v = dec_slots(A2[0]);
            for (int s = 0; s < S; s++)
            {
                const bool cleared = (s % prs) == idx && s / prs < prs / 2;
                e = std::max(e, std::fabs(v[s] - (a[(s + idx) % S] + (cleared ? 0.0 : cache[s]))));
            }
            report("augment_value_row / augment_value_col (KV cache) vs plain", e < kTol, e, since(t));
        }

        // ------------------------------------------------------------ block pieces on fixture inputs
        std::vector<std::vector<double>> keep(T, std::vector<double>(T, 0.0));
        for (int r = 0; r < T; r++)
            for (int j = 0; j <= r; j++) keep[r][j] = 1.0;
        AttentionParams ap;
        if (hdr.count("inv_iters")) ap.inv_iters = (int)hdr.at("inv_iters");
        // a fixture made with make_fixture.py --gelu-ref: the block's GELU x piece as poly.py writes it
        if (hdr.count("gelu_ref") && hdr.at("gelu_ref") != 0) ap.gelu_last = GeluLastPiece::reference;
        BlockDims dims;
        dims.rows = T;
        dims.d_model = d;
        dims.heads = H;
        dims.d_ff = F;
        PlainBlockWeights pw;
        for (auto &kv : std::map<std::string, std::vector<double> *>{
                 { "ln1_g", &pw.ln1_g }, { "ln1_b", &pw.ln1_b }, { "qw", &pw.qw },     { "qb", &pw.qb },
                 { "kw", &pw.kw },       { "kb", &pw.kb },       { "vw", &pw.vw },     { "vb", &pw.vb },
                 { "ow", &pw.ow },       { "ob", &pw.ob },       { "ln2_g", &pw.ln2_g }, { "ln2_b", &pw.ln2_b },
                 { "fc_w", &pw.fc_w },   { "fc_b", &pw.fc_b },   { "pj_w", &pw.pj_w }, { "pj_b", &pw.pj_b } })
            *kv.second = vec(fx.at(kv.first));
        BlockWeights bw;
        {
            auto t = std::chrono::steady_clock::now();
            encrypt_block_weights(pw, bw, dims, encoder, encryptor, decryptor, evaluator, gk, rk, remaining_level + 1);
            std::printf("block weights encrypted and packed: %.2f s\n", since(t));
        }
        if (!block_only)
        {
            auto t = std::chrono::steady_clock::now();
            auto xin = enc_rows(X);
            Ciphertext out;
            layer_norm_rows(xin[0], out, pw.ln1_g, pw.ln1_b, T, d, ap.newton_iters, bt, encoder, encryptor, decryptor,
                            evaluator, gk, rk);
            const double e = err_rows({ out }, fx.at("ln1"));
            std::printf("   layer_norm_rows: %zu limbs out\n", out.coeff_modulus_size());
            report("layer_norm_rows(x) vs restated LN1", e < kTol, e, since(t));
        }
        if (!block_only)
        {
            auto t = std::chrono::steady_clock::now();
            auto a = enc_rows(fx.at("ln1"));
            std::vector<Ciphertext> Q, V;
            attn_proj_heads(a, bw.qw, bw.qb, Q, T, d, H, false, encoder, encryptor, decryptor, evaluator, gk, rk);
            attn_proj_heads(a, bw.vw, bw.vb, V, T, d, H, true, encoder, encryptor, decryptor, evaluator, gk, rk);
            const Mat &q = fx.at("q"), &vv = fx.at("v");
            double e = 0;
            for (int h = 0; h < H; h++)
            {
                const auto qs = dec_slots(Q[h]), vs = dec_slots(V[h]);
                for (int s = 0; s < S; s++)
                {
                    const int r = s / (2 * dh), j = s % (2 * dh);
                    e = std::max(e, std::fabs(qs[s] - (r < T && j < dh ? q.at(r, h * dh + j) : 0.0)));
                    const int jc = s / (2 * T), rc = s % (2 * T);
                    e = std::max(e, std::fabs(vs[s] - (jc < dh && rc < T ? vv.at(rc, h * dh + jc) : 0.0)));
                }
            }
            report("attn_proj_heads: Q (row head layout) and V (column head layout), all slots", e < kTol, e, since(t));
        }
        if (!block_only)
        {
            auto t = std::chrono::steady_clock::now();
            auto hin = enc_rows(fx.at("hidden"));
            Ciphertext g;
            compute_gelu_block(hin[0], g, ap.gelu_alpha, encoder, encryptor, decryptor, evaluator, gk, rk);
            const double e = err_rows({ g }, fx.at("gelu"));
            std::printf("   compute_gelu_block: %zu limbs out\n", g.coeff_modulus_size());
            report("compute_gelu_block(hidden) vs restated GELU", e < kTol, e, since(t));
        }
        if (!block_only && std::ifstream(dir + "/gelu_ref.txt"))
        {
            // the GELU piece against the reference's own plain formula: plain_approx/poly.py:30-35
            // restated in numpy (make_gelu_ref.py, np.sign, b3 = 0.5 s2) vs compute_gelu_block with
            // GeluLastPiece::reference; and the block's default (indicator s2 + 1/2, a departure)
            // vs its restatement, on the same 4096 inputs >= 0.5 from each breakpoint
            const auto gx = load_fixture(dir, "gelu_ref");
            const Mat &gxin = gx.at("x"), &gref = gx.at("poly_gelu"), &gblk = gx.at("gelu_block");
            std::vector<double> v(S, 0.0);
            for (int i = 0; i < gxin.cols; i++) v[i] = gxin.v[i];
            for (int variant = 0; variant < 2; variant++)
            {
                auto t = std::chrono::steady_clock::now();
                Ciphertext in = enc_slots(v), g;
                const bool ref = variant == 0;
                compute_gelu_block(in, g, ap.gelu_alpha, encoder, encryptor, decryptor, evaluator, gk, rk,
                                   ref ? GeluLastPiece::reference : GeluLastPiece::indicator);
                const auto got = dec_slots(g);
                double e = 0;
                for (int i = 0; i < gxin.cols; i++) e = std::max(e, std::fabs(got[i] - (ref ? gref : gblk).v[i]));
                report(ref ? "compute_gelu_block(GeluLastPiece::reference) vs plain_approx/poly.py gelu (b3 = 0.5 s2), "
                             "4096 inputs"
                           : "compute_gelu_block (block default: indicator s2 + 1/2, departure from poly.py's 0.5 s2) "
                             "vs its restatement",
                       e < kTol, e, since(t));
            }
        }
        if (!block_only)
        {
            auto t = std::chrono::steady_clock::now();
            auto a = enc_rows(fx.at("ln2"));
            // the row-packed FC1 bias of the reference layout (the block itself holds the hidden
            // state in d-wide chunks with one bias ciphertext each)
            std::vector<double> fb = pw.fc_b;
            Ciphertext fcb;
            expand_bias(fb, fcb, encoder, encryptor, decryptor, evaluator, gk, rk,
                        std::min(T, S / (2 * round_to_2(F))));
            std::vector<Ciphertext> hid, bias{ fcb };
            row_matmul(a, bw.fc_w, bias, hid, T, d, F, encoder, encryptor, decryptor, evaluator, gk, rk);
            const double e = err_rows(hid, fx.at("hidden"));
            report("row_matmul ln2 x W_fc + b (16 x 64 . 64 x 256)", e < kTol, e, since(t));
        }

        // ------------------------------------------------------------ the block
        {
            auto x = enc_rows(X);
            std::vector<Ciphertext> y;
            BlockTrace tr;
            const auto t = std::chrono::steady_clock::now();
            transformer_block(x, bw, keep, y, dims, ap, bt, keygen, encoder, encryptor, decryptor, evaluator, gk, rk, &tr);
            const double secs = since(t);
            const double e_ln1 = err_rows(tr.ln1, fx.at("ln1")), e_attn = err_rows(tr.attn, fx.at("attn")),
                         e_x1 = err_rows(tr.x1, fx.at("x1")), e_ln2 = err_rows(tr.ln2, fx.at("ln2")),
                         e_ffn = err_rows(tr.ffn, fx.at("ffn")), e_y = err_rows(y, fx.at("y"));
            double e_exact = err_rows(y, fx.at("y_exact"));
            std::printf("   stages: ln1 %.3g  attn %.3g  x1 %.3g  ln2 %.3g  ffn %.3g  y %.3g; y %zu limbs; "
                        "vs exact GPT-2 block math %.3g\n",
                        e_ln1, e_attn, e_x1, e_ln2, e_ffn, e_y, y[0].coeff_modulus_size(), e_exact);
            if (fx.count("y_polygelu"))
                std::printf("   GELU x piece %s; y vs the block with plain_approx/poly.py's gelu as written (np.sign "
                            "on x, no sign approximation): %.3g\n",
                            ap.gelu_last == GeluLastPiece::reference ? "0.5 s2 (reference)" : "s2 + 1/2 (indicator)",
                            err_rows(y, fx.at("y_polygelu")));
            std::printf("block_seconds %.3f\n", secs);
            report("GPT-2 block (T " + std::to_string(T) + ", d " + std::to_string(d) + ", " + std::to_string(H) +
                       " heads, d_ff " + std::to_string(F) + ") vs plain restatement",
                   std::max({ e_ln1, e_attn, e_x1, e_ln2, e_ffn, e_y }) < kTol, e_y, secs);
        }
    }
    catch (const std::exception &e)
    {
        std::printf("exception: %s\nFAILED\n", e.what());
        return 1;
    }
    std::printf(g_fail ? "FAILED (%d)\n" : "ALL PASSED\n", g_fail);
    return g_fail ? 1 : 0;
}
