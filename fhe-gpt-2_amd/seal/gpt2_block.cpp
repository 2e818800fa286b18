// gpt2_block.cpp -- one GPT-2 transformer block over the encrypted packed layouts of the reference
// (gpt2_ckks/gpt2-ckks/single-key/gpt2/layers.cpp:3-72, which does not compile as written, and the
// plain pipeline it restates: plain_approx/full_gpt2.py:94-147, layers.py:24-116, attn.py:168-381,
// matrix_mul.py:51-109), plus the packing helpers of pack.cpp / pack.py and the KV-cache
// augmentation of optimize.cpp.
//
// Layouts (all in 32768-slot ciphertexts, as the reference):
//   row-packed  X (rows x d)      row r at slot (r % c) * 2R + j of ciphertext r / c, R = round_to_2(d),
//                                 c = 32768 / 2R                     (util.cpp:303-316, pack.py:55-75)
//   weights     W (d_in x d_out)  pack_from_row(W^T): column k of W as a row of the layout above
//   Q / K head  h                 row r at slot r * 2 dh + j of ciphertext h       (attn.py:99-118)
//   V head      h                 column j at slot j * 2T + r of ciphertext h      (attn.py:142-161)
//   scores head h                 row r at slot r * 2T + j of ciphertext h         (attn.py:187-203)
// Every matrix product is the reference's rotate / multiply / fold / quickSum followed by one mask
// and one rotation per output element (MatrixMul.cpp:118-188); products whose row or column falls
// outside the matrices contribute zeros and are skipped.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <exception>
#include <mutex>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <tuple>

#include "mhe_gpt2.h"

namespace gpt2
{
using seal::Plaintext;

namespace
{
constexpr int kSlots = 32768;

int wrap(long k)
{
    long m = k % kSlots;
    return (int)(m < 0 ? m + kSlots : m);
}

struct Ops
{
    CKKSEncoder &encoder;
    Encryptor &encryptor;
    Decryptor &decryptor;
    Evaluator &evaluator;
    GaloisKeys &gal_keys;
    RelinKeys &relin_keys;
};

// The limbs a matrix product's operands are dropped to before it runs: the product and the mask
// take two levels, and two limbs stay so the next bootstrap can prescale (gpt2.cpp).  Key
// switches cost ~L^2, so a product on a freshly bootstrapped (22-limb) operand is ~15x the cost
// at 5 limbs; dropping limbs does not change the values.  The second operand (weights, K, V) is
// kept one level above the first, so every product takes multiply_reduced_error's unequal-level
// path, which rescales it to the first operand's scale (evaluator.cpp:312-362) -- at equal levels
// the reduced-error product would overwrite that scale instead.
constexpr int kMatmulLimbs = 5;

Ciphertext dropped(const Ciphertext &c, int limbs, Evaluator &ev)
{
    Ciphertext r = c;
    while ((int)r.coeff_modulus_size() > limbs) ev.mod_switch_to_next_inplace(r);
    return r;
}

constexpr std::size_t kBatch = 8; // independent ciphertexts per batched launch (MHE_MAXB)

struct Accum
{
    std::vector<Ciphertext> &out;
    std::vector<char> has;
    Accum(std::vector<Ciphertext> &o, std::size_t n) : out(o), has(n, 0) { out.assign(n, Ciphertext()); }
    void add(std::size_t idx, Ciphertext &c, Evaluator &ev)
    {
        if (!has[idx])
        {
            out[idx] = c;
            has[idx] = 1;
        }
        else
            ev.add_inplace_reduced_error(out[idx], c);
    }
};

// x + x rotated right by `by` slots, folded by quickSum over `window` (the row sums of a row-packed
// ciphertext at every slot of the row)
void fold_sum(Ciphertext &x, int by, int window, Ciphertext &out, Ops &o)
{
    Ciphertext rolled;
    o.evaluator.rotate_vector(x, kSlots - by, o.gal_keys, rolled);
    o.evaluator.add_inplace_reduced_error(rolled, x);
    quickSum(rolled, out, window, o.encoder, o.encryptor, o.decryptor, o.evaluator, o.gal_keys, o.relin_keys);
}

// fold_sum(x, by, window) of every x in xs in place, each step's rotations in one batched launch
// (Evaluator::rotate_vectors): the same rotate / add sequence as fold_sum + quickSum (Fold.cpp:20-45)
void fold_many(std::vector<Ciphertext> &xs, int by, int window, Ops &o)
{
    const std::size_t B = xs.size();
    if (!B) return;
    std::vector<Ciphertext> tmp(B);
    std::vector<const Ciphertext *> in(B);
    std::vector<Ciphertext *> out(B);
    for (std::size_t b = 0; b < B; b++)
    {
        in[b] = &xs[b];
        out[b] = &tmp[b];
    }
    auto step = [&](int s) {
        o.evaluator.rotate_vectors(in, std::vector<int>(B, s), o.gal_keys, out);
        for (std::size_t b = 0; b < B; b++) o.evaluator.add_inplace_reduced_error(xs[b], tmp[b]);
    };
    step(kSlots - by);
    for (int s = 1; s < window; s *= 2) step(s);
}

// Output placement of folded products.  After fold_many(x, w, w) the dot product of a row whose
// window starts at slot w0 sits at EVERY slot of [w0, w0 + w), so an element bound for slot `dst`
// of output ciphertext t is read at src = w0 + ((dst - w0) mod w): its rotation k = src - dst is a
// multiple of w.  Elements sharing (t, k) are masked into one accumulator (one fused
// multiply_plain + add per folded ciphertext and group) and rotated once at the end, since rotation
// is linear -- instead of one mask, rescale and rotation per element (MatrixMul.cpp:160-180).
struct Placer
{
    Ops &o;
    explicit Placer(Ops &ops) : o(ops) {}
    std::map<std::tuple<int, int, std::size_t>, Ciphertext> groups; // (output, rotation, limbs)
    std::map<std::pair<int, int>, std::vector<std::pair<int, double>>> staged;
    Plaintext scratch;

    void element(int w0, int width, int t, int dst, double factor)
    {
        const int off = (int)((((long)dst - w0) % width + width) % width), src = w0 + off;
        staged[{ t, wrap((long)src - dst) }].push_back({ src, factor });
    }
    void flush(const Ciphertext &folded)
    {
        for (auto &kv : staged)
        {
            auto &el = kv.second;
            std::sort(el.begin(), el.end());
            // recipe id of the mask: two FNV-1a streams over its (slot, factor) pairs
            std::uint64_t hi = 0xcbf29ce484222325ULL, lo = 0x84222325cbf29ce4ULL;
            for (auto &e : el)
            {
                std::uint64_t fb;
                std::memcpy(&fb, &e.second, 8);
                for (std::uint64_t w : { (std::uint64_t)e.first, fb })
                {
                    hi = (hi ^ w) * 0x100000001b3ULL;
                    lo = (lo ^ (w + 0x9e3779b97f4a7c15ULL)) * 0x100000001b3ULL;
                    lo ^= lo >> 29;
                }
            }
            const Plaintext &pt = o.evaluator.cached_vector_plain(
                folded, hi, lo,
                [&]() {
                    std::vector<double> m(kSlots, 0.0);
                    for (auto &e : el) m[e.first] = e.second;
                    return m;
                },
                scratch);
            const auto key = std::make_tuple(kv.first.first, kv.first.second, folded.coeff_modulus_size());
            auto it = groups.find(key);
            if (it == groups.end())
                o.evaluator.multiply_plain(folded, pt, groups[key]);
            else
                o.evaluator.multiply_plain_add_reduced_error(it->second, folded, pt);
        }
        staged.clear();
    }
    // rescale every group, rotate it by its k (batched), sum into outputs[t]
    void finish(std::vector<Ciphertext> &outputs, std::size_t n_out)
    {
        std::vector<Ciphertext *> all;
        for (auto &g : groups) all.push_back(&g.second);
        o.evaluator.rescale_to_next_inplace_many(all);
        std::vector<const Ciphertext *> in;
        std::vector<int> steps;
        std::vector<Ciphertext> rotated;
        rotated.reserve(groups.size());
        std::vector<Ciphertext *> out;
        for (auto &g : groups)
            if (std::get<1>(g.first))
            {
                in.push_back(&g.second);
                steps.push_back(std::get<1>(g.first));
                rotated.emplace_back();
            }
        for (auto &r : rotated) out.push_back(&r);
        for (std::size_t b = 0; b < in.size(); b += kBatch)
        {
            const std::size_t e = std::min(in.size(), b + kBatch);
            o.evaluator.rotate_vectors(std::vector<const Ciphertext *>(in.begin() + b, in.begin() + e),
                                       std::vector<int>(steps.begin() + b, steps.begin() + e), o.gal_keys,
                                       std::vector<Ciphertext *>(out.begin() + b, out.begin() + e));
        }
        Accum acc(outputs, n_out);
        std::size_t r = 0;
        for (auto &g : groups)
        {
            const int t = std::get<0>(g.first);
            if ((std::size_t)t >= n_out) throw std::logic_error("Placer: output index");
            acc.add((std::size_t)t, std::get<1>(g.first) ? rotated[r++] : g.second, o.evaluator);
        }
        groups.clear();
        for (std::size_t k = 0; k < n_out; k++)
            if (!acc.has[k]) throw std::invalid_argument("packed_matmul: an output ciphertext received no element");
    }
};

// prods[b] = a[b] x w[b] (multiply_reduced_error), relinearized and rescaled in batched launches
void products(const std::vector<const Ciphertext *> &a, const std::vector<const Ciphertext *> &w,
              std::vector<Ciphertext> &prods, Ops &o)
{
    prods.assign(a.size(), Ciphertext());
    std::vector<Ciphertext *> p;
    for (auto &c : prods) p.push_back(&c);
    o.evaluator.multiply_reduced_error_many(a, w, o.relin_keys, p);
    o.evaluator.rescale_to_next_inplace_many(p);
}

// outs[b] = x rotated by steps[b] (0: a copy), in batched launches
void rotations_of(const Ciphertext &x, const std::vector<int> &steps, std::vector<Ciphertext> &outs, Ops &o)
{
    outs.assign(steps.size(), Ciphertext());
    std::vector<const Ciphertext *> in;
    std::vector<int> st;
    std::vector<Ciphertext *> out;
    for (std::size_t b = 0; b < steps.size(); b++)
        if (steps[b])
        {
            in.push_back(&x);
            st.push_back(steps[b]);
            out.push_back(&outs[b]);
        }
        else
            outs[b] = x;
    if (!in.empty()) o.evaluator.rotate_vectors(in, st, o.gal_keys, out);
}

// MatrixMul.cpp:118-188 / matrix_mul.py:51-109 with the output placement as a parameter:
// sink(row, col) -> {ciphertext index, destination slot, factor}; index < 0 drops the element.
// Each weight ciphertext's rotations are made once and shared by every input ciphertext; the
// products of one rotation run as a batch (products, rescales and every fold step in batched
// launches), and the placement is grouped (Placer).
struct Target
{
    int index, slot;
    double factor;
};
template <class Sink>
void packed_matmul_into(Placer &pl, const std::vector<Ciphertext> &A, const std::vector<Ciphertext> &W, int A_rows,
                        int A_cols, int W_cols, std::size_t n_out, Sink sink, Ops &o)
{
    const int R = round_to_2(A_cols), SA = 2 * R, c = kSlots / SA;
    if (A_cols < 1 || SA > kSlots) throw std::invalid_argument("packed_matmul: A_cols out of range");
    if ((long)A.size() * c < A_rows) throw std::invalid_argument("packed_matmul: too few input ciphertexts");
    if ((long)W.size() * c < W_cols) throw std::invalid_argument("packed_matmul: too few weight ciphertexts");
    Ciphertext rolled, Wj;
    std::vector<Ciphertext> prods;
    // operands at the fewest limbs the product needs (kMatmulLimbs), W one level above A
    std::vector<Ciphertext> Ad(A.size());
    int la = kMatmulLimbs;
    for (std::size_t i = 0; i < A.size(); i++)
    {
        Ad[i] = dropped(A[i], kMatmulLimbs, o.evaluator);
        la = std::min(la, (int)Ad[i].coeff_modulus_size());
    }
    std::size_t wj = W.size();
    for (std::size_t j = 0; j < W.size(); j++)
        for (int rots = 0; rots < c; rots++)
        {
            std::vector<std::size_t> is;
            for (std::size_t i = 0; i < A.size(); i++)
            {
                bool any = false;
                for (int pos = 0; pos < c && !any; pos++)
                    any = (int)i * c + pos < A_rows && (int)j * c + (rots + pos) % c < W_cols;
                if (any) is.push_back(i);
            }
            if (is.empty()) continue;
            if (wj != j)
            {
                Wj = dropped(W[j], la + 1, o.evaluator);
                wj = j;
            }
            if (rots)
                o.evaluator.rotate_vector(Wj, rots * SA, o.gal_keys, rolled);
            else
                rolled = Wj;
            for (std::size_t b0 = 0; b0 < is.size(); b0 += kBatch)
            {
                const std::size_t nb = std::min(kBatch, is.size() - b0);
                std::vector<const Ciphertext *> a(nb), w(nb, &rolled);
                for (std::size_t b = 0; b < nb; b++) a[b] = &Ad[is[b0 + b]];
                products(a, w, prods, o);
                fold_many(prods, R, R, o);
                for (std::size_t b = 0; b < nb; b++)
                {
                    const int i = (int)is[b0 + b];
                    for (int pos = 0; pos < c; pos++)
                    {
                        const int row = i * c + pos, col = (int)j * c + (rots + pos) % c;
                        if (row >= A_rows || col >= W_cols) continue;
                        const Target t = sink(row, col);
                        if (t.index < 0) continue;
                        if ((std::size_t)t.index >= n_out) throw std::logic_error("packed_matmul: sink index");
                        pl.element(pos * SA, R, t.index, t.slot, t.factor);
                    }
                    pl.flush(prods[b]);
                }
            }
        }
}

template <class Sink>
void packed_matmul(std::vector<Ciphertext> &A, std::vector<Ciphertext> &W, int A_rows, int A_cols, int W_cols,
                   std::size_t n_out, std::vector<Ciphertext> &outputs, Sink sink, Ops &o)
{
    Placer pl(o);
    packed_matmul_into(pl, A, W, A_rows, A_cols, W_cols, n_out, sink, o);
    pl.finish(outputs, n_out);
}

void add_bias(std::vector<Ciphertext> &outs, std::vector<Ciphertext> &bias, Evaluator &ev)
{
    if (bias.empty()) return;
    if (bias.size() != 1 && bias.size() < outs.size()) throw std::invalid_argument("bias: one ciphertext or one per output");
    for (std::size_t k = 0; k < outs.size(); k++) ev.add_inplace_reduced_error(outs[k], bias[bias.size() == 1 ? 0 : k]);
}

// replicate the first `period` slots over the whole ciphertext (period a power of two)
void replicate(Ciphertext &x, int period, Ops &o)
{
    Ciphertext rolled;
    for (int p = period; p < kSlots; p *= 2)
    {
        o.evaluator.rotate_vector(x, kSlots - p, o.gal_keys, rolled);
        o.evaluator.add_inplace_reduced_error(x, rolled);
    }
}

void ensure_levels(Ciphertext &c, int levels, Bootstrapper &bt, Evaluator &ev)
{
    // keep two limbs after `levels` rescales so the next bootstrap can prescale (gpt2.cpp)
    if ((int)c.coeff_modulus_size() - levels < 2)
    {
        Ciphertext r;
        bootstrap(c, r, bt, ev);
        c = r;
    }
}

// MHE_BLOCK_VERBOSE=1: elapsed seconds since the first call, per block sub-stage
void block_progress(const char *what)
{
    static const bool on = [] {
        const char *e = std::getenv("MHE_BLOCK_VERBOSE");
        return e && std::atoi(e) != 0;
    }();
    static const auto t0 = std::chrono::steady_clock::now();
    if (on)
        std::printf("    %-16s %.2f s\n", what,
                    std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
}

// f(i) for i in [0, n) on up to MHE_GPT2_THREADS threads (default 4; 1 = in order on the calling
// thread) whose evaluator calls merge into batched launches (seal::Lockstep): the heads / hidden
// ciphertexts / row groups of one block stage run the same operation sequence on different data
template <class F>
void lockstep_for(std::size_t n, F f)
{
    static const int threads = [] {
        const char *e = std::getenv("MHE_GPT2_THREADS");
        return e ? std::max(1, std::atoi(e)) : 4;
    }();
    if (threads <= 1 || n <= 1)
    {
        for (std::size_t i = 0; i < n; i++) f(i);
        return;
    }
    const std::size_t nt = std::min<std::size_t>((std::size_t)threads, n);
    seal::Lockstep group(nt);
    std::atomic<std::size_t> next{ 0 };
    std::exception_ptr err;
    std::mutex mu;
    std::vector<std::thread> pool;
    for (std::size_t t = 0; t < nt; t++)
        pool.emplace_back([&] {
            seal::Lockstep::Member member(group);
            try
            {
                for (std::size_t i; (i = next.fetch_add(1)) < n;) f(i);
            }
            catch (...)
            {
                std::lock_guard<std::mutex> g(mu);
                if (!err) err = std::current_exception();
            }
        });
    for (auto &t : pool) t.join();
    if (err) std::rethrow_exception(err);
}

void ensure_levels_all(std::vector<Ciphertext> &cs, int levels, Bootstrapper &bt, Evaluator &ev)
{
    lockstep_for(cs.size(), [&](std::size_t i) { ensure_levels(cs[i], levels, bt, ev); });
}

std::vector<double> tiled(const std::vector<double> &v, int rows, int stride, int first_row = 0)
{
    std::vector<double> out(kSlots, 0.0);
    for (int r = 0; r < rows; r++)
        for (std::size_t j = 0; j < v.size(); j++) out[(std::size_t)(first_row + r) * stride + j] = v[j];
    return out;
}
} // namespace

// ============================================================================ packing helpers
std::vector<double> repeat(const std::vector<double> &input, int times)
{
    // pack.cpp:180-187
    std::vector<double> result;
    result.reserve(input.size() * times);
    for (int r = 0; r < times; r++) result.insert(result.end(), input.begin(), input.end());
    return result;
}

void expand_bias(std::vector<double> &input, Ciphertext &output, CKKSEncoder &encoder, Encryptor &encryptor,
                 Decryptor &, Evaluator &, GaloisKeys &, RelinKeys &, int rows)
{
    // pack.py:78-83 (|bias|000|bias|000|...; pack.cpp:189-207 resizes the tile to the padding length
    // instead of padding it): the bias at the start of every 2 round_to_2(|bias|) slots, for the
    // first `rows` rows (all of them by default)
    const int sz = (int)input.size(), stride = round_to_2(sz) * 2;
    if (sz < 1 || stride > kSlots) throw std::invalid_argument("expand_bias: bias length");
    const int n = rows < 0 ? kSlots / stride : rows;
    if (n > kSlots / stride) throw std::invalid_argument("expand_bias: rows exceed one ciphertext");
    Plaintext plain;
    encoder.encode(tiled(input, n, stride), encode_scale(), plain);
    encryptor.encrypt(plain, output);
}

void expand_bias_head_row(std::vector<double> &input, std::vector<Ciphertext> &output, int heads,
                          CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &, Evaluator &, GaloisKeys &,
                          RelinKeys &, int rows)
{
    // pack.py:86-97 (pack.cpp:210-227 builds the vectors and drops them): head i's slice of the bias
    // at the start of every 2 sz slots for `rows` rows (16384 / 2 sz by default), one ciphertext per head
    if (heads < 1 || input.size() % heads) throw std::invalid_argument("expand_bias_head_row: heads must divide the bias");
    const int sz = (int)input.size() / heads;
    const int n = rows < 0 ? 16384 / (2 * sz) : rows;
    if ((long)n * 2 * sz > kSlots) throw std::invalid_argument("expand_bias_head_row: rows exceed one ciphertext");
    Plaintext plain;
    Ciphertext c;
    for (int i = 0; i < heads; i++)
    {
        std::vector<double> slice(input.begin() + i * sz, input.begin() + (i + 1) * sz);
        encoder.encode(tiled(slice, n, 2 * sz), encode_scale(), plain);
        encryptor.encrypt(plain, c);
        output.push_back(c);
    }
}

void expand_bias_head_col(std::vector<double> &input, std::vector<Ciphertext> &output, int heads, int rows, int cols,
                          CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &, Evaluator &evaluator, GaloisKeys &,
                          RelinKeys &)
{
    // pack.py:101-113 (pack.cpp:230-250 keeps adding a growing vector): head i's bias element j
    // repeated over slots [j 2 rows, j 2 rows + rows); added to output[i] when present (the
    // reference's "preformatted output"), encrypted otherwise
    if (heads < 1 || (long)heads * cols != (long)input.size())
        throw std::invalid_argument("expand_bias_head_col: heads * cols must equal the bias length");
    if ((long)cols * 2 * rows > kSlots) throw std::invalid_argument("expand_bias_head_col: cols x 2 rows exceed 32768");
    Plaintext plain;
    for (int i = 0; i < heads; i++)
    {
        std::vector<double> res(kSlots, 0.0);
        for (int j = 0; j < cols; j++) std::fill(res.begin() + (long)j * rows * 2, res.begin() + (long)j * rows * 2 + rows, input[i * cols + j]);
        if ((std::size_t)i < output.size())
        {
            encoder.encode(res, output[i].scale(), plain);
            evaluator.mod_switch_to_inplace(plain, output[i].parms_id());
            evaluator.add_plain_inplace(output[i], plain);
        }
        else
        {
            Ciphertext c;
            encoder.encode(res, encode_scale(), plain);
            encryptor.encrypt(plain, c);
            output.push_back(c);
        }
    }
}

std::vector<std::vector<std::vector<double>>> unpack_heads(const std::vector<std::vector<double>> &heads, int num_ciphers,
                                                           int num_rows, int row_size)
{
    // pack.py:116-125
    std::vector<std::vector<std::vector<double>>> out(num_ciphers,
                                                      std::vector<std::vector<double>>(num_rows, std::vector<double>(row_size)));
    for (int i = 0; i < num_ciphers; i++)
        for (int j = 0; j < num_rows; j++)
            for (int k = 0; k < row_size; k++) out[i][j][k] = heads.at(i).at((std::size_t)row_size * 2 * j + k);
    return out;
}

void pack_heads(std::vector<Ciphertext> &, std::vector<std::vector<double>> &output, int heads, int num_ciphers,
                int num_rows, int row_size, CKKSEncoder &, Encryptor &, Decryptor &, Evaluator &, GaloisKeys &,
                RelinKeys &)
{
    // pack.cpp:253-257 is an empty TODO; pack.py:127-133 is the plain operation, kept here on the
    // plain values of `output` (num_ciphers x num_rows*row_size, row-major): row j at slot 2 row_size j
    (void)heads;
    std::vector<std::vector<double>> packed(num_ciphers, std::vector<double>(kSlots, 0.0));
    for (int i = 0; i < num_ciphers; i++)
        for (int j = 0; j < num_rows; j++)
            for (int k = 0; k < row_size; k++)
                packed[i][(std::size_t)row_size * 2 * j + k] = output.at(i).at((std::size_t)j * row_size + k);
    output = packed;
}

void pack_tight(std::vector<Ciphertext> &input, std::vector<Ciphertext> &output, int rows, int row_size, int stride,
                CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator,
                GaloisKeys &gal_keys, RelinKeys &relin_keys)
{
    // pack.cpp:10-61 / pack.py:12-49 for any shape: `rows` rows of `row_size` values at `stride`
    // slots (32768 / stride rows per ciphertext) become one contiguous run; a row crossing a
    // ciphertext boundary is split in two masked pieces.  The reference's 768 / 2048 / 128 rows
    // (8 -> 3 ciphertexts) is pack_tight(input, output, 128, 768, 2048, ...).
    Ops o{ encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys };
    const int c = kSlots / stride;
    if (stride < row_size || (long)input.size() * c < rows) throw std::invalid_argument("pack_tight: shape");
    const std::size_t n_out = ((std::size_t)rows * row_size + kSlots - 1) / kSlots;
    Accum acc(output, n_out);
    Ciphertext piece;
    for (int r = 0; r < rows; r++)
    {
        const long g = (long)r * row_size;
        const int src = (r % c) * stride;
        int done = 0;
        while (done < row_size)
        {
            const long gd = g + done;
            const int dst = (int)(gd % kSlots), len = std::min(row_size - done, kSlots - dst);
            std::vector<double> m(kSlots, 0.0);
            std::fill(m.begin() + src + done, m.begin() + src + done + len, 1.0);
            o.evaluator.multiply_vector_reduced_error(input[r / c], m, piece);
            o.evaluator.rescale_to_next_inplace(piece);
            const int k = wrap((long)src + done - dst);
            if (k) o.evaluator.rotate_vector_inplace(piece, k, o.gal_keys);
            acc.add((std::size_t)(gd / kSlots), piece, o.evaluator);
            done += len;
        }
    }
}

void pack_tight(std::vector<Ciphertext> &input, std::vector<Ciphertext> &output, CKKSEncoder &encoder,
                Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                RelinKeys &relin_keys)
{
    pack_tight(input, output, 128, 768, 2048, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
}

void unpack_tight(std::vector<Ciphertext> &input, std::vector<Ciphertext> &output, int rows, int row_size, int stride,
                  CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator,
                  GaloisKeys &gal_keys, RelinKeys &relin_keys)
{
    // pack.cpp:101-150 / its pack.py comment: the inverse of pack_tight
    Ops o{ encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys };
    const int c = kSlots / stride;
    if (stride < row_size || (long)input.size() * kSlots < (long)rows * row_size) throw std::invalid_argument("unpack_tight: shape");
    const std::size_t n_out = ((std::size_t)rows + c - 1) / c;
    Accum acc(output, n_out);
    Ciphertext piece;
    for (int r = 0; r < rows; r++)
    {
        const long g = (long)r * row_size;
        const int dst = (r % c) * stride;
        int done = 0;
        while (done < row_size)
        {
            const long gs = g + done;
            const int src = (int)(gs % kSlots), len = std::min(row_size - done, kSlots - src);
            std::vector<double> m(kSlots, 0.0);
            std::fill(m.begin() + src, m.begin() + src + len, 1.0);
            o.evaluator.multiply_vector_reduced_error(input[gs / kSlots], m, piece);
            o.evaluator.rescale_to_next_inplace(piece);
            const int k = wrap((long)src - (dst + done));
            if (k) o.evaluator.rotate_vector_inplace(piece, k, o.gal_keys);
            acc.add((std::size_t)(r / c), piece, o.evaluator);
            done += len;
        }
    }
}

void unpack_tight(std::vector<Ciphertext> &input, std::vector<Ciphertext> &output, CKKSEncoder &encoder,
                  Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                  RelinKeys &relin_keys)
{
    unpack_tight(input, output, 128, 768, 2048, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
}

// ============================================================================ KV cache (optimize.cpp)
void augment_value_row(std::vector<Ciphertext> &A, std::vector<Ciphertext> &cached_val, int padded_row_size, int idx,
                       CKKSEncoder &, Encryptor &, Decryptor &, Evaluator &evaluator, GaloisKeys &, RelinKeys &)
{
    // optimize.cpp:4-22: row idx of A kept, every other row taken from the cache
    if (cached_val.size() < A.size()) throw std::invalid_argument("augment_value_row: cache smaller than A");
    if ((long)(idx + 1) * padded_row_size > kSlots) throw std::invalid_argument("augment_value_row: idx");
    std::vector<double> mask(kSlots, 1.0);
    std::fill(mask.begin() + (long)idx * padded_row_size, mask.begin() + (long)(idx + 1) * padded_row_size, 0.0);
    for (std::size_t i = 0; i < A.size(); i++)
    {
        evaluator.multiply_vector_inplace_reduced_error(A[i], mask);
        evaluator.rescale_to_next_inplace(A[i]);
        evaluator.add_inplace_reduced_error(A[i], cached_val[i]);
    }
}

void augment_value_col(std::vector<Ciphertext> &A, std::vector<Ciphertext> &cached_val, int padded_row_size, int idx,
                       CKKSEncoder &, Encryptor &, Decryptor &, Evaluator &evaluator, GaloisKeys &gal_keys,
                       RelinKeys &)
{
    // optimize.cpp:24-40: column idx of the cache cleared, A rotated by idx and added.  The reference
    // multiplies the cache by the mask without rescaling and then adds at the same level, where
    // add_inplace_reduced_error overwrites A's scale with the product's squared scale; the product
    // is rescaled first here.
    if (cached_val.size() < A.size()) throw std::invalid_argument("augment_value_col: cache smaller than A");
    std::vector<double> mask(kSlots, 1.0);
    for (int i = 0; i < padded_row_size / 2; i++)
        if ((long)i * padded_row_size + idx < kSlots) mask[(std::size_t)i * padded_row_size + idx] = 0.0;
    for (std::size_t i = 0; i < A.size(); i++)
    {
        evaluator.multiply_vector_inplace_reduced_error(cached_val[i], mask);
        evaluator.rescale_to_next_inplace(cached_val[i]);
        evaluator.rotate_vector_inplace(A[i], idx, gal_keys);
        evaluator.add_inplace_reduced_error(A[i], cached_val[i]);
    }
}

// ============================================================================ block pieces
void row_matmul(std::vector<Ciphertext> &A, std::vector<Ciphertext> &W, std::vector<Ciphertext> bias,
                std::vector<Ciphertext> &outputs, int A_rows, int A_cols, int W_cols, CKKSEncoder &encoder,
                Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                RelinKeys &relin_keys)
{
    // generic_matrix_mul (matrix_mul.py:51-109): A (A_rows x A_cols) times W, W given as
    // pack_from_row(W^T); the output row-packed at 2 round_to_2(W_cols)
    Ops o{ encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys };
    const int SO = 2 * round_to_2(W_cols), cO = kSlots / SO;
    if (SO > kSlots) throw std::invalid_argument("row_matmul: W_cols");
    const std::size_t n_out = (std::size_t)(A_rows + cO - 1) / cO;
    packed_matmul(A, W, A_rows, A_cols, W_cols, n_out, outputs,
                  [&](int row, int col) { return Target{ row / cO, (row % cO) * SO + col, 1.0 }; }, o);
    add_bias(outputs, bias, evaluator);
}

void attn_proj_heads(std::vector<Ciphertext> &A, std::vector<Ciphertext> &W, std::vector<Ciphertext> &bias,
                     std::vector<Ciphertext> &outputs, int rows, int d_model, int heads, bool column_layout,
                     CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator,
                     GaloisKeys &gal_keys, RelinKeys &relin_keys)
{
    // expensive_matrix_mul_row / _col (attn.py:77-166): the projection of A by W, element (r, col)
    // sent to head col / dh at r * 2 dh + col % dh (row layout) or (col % dh) * 2 rows + r (column
    // layout); MatrixMul.cpp:244-478 is this operation in its unfinished state (gpt2.cpp)
    Ops o{ encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys };
    if (heads < 1 || d_model % heads) throw std::invalid_argument("attn_proj_heads: heads must divide d_model");
    const int dh = d_model / heads;
    if (column_layout ? (long)dh * 2 * rows > kSlots : (long)rows * 2 * dh > kSlots)
        throw std::invalid_argument("attn_proj_heads: one head must fit one ciphertext");
    packed_matmul(A, W, rows, d_model, d_model, (std::size_t)heads, outputs,
                  [&](int row, int col) {
                      const int h = col / dh, hc = col % dh;
                      return Target{ h, column_layout ? hc * 2 * rows + row : row * 2 * dh + hc, 1.0 };
                  },
                  o);
    add_bias(outputs, bias, evaluator);
}

void qk_heads(std::vector<Ciphertext> &Q, std::vector<Ciphertext> &K, std::vector<Ciphertext> &outputs, int rows,
              int head_dim, CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator,
              GaloisKeys &gal_keys, RelinKeys &relin_keys)
{
    // qk_matmul (attn.py:168-204, MatrixMul.cpp:480-533): K replicated with period rows * 2 dh, rotated
    // by whole rows, multiplied with Q, folded over dh; entry (r, (r + rots) % rows) placed at
    // r * 2 rows + col of the head's score ciphertext, scaled by 1 / sqrt(dh) (attn.py:359).  The
    // rotations of K, the products and the folds of kBatch row offsets run as batches; placement
    // grouped (Placer).
    Ops o{ encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys };
    const int dh = head_dim, P = rows * 2 * dh;
    if (P > kSlots || (long)rows * 2 * rows > kSlots || (kSlots % P)) throw std::invalid_argument("qk_heads: shape");
    if (K.size() < Q.size()) throw std::invalid_argument("qk_heads: one K ciphertext per Q ciphertext");
    outputs.assign(Q.size(), Ciphertext());
    const double inv_sqrt = 1.0 / std::sqrt((double)dh);
    Ciphertext dup;
    std::vector<Ciphertext> rolled, prods;
    for (std::size_t h = 0; h < Q.size(); h++)
    {
        const Ciphertext q = dropped(Q[h], kMatmulLimbs, o.evaluator);
        dup = dropped(K[h], (int)q.coeff_modulus_size() + 1, o.evaluator);
        replicate(dup, P, o);
        Placer pl(o);
        for (int r0 = 0; r0 < rows; r0 += (int)kBatch)
        {
            const int nb = std::min((int)kBatch, rows - r0);
            std::vector<int> steps(nb);
            for (int b = 0; b < nb; b++) steps[b] = (r0 + b) * 2 * dh;
            rotations_of(dup, steps, rolled, o);
            std::vector<const Ciphertext *> a(nb, &q), w(nb);
            for (int b = 0; b < nb; b++) w[b] = &rolled[b];
            products(a, w, prods, o);
            fold_many(prods, dh, dh, o);
            for (int b = 0; b < nb; b++)
            {
                const int rots = r0 + b;
                for (int pos = 0; pos < rows; pos++)
                    pl.element(pos * 2 * dh, dh, 0, pos * 2 * rows + (pos + rots) % rows, inv_sqrt);
                pl.flush(prods[b]);
            }
        }
        std::vector<Ciphertext> one;
        pl.finish(one, 1);
        outputs[h] = one[0];
    }
}

void sv_heads(std::vector<Ciphertext> &S, std::vector<Ciphertext> &V, std::vector<Ciphertext> &outputs, int rows,
              int head_dim, int d_model, CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor,
              Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys)
{
    // sv_matmul (attn.py:271-316, MatrixMul.cpp:535-584): V (column layout) replicated with period
    // dh * 2 rows, rotated by whole rows, multiplied with the scores, folded over rows; entry
    // (r, (r + rots) % dh) of head h placed at row r, column h dh + that of the row-packed output.
    // Batched and grouped as qk_heads.
    Ops o{ encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys };
    const int dh = head_dim, P = dh * 2 * rows, SO = 2 * round_to_2(d_model), cO = kSlots / SO;
    if (P > kSlots || (kSlots % P)) throw std::invalid_argument("sv_heads: shape");
    if (V.size() < S.size()) throw std::invalid_argument("sv_heads: one V ciphertext per score ciphertext");
    const std::size_t n_out = (std::size_t)(rows + cO - 1) / cO;
    Placer pl(o);
    Ciphertext dup;
    std::vector<Ciphertext> rolled, prods;
    for (std::size_t h = 0; h < S.size(); h++)
    {
        const Ciphertext sc = dropped(S[h], kMatmulLimbs, o.evaluator);
        dup = dropped(V[h], (int)sc.coeff_modulus_size() + 1, o.evaluator);
        replicate(dup, P, o);
        for (int r0 = 0; r0 < dh; r0 += (int)kBatch)
        {
            const int nb = std::min((int)kBatch, dh - r0);
            std::vector<int> steps(nb);
            for (int b = 0; b < nb; b++) steps[b] = (r0 + b) * 2 * rows;
            rotations_of(dup, steps, rolled, o);
            std::vector<const Ciphertext *> a(nb, &sc), w(nb);
            for (int b = 0; b < nb; b++) w[b] = &rolled[b];
            products(a, w, prods, o);
            fold_many(prods, rows, rows, o);
            for (int b = 0; b < nb; b++)
            {
                const int rots = r0 + b;
                for (int pos = 0; pos < rows; pos++)
                {
                    const int col = (int)h * dh + (pos + rots) % dh;
                    pl.element(pos * 2 * rows, rows, pos / cO, (pos % cO) * SO + col, 1.0);
                }
                pl.flush(prods[b]);
            }
        }
    }
    pl.finish(outputs, n_out);
}

void compute_inverse_norm(Ciphertext &input, Ciphertext &output, int iters, double normalize_factor,
                          CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &, Evaluator &evaluator, GaloisKeys &,
                          RelinKeys &relin_keys)
{
    // IterApprox.cpp:15-68 with the normalisation as a parameter (the reference's 0.001)
    Ciphertext two_cipher, d_cipher, f_cipher;
    Plaintext plain;
    std::vector<double> one_vec(kSlots, normalize_factor), two_vec(kSlots, 2.0);
    encoder.encode(one_vec, encode_scale(), plain);
    evaluator.mod_switch_to_inplace(plain, input.parms_id());
    encryptor.encrypt(plain, output);
    encoder.encode(two_vec, encode_scale(), plain);
    evaluator.mod_switch_to_inplace(plain, input.parms_id());
    encryptor.encrypt(plain, two_cipher);
    evaluator.multiply_const(input, normalize_factor, d_cipher);
    evaluator.rescale_to_next_inplace(d_cipher);
    for (int i = 0; i < iters; i++)
    {
        evaluator.sub_reduced_error(two_cipher, d_cipher, f_cipher);
        evaluator.multiply_inplace_reduced_error(output, f_cipher, relin_keys);
        evaluator.rescale_to_next_inplace(output);
        evaluator.multiply_inplace_reduced_error(d_cipher, f_cipher, relin_keys);
        evaluator.rescale_to_next_inplace(d_cipher);
    }
}

void compute_softmax_rows(Ciphertext &input, int n, const std::vector<double> &keep_mask, double inv_norm,
                          int inv_iters, Bootstrapper &bootstrapper, CKKSEncoder &encoder, Encryptor &encryptor,
                          Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys)
{
    // compute_softmax (PolyApprox.cpp:533-593) for rows of n at stride 2n: fold the row into its
    // padding, quickMax over n (bootstrapped), x - max, exp, keep_mask (padding and masked
    // entries to 0), bootstrap, fold + quickSum, Goldschmidt 1/sum, product
    if (n < 2 || (n & (n - 1)) || (int)keep_mask.size() != kSlots)
        throw std::invalid_argument("compute_softmax_rows: n a power of two >= 2, keep_mask 32768 slots");
    Ciphertext rolled, maxes, exps, summed, inverses;
    evaluator.rotate_vector(input, kSlots - n, gal_keys, rolled);
    evaluator.add_inplace_reduced_error(input, rolled);
    ensure_levels(input, 20, bootstrapper, evaluator);
    quickMax(input, maxes, n, bootstrapper, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
    evaluator.sub_inplace_reduced_error(input, maxes);
    compute_exp(input, exps, 6, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
    evaluator.multiply_vector_inplace_reduced_error(exps, keep_mask);
    evaluator.rescale_to_next_inplace(exps);
    {
        Ciphertext refreshed;
        bootstrap(exps, refreshed, bootstrapper, evaluator);
        exps = refreshed;
    }
    evaluator.rotate_vector(exps, -n, gal_keys, rolled);
    evaluator.add_inplace_reduced_error(rolled, exps);
    quickSum(rolled, summed, n, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
    compute_inverse_norm(summed, inverses, inv_iters, inv_norm, encoder, encryptor, decryptor, evaluator, gal_keys,
                         relin_keys);
    evaluator.multiply_reduced_error(exps, inverses, relin_keys, input);
    evaluator.rescale_to_next_inplace(input);
}

void layer_norm_rows(Ciphertext &input, Ciphertext &output, const std::vector<double> &gamma,
                     const std::vector<double> &beta, int rows, int row_size, int newton_iters,
                     Bootstrapper &bootstrapper, CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor,
                     Evaluator &evaluator, GaloisKeys &gal_keys, RelinKeys &relin_keys)
{
    // layer_norm (plain_approx/layers.py:24-90) on one row-packed ciphertext holding `rows` rows:
    // row sums by fold + quickSum, mean by 1/d, z = x - mean masked to the rows, variance the same
    // way, 1/sqrt(var) from 1 - (u-1)/2 + 3(u-1)^2/8 and Newton steps y (1.5 - u/2 y^2)
    // (iterations.py:15-21; compute_inv_sqrt's fakeBootstrap decrypts, here every level is
    // budgeted and the input refreshed by bootstrapping when it is short), then gamma, beta
    Ops o{ encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys };
    const int R = round_to_2(row_size), S = 2 * R;
    if ((int)gamma.size() != row_size || (int)beta.size() != row_size || (long)rows * S > kSlots)
        throw std::invalid_argument("layer_norm_rows: gamma / beta length or rows");
    std::vector<double> rowmask(kSlots, 0.0);
    for (int r = 0; r < rows; r++) std::fill(rowmask.begin() + (long)r * S, rowmask.begin() + (long)r * S + row_size, 1.0);
    ensure_levels(input, 6 + 3 * newton_iters + 2, bootstrapper, evaluator);
    Ciphertext sums, mean, z, sq, u, t, t2, a, b, y, h, y2, w;
    fold_sum(input, R, R, sums, o);
    evaluator.multiply_const(sums, 1.0 / row_size, mean);
    evaluator.rescale_to_next_inplace(mean);
    evaluator.sub_reduced_error(input, mean, z);
    evaluator.multiply_vector_inplace_reduced_error(z, rowmask);
    evaluator.rescale_to_next_inplace(z);
    evaluator.square(z, sq);
    evaluator.relinearize_inplace(sq, relin_keys);
    evaluator.rescale_to_next_inplace(sq);
    fold_sum(sq, R, R, sums, o);
    evaluator.multiply_const(sums, 1.0 / row_size, u);
    evaluator.rescale_to_next_inplace(u);
    // y0 = 1 + (-1/2)(u - 1) + (3/8)(u - 1)^2
    evaluator.add_const(u, -1.0, t);
    evaluator.square(t, t2);
    evaluator.relinearize_inplace(t2, relin_keys);
    evaluator.rescale_to_next_inplace(t2);
    evaluator.multiply_const(t, -0.5, a);
    evaluator.rescale_to_next_inplace(a);
    evaluator.add_const_inplace(a, 1.0);
    evaluator.multiply_const(t2, 0.375, b);
    evaluator.rescale_to_next_inplace(b);
    evaluator.add_reduced_error(a, b, y);
    evaluator.multiply_const(u, -0.5, h);
    evaluator.rescale_to_next_inplace(h);
    for (int k = 0; k < newton_iters; k++)
    {
        evaluator.square(y, y2);
        evaluator.relinearize_inplace(y2, relin_keys);
        evaluator.rescale_to_next_inplace(y2);
        evaluator.multiply_reduced_error(y2, h, relin_keys, w);
        evaluator.rescale_to_next_inplace(w);
        evaluator.add_const_inplace(w, 1.5);
        evaluator.multiply_inplace_reduced_error(y, w, relin_keys);
        evaluator.rescale_to_next_inplace(y);
    }
    evaluator.multiply_reduced_error(z, y, relin_keys, output);
    evaluator.rescale_to_next_inplace(output);
    std::vector<double> g = tiled(gamma, rows, S), bb = tiled(beta, rows, S);
    evaluator.multiply_vector_inplace_reduced_error(output, g);
    evaluator.rescale_to_next_inplace(output);
    Plaintext plain;
    encoder.encode(bb, output.scale(), plain);
    evaluator.mod_switch_to_inplace(plain, output.parms_id());
    evaluator.add_plain_inplace(output, plain);
}

void compute_gelu_block(Ciphertext &inputs, Ciphertext &outputs, double alpha, CKKSEncoder &encoder,
                        Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                        RelinKeys &relin_keys, GeluLastPiece last)
{
    // compute_gelu (PolyApprox.cpp:443-504, poly.py:30-35) with the signs taken of alpha (x + shift)
    // so they stay inside the composite sign's [-1, 1] (the reference feeds x - 3, x + 1.95, x + 4
    // unscaled, where the composite sign diverges), and the x piece weighted by s2 + 1/2 (the
    // indicator of x >= 3) or, with GeluLastPiece::reference, by 0.5 s2 as the reference writes it
    // (multiply_const + rescale, PolyApprox.cpp:484-485)
    Ciphertext y, s0, s1, s2, tc, b1, b2, b3, p, q;
    evaluator.multiply_const(inputs, alpha, y);
    evaluator.rescale_to_next_inplace(y);
    auto half_sign = [&](double shift, Ciphertext &s) {
        evaluator.add_const(y, alpha * shift, s);
        sign_function(s, tc, 2, 2, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
        evaluator.multiply_const(tc, 0.5, s);
        evaluator.rescale_to_next_inplace(s);
    };
    half_sign(-3.0, s2);
    half_sign(1.95, s1);
    half_sign(4.0, s0);
    evaluator.sub_reduced_error(s0, s1, b1);
    evaluator.sub_reduced_error(s1, s2, b2);
    if (last == GeluLastPiece::reference)
    {
        evaluator.multiply_const(s2, 0.5, b3);
        evaluator.rescale_to_next_inplace(b3);
    }
    else
        evaluator.add_const(s2, 0.5, b3);
    compute_gelu_p(inputs, p, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
    compute_gelu_q(inputs, q, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
    evaluator.multiply_reduced_error(b1, p, relin_keys, outputs);
    evaluator.rescale_to_next_inplace(outputs);
    evaluator.multiply_inplace_reduced_error(b2, q, relin_keys);
    evaluator.rescale_to_next_inplace(b2);
    evaluator.multiply_inplace_reduced_error(b3, inputs, relin_keys);
    evaluator.rescale_to_next_inplace(b3);
    evaluator.add_inplace_reduced_error(outputs, b2);
    evaluator.add_inplace_reduced_error(outputs, b3);
}

// ============================================================================ layers.cpp
void attentionLayer(std::vector<Ciphertext> &A, std::vector<Ciphertext> &qw, std::vector<Ciphertext> &qb,
                    std::vector<Ciphertext> &kw, std::vector<Ciphertext> &kb, std::vector<Ciphertext> &vw,
                    std::vector<Ciphertext> &vb, std::vector<Ciphertext> &w_out, Ciphertext &b_out,
                    const std::vector<std::vector<double>> &keep, std::vector<std::vector<Ciphertext>> &kv_cache,
                    std::vector<Ciphertext> &outputs, int rows, int cols, int heads, int idx,
                    const AttentionParams &params, Bootstrapper &bootstrapper, seal::KeyGenerator &,
                    CKKSEncoder &encoder, Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator,
                    GaloisKeys &gal_keys, RelinKeys &relin_keys)
{
    // layers.cpp:26-72 (attn.py:324-381): Q, K (row head layout) and V (column head layout)
    // projections, the KV-cache augmentation when a cache is given, Q K^T / sqrt(dh), the causal
    // mask, softmax per head, S V into the row-packed layout and the output projection.  The mask
    // is `keep` (rows x rows, 1 = attend): masked scores are set to params.masked_score before the
    // row max and the masked probabilities to 0 after exp (attn.py:365 adds -1e5, which the sign
    // step of computeMax cannot take).
    if (heads < 1 || cols % heads) throw std::invalid_argument("attentionLayer: heads must divide cols");
    if ((int)keep.size() != rows) throw std::invalid_argument("attentionLayer: keep must be rows x rows");
    const int dh = cols / heads;
    ensure_levels_all(A, 4, bootstrapper, evaluator);
    std::vector<Ciphertext> Q, K, V, S, pre_out;
    attn_proj_heads(A, qw, qb, Q, rows, cols, heads, false, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
    attn_proj_heads(A, kw, kb, K, rows, cols, heads, false, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
    attn_proj_heads(A, vw, vb, V, rows, cols, heads, true, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
    block_progress("qkv projections");
    if (!kv_cache.empty())
    {
        if (kv_cache.size() < 2) throw std::invalid_argument("attentionLayer: kv_cache holds K and V");
        augment_value_row(K, kv_cache[0], 2 * dh, idx, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
        augment_value_col(V, kv_cache[1], 2 * rows, idx, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
        kv_cache[0] = K;
        kv_cache[1] = V;
    }
    ensure_levels_all(Q, 3, bootstrapper, evaluator);
    ensure_levels_all(K, 3, bootstrapper, evaluator);
    qk_heads(Q, K, S, rows, dh, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
    block_progress("q.k^t");
    std::vector<double> keep_slots(kSlots, 0.0), pin(kSlots, 0.0);
    for (int r = 0; r < rows; r++)
    {
        if ((int)keep[r].size() != rows) throw std::invalid_argument("attentionLayer: keep must be rows x rows");
        for (int j = 0; j < rows; j++)
        {
            keep_slots[(std::size_t)r * 2 * rows + j] = keep[r][j] != 0.0 ? 1.0 : 0.0;
            pin[(std::size_t)r * 2 * rows + j] = keep[r][j] != 0.0 ? 0.0 : params.masked_score;
        }
    }
    lockstep_for(S.size(), [&](std::size_t h) {
        Ciphertext &s = S[h];
        Plaintext plain;
        ensure_levels(s, 1, bootstrapper, evaluator);
        evaluator.multiply_vector_inplace_reduced_error(s, keep_slots);
        evaluator.rescale_to_next_inplace(s);
        encoder.encode(pin, s.scale(), plain);
        evaluator.mod_switch_to_inplace(plain, s.parms_id());
        evaluator.add_plain_inplace(s, plain);
        compute_softmax_rows(s, rows, keep_slots, params.inv_norm > 0 ? params.inv_norm : 1.0 / rows, params.inv_iters,
                             bootstrapper, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
    });
    block_progress("softmax");
    ensure_levels_all(V, 3, bootstrapper, evaluator);
    ensure_levels_all(S, 3, bootstrapper, evaluator);
    sv_heads(S, V, pre_out, rows, dh, cols, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
    block_progress("s.v");
    ensure_levels_all(pre_out, 3, bootstrapper, evaluator);
    std::vector<Ciphertext> bias{ b_out };
    row_matmul(pre_out, w_out, bias, outputs, rows, cols, cols, encoder, encryptor, decryptor, evaluator, gal_keys,
               relin_keys);
}

void FeedForwardLayer(std::vector<Ciphertext> &A, std::vector<Ciphertext> &W1, std::vector<Ciphertext> &b1,
                      std::vector<Ciphertext> &W2, Ciphertext b2, std::vector<Ciphertext> &outputs, int rows, int cols,
                      int d_ff, double gelu_alpha, Bootstrapper &bootstrapper, CKKSEncoder &encoder,
                      Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                      RelinKeys &relin_keys, GeluLastPiece gelu_last)
{
    // layers.cpp:3-24 (layers.py:93-116): dense to d_ff, GELU, dense back, biases after each.  The
    // hidden state is held in `cols`-wide column chunks, each row-packed like the input: FC1 then
    // places every element inside its own row's window (one mask per folded product instead of one
    // per output row; the reference's stride-2*d_ff layout would need a rotation group per row), GELU
    // is elementwise, and FC2 sums the chunks' products (chunk k times rows k*cols.. of W2) into one
    // placement.  W2 / b1 come chunked from encrypt_block_weights.
    Ops o{ encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys };
    const int SA = 2 * round_to_2(cols), c = kSlots / SA, cpc = (rows + c - 1) / c;
    const int nchunk = (d_ff + cols - 1) / cols, wpc = (cols + c - 1) / c;
    if ((int)b1.size() != nchunk) throw std::invalid_argument("FeedForwardLayer: one FC1 bias per hidden chunk");
    if ((int)W2.size() != nchunk * wpc) throw std::invalid_argument("FeedForwardLayer: W2 must be packed per chunk");
    ensure_levels_all(A, 3, bootstrapper, evaluator);
    std::vector<Ciphertext> hidden;
    packed_matmul(A, W1, rows, cols, d_ff, (std::size_t)(nchunk * cpc), hidden,
                  [&](int row, int col) {
                      return Target{ (col / cols) * cpc + row / c, (row % c) * SA + col % cols, 1.0 };
                  },
                  o);
    for (int k = 0; k < nchunk; k++)
        for (int i = 0; i < cpc; i++) evaluator.add_inplace_reduced_error(hidden[(std::size_t)(k * cpc + i)], b1[k]);
    block_progress("fc");
    lockstep_for(hidden.size(), [&](std::size_t i) {
        Ciphertext &h = hidden[i];
        ensure_levels(h, 20, bootstrapper, evaluator);
        Ciphertext g;
        compute_gelu_block(h, g, gelu_alpha, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys, gelu_last);
        h = g;
        ensure_levels(h, 3, bootstrapper, evaluator);
    });
    block_progress("gelu");
    Placer pl(o);
    for (int k = 0; k < nchunk; k++)
    {
        std::vector<Ciphertext> hk(hidden.begin() + k * cpc, hidden.begin() + (k + 1) * cpc);
        std::vector<Ciphertext> wk(W2.begin() + k * wpc, W2.begin() + (k + 1) * wpc);
        packed_matmul_into(pl, hk, wk, rows, cols, cols, (std::size_t)cpc,
                           [&](int row, int col) { return Target{ row / c, (row % c) * SA + col, 1.0 }; }, o);
    }
    pl.finish(outputs, (std::size_t)cpc);
    std::vector<Ciphertext> bias2{ b2 };
    add_bias(outputs, bias2, evaluator);
}

void transformer_block(std::vector<Ciphertext> &x, BlockWeights &w, const std::vector<std::vector<double>> &keep,
                       std::vector<Ciphertext> &y, const BlockDims &dims, const AttentionParams &params,
                       Bootstrapper &bootstrapper, seal::KeyGenerator &keygen, CKKSEncoder &encoder,
                       Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                       RelinKeys &relin_keys, BlockTrace *trace)
{
    // full_gpt2.py:94-147: LN1 -> attention -> residual -> LN2 -> MLP -> residual
    const int T = dims.rows, d = dims.d_model;
    // MHE_BLOCK_VERBOSE=1: the elapsed time after each stage on stdout
    static const bool verbose = [] {
        const char *e = std::getenv("MHE_BLOCK_VERBOSE");
        return e && std::atoi(e) != 0;
    }();
    const auto t0 = std::chrono::steady_clock::now();
    auto stage = [&](const char *name) {
        if (verbose)
            std::printf("  block stage %-10s done at %.2f s\n", name,
                        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    };
    const int c = kSlots / (2 * round_to_2(d));
    auto ln = [&](std::vector<Ciphertext> &in, const std::vector<double> &g, const std::vector<double> &b) {
        std::vector<Ciphertext> out(in.size());
        lockstep_for(in.size(), [&](std::size_t i) {
            const int r = std::min(c, T - (int)i * c);
            layer_norm_rows(in[i], out[i], g, b, r, d, params.newton_iters, bootstrapper, encoder, encryptor,
                            decryptor, evaluator, gal_keys, relin_keys);
        });
        return out;
    };
    std::vector<std::vector<Ciphertext>> no_cache;
    std::vector<Ciphertext> ln1 = ln(x, w.ln1_g, w.ln1_b);
    stage("ln1");
    if (trace) trace->ln1 = ln1;
    std::vector<Ciphertext> attn;
    attentionLayer(ln1, w.qw, w.qb, w.kw, w.kb, w.vw, w.vb, w.ow, w.ob, keep, no_cache, attn, T, d, dims.heads, 0,
                   params, bootstrapper, keygen, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
    stage("attention");
    if (trace) trace->attn = attn;
    std::vector<Ciphertext> x1(x.size());
    for (std::size_t i = 0; i < x.size(); i++) evaluator.add_reduced_error(attn[i], x[i], x1[i]);
    if (trace) trace->x1 = x1;
    std::vector<Ciphertext> ln2 = ln(x1, w.ln2_g, w.ln2_b);
    stage("ln2");
    if (trace) trace->ln2 = ln2;
    std::vector<Ciphertext> ffn;
    FeedForwardLayer(ln2, w.fc_w, w.fc_b, w.pj_w, w.pj_b, ffn, T, d, dims.d_ff, params.gelu_alpha, bootstrapper,
                     encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys, params.gelu_last);
    stage("ffn");
    if (trace) trace->ffn = ffn;
    y.assign(x.size(), Ciphertext());
    for (std::size_t i = 0; i < x.size(); i++) evaluator.add_reduced_error(ffn[i], x1[i], y[i]);
}

void encrypt_block_weights(const PlainBlockWeights &p, BlockWeights &w, const BlockDims &dims, CKKSEncoder &encoder,
                           Encryptor &encryptor, Decryptor &decryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                           RelinKeys &relin_keys, int limbs)
{
    // full_gpt2.py:17-78 (gpt2_setup): weights column-packed by pack_from_row(W^T), Q/K biases by
    // expand_bias_head_row, the V bias by expand_bias_head_col, the others by expand_bias -- limited
    // to the block's rows.  Ciphertexts are dropped to `limbs` (the levels a bootstrap refreshes).
    const int T = dims.rows, d = dims.d_model, H = dims.heads, dh = d / H, F = dims.d_ff;
    auto drop = [&](Ciphertext &c) {
        while (limbs > 0 && (int)c.coeff_modulus_size() > limbs) evaluator.mod_switch_to_next_inplace(c);
    };
    auto pack_w = [&](const std::vector<double> &W, int din, int dout, std::vector<Ciphertext> &out) {
        if ((long)W.size() != (long)din * dout) throw std::invalid_argument("encrypt_block_weights: weight shape");
        std::vector<std::vector<double>> wt(dout, std::vector<double>(din));
        for (int i = 0; i < din; i++)
            for (int j = 0; j < dout; j++) wt[j][i] = W[(std::size_t)i * dout + j];
        out.clear();
        pack_from_row(wt, out, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
        for (auto &c : out) drop(c);
    };
    pack_w(p.qw, d, d, w.qw);
    pack_w(p.kw, d, d, w.kw);
    pack_w(p.vw, d, d, w.vw);
    pack_w(p.ow, d, d, w.ow);
    pack_w(p.fc_w, d, F, w.fc_w);
    // W2 (F x d) by d-row chunks (FeedForwardLayer's hidden chunks), the last one zero-padded to d rows
    const int nchunk = (F + d - 1) / d;
    w.pj_w.clear();
    for (int k = 0; k < nchunk; k++)
    {
        std::vector<double> wk((std::size_t)d * d, 0.0);
        for (int r = 0; r < d && k * d + r < F; r++)
            for (int j = 0; j < d; j++) wk[(std::size_t)r * d + j] = p.pj_w[(std::size_t)(k * d + r) * d + j];
        std::vector<Ciphertext> part;
        pack_w(wk, d, d, part);
        w.pj_w.insert(w.pj_w.end(), part.begin(), part.end());
    }
    std::vector<double> qb = p.qb, kb = p.kb, vb = p.vb, ob = p.ob, fb = p.fc_b, pb = p.pj_b;
    w.qb.clear();
    w.kb.clear();
    w.vb.clear();
    expand_bias_head_row(qb, w.qb, H, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys, T);
    expand_bias_head_row(kb, w.kb, H, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys, T);
    expand_bias_head_col(vb, w.vb, H, T, dh, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys);
    // one row-packed bias ciphertext serves every output ciphertext: the rows one ciphertext holds
    auto rows_per_ct = [&](int len) { return std::min(T, kSlots / (2 * round_to_2(len))); };
    expand_bias(ob, w.ob, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys, rows_per_ct(d));
    w.fc_b.clear();
    for (int k = 0; k < nchunk; k++)
    {
        std::vector<double> bk(d, 0.0);
        for (int j = 0; j < d && k * d + j < F; j++) bk[j] = fb[(std::size_t)(k * d + j)];
        Ciphertext cb;
        expand_bias(bk, cb, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys, rows_per_ct(d));
        w.fc_b.push_back(cb);
    }
    expand_bias(pb, w.pj_b, encoder, encryptor, decryptor, evaluator, gal_keys, relin_keys, rows_per_ct(d));
    for (auto *v : { &w.qb, &w.kb, &w.vb })
        for (auto &c : *v) drop(c);
    drop(w.ob);
    for (auto &cb : w.fc_b) drop(cb);
    drop(w.pj_b);
    w.ln1_g = p.ln1_g;
    w.ln1_b = p.ln1_b;
    w.ln2_g = p.ln2_g;
    w.ln2_b = p.ln2_b;
}

std::vector<int> block_rotation_steps(int logN)
{
    // every rotation the block makes is composed from +-2^i (SEAL's NAF path)
    std::vector<int> steps;
    const int slots = 1 << (logN - 1);
    for (int i = 0; i < logN - 1; i++)
    {
        steps.push_back(1 << i);
        steps.push_back(slots - (1 << i));
    }
    return steps;
}
} // namespace gpt2
