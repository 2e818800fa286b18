// cnn.cpp -- multiplexed-packing CNN layers (include/mhe_cnn.h) over the seal:: surface.
//
// The reference's layers (cnn_ckks/cpu-ckks/single-key/cnn/cnn_seal.cpp) are host loops that
// build plaintext masks/weights and issue rotations, multiply_vector, add and rescale on one
// ciphertext.  Here the same operation sequence runs on the GPU engine; the host work (mask and
// weight vectors) is computed once per call as in the reference.  Packing (Lee et al.,
// "multiplexed parallel convolution"): slot s of a TensorCipher (k, h, w, c, t, p) is copy
// s / (n/p); inside a copy, local index = k^2*h*w*u + k*w*R + C encodes channel
// k^2*u + k*(R%k) + C%k at pixel (R/k, C/k).
#include "mhe_cnn.h"

#include <cmath>
#include <cstring>
#include <functional>
#include <iostream>
#include <stdexcept>

using namespace seal;

long pow2(long n)
{
    return 1L << n;
}

int floor_to_int(double x)
{
    return static_cast<int>(std::floor(x) + 0.5);
}

long log2_long(long n)
{
    // -1 unless n is a power of two in [1, 65536] (common/MinicompFunc.cpp:37-46)
    if (n > 65536 || n <= 0) throw std::out_of_range("n is too large.");
    for (int i = 0; i <= 16; i++)
        if ((1L << i) == n) return i;
    return -1;
}

namespace
{
// Slot decomposition of the multiplexed layout (cnn_seal.cpp:359-360, 551-552, 601-603).
struct Mux
{
    long n;
    int k, h, w, t, p;
    long copy_len() const { return n / p; }
    struct Slot
    {
        long copy;    // which of the p replicas
        long local;   // index inside the replica
        int u;        // channel group
        int rb, cb;   // multiplexed row / column (k*h x k*w grid)
        int channel;  // k^2*u + k*(rb%k) + cb%k
        int row, col; // pixel
    };
    Slot at(long s) const
    {
        Slot r;
        r.copy = s / copy_len();
        r.local = s % copy_len();
        const long plane = (long)k * k * h * w;
        r.u = (int)(r.local / plane);
        const long rem = r.local % plane;
        r.rb = (int)(rem / ((long)k * w));
        r.cb = (int)(rem % ((long)k * w));
        r.channel = k * k * r.u + k * (r.rb % k) + r.cb % k;
        r.row = r.rb / k;
        r.col = r.cb / k;
        return r;
    }
    bool in_tensor(const Slot &r) const { return r.local < (long)k * k * h * w * t; }
};

// 128-bit id of a static plaintext operand (Evaluator::cached_vector_plain): two independent
// 64-bit hashes (FNV-1a and a splitmix64 chain) over everything the vector is built from.
struct Recipe
{
    std::uint64_t a = 0xcbf29ce484222325ull, b = 0x243f6a8885a308d3ull;
    Recipe &add(std::uint64_t x)
    {
        for (int i = 0; i < 8; i++) a = (a ^ ((x >> (8 * i)) & 0xff)) * 0x100000001b3ull;
        std::uint64_t z = (b ^ x) + 0x9e3779b97f4a7c15ull;
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        b = z ^ (z >> 31);
        return *this;
    }
    Recipe &add(double d)
    {
        std::uint64_t x;
        std::memcpy(&x, &d, sizeof x);
        return add(x);
    }
    Recipe &add(const std::vector<double> &v)
    {
        add((std::uint64_t)v.size());
        for (double d : v) add(d);
        return *this;
    }
    Recipe &ints(std::initializer_list<long> xs)
    {
        for (long x : xs) add((std::uint64_t)x);
        return *this;
    }
};

// multiply_vector_inplace(_reduced_error)(ct, make()) with the encoded vector cached under `id`
void multiply_static_vector(Evaluator &evaluator, Ciphertext &ct, const Recipe &id,
                            const std::function<std::vector<double>()> &make)
{
    Plaintext scratch;
    const Plaintext &pt = evaluator.cached_vector_plain(ct, id.a, id.b, make, scratch);
    evaluator.multiply_plain_inplace(ct, pt);
}
} // namespace

// ------------------------------------------------------------------------ TensorCipher
TensorCipher::TensorCipher() = default;

TensorCipher::TensorCipher(int logn, int k, int h, int w, int c, int t, int p, std::vector<double> data,
                           Encryptor &encryptor, CKKSEncoder &encoder, int logp)
    : k_(k), h_(h), w_(w), c_(c), t_(t), p_(p), logn_(logn)
{
    // cnn_seal.cpp:12-48
    if (k != 1) throw std::invalid_argument("supported k is only 1 right now");
    if (logn < 1 || logn > 16) throw std::out_of_range("the value of logn is out of range");
    if (data.size() > static_cast<std::size_t>(1L << logn)) throw std::out_of_range("the size of data is larger than n");
    data.resize(static_cast<std::size_t>(1L << logn), 0.0); // zero padding to n slots
    Plaintext plain;
    encoder.encode(data, std::pow(2.0, logp), plain);
    encryptor.encrypt(plain, cipher_);
}

TensorCipher::TensorCipher(int logn, int k, int h, int w, int c, int t, int p, Ciphertext cipher)
    : k_(k), h_(h), w_(w), c_(c), t_(t), p_(p), logn_(logn), cipher_(std::move(cipher))
{}

void TensorCipher::print_parms()
{
    std::cout << "k: " << k_ << "\nh: " << h_ << "\nw: " << w_ << "\nc: " << c_ << "\nt: " << t_ << "\np: " << p_
              << std::endl;
}

// ------------------------------------------------------------------------ rotations
void memory_save_rotate(const Ciphertext &cipher_in, Ciphertext &cipher_out, int steps, Evaluator &evaluator,
                        GaloisKeys &gal_keys)
{
    // cnn_seal.cpp:788-809: steps in 34..55 and 57..61 go through a first rotation by 33 (the
    // key set of infer_seal.cpp lacks them); a zero rotation leaves cipher_out untouched.
    const long slots = static_cast<long>(cipher_in.poly_modulus_degree() / 2);
    const long s = (steps + slots) % slots; // C++ remainder, as the reference: 0..slots-1 for steps >= -slots
    if (s == 0) return;
    Ciphertext temp; // out-of-place rotations: no copy of cipher_in
    const bool split = (s >= 34 && s <= 55) || (s >= 57 && s <= 61);
    if (split)
    {
        evaluator.rotate_vector(cipher_in, 33, gal_keys, temp);
        evaluator.rotate_vector_inplace(temp, static_cast<int>(s - 33), gal_keys);
    }
    else
        evaluator.rotate_vector(cipher_in, static_cast<int>(s), gal_keys, temp);
    cipher_out = std::move(temp);
}

namespace
{
// `out = in; memory_save_rotate(out, out, steps)` without the copy when the rotation is not zero
void rotate_copy(const Ciphertext &in, Ciphertext &out, int steps, Evaluator &evaluator, GaloisKeys &gal_keys)
{
    const long slots = static_cast<long>(in.poly_modulus_degree() / 2);
    if ((steps + slots) % slots == 0)
        out = in;
    else
        memory_save_rotate(in, out, steps, evaluator, gal_keys);
}

// rotate_copy(*ins[i], *outs[i], steps[i]) for every i, the independent rotations in batched
// launches (Evaluator::rotate_vectors): first every rotation by s (or by 33 for
// memory_save_rotate's split steps), then the second rotation of the split ones -- the same words
// as the one-by-one calls.  outs must be distinct and not inputs, except an out that is its own
// input with a zero step.
void rotate_copies(const std::vector<const Ciphertext *> &ins, const std::vector<int> &steps,
                   const std::vector<Ciphertext *> &outs, Evaluator &evaluator, GaloisKeys &gal_keys)
{
    if (ins.empty()) return;
    const long slots = static_cast<long>(ins[0]->poly_modulus_degree() / 2);
    std::vector<Ciphertext> mid(steps.size());
    std::vector<const Ciphertext *> in1, in2;
    std::vector<int> st1, st2;
    std::vector<Ciphertext *> out1, out2;
    for (std::size_t i = 0; i < steps.size(); i++)
    {
        const long s = (steps[i] + slots) % slots;
        if (s == 0) continue;
        const bool split = (s >= 34 && s <= 55) || (s >= 57 && s <= 61);
        in1.push_back(ins[i]);
        st1.push_back(split ? 33 : static_cast<int>(s));
        out1.push_back(split ? &mid[i] : outs[i]);
        if (split)
        {
            in2.push_back(&mid[i]);
            st2.push_back(static_cast<int>(s - 33));
            out2.push_back(outs[i]);
        }
    }
    evaluator.rotate_vectors(in1, st1, gal_keys, out1);
    if (!in2.empty()) evaluator.rotate_vectors(in2, st2, gal_keys, out2);
    for (std::size_t i = 0; i < steps.size(); i++)
        if ((steps[i] + slots) % slots == 0 && outs[i] != ins[i]) *outs[i] = *ins[i];
}

void rotate_copies(const Ciphertext &in, const std::vector<int> &steps, const std::vector<Ciphertext *> &outs,
                   Evaluator &evaluator, GaloisKeys &gal_keys)
{
    rotate_copies(std::vector<const Ciphertext *>(steps.size(), &in), steps, outs, evaluator, gal_keys);
}
} // namespace

// ------------------------------------------------------------------------ convolution
void multiplexed_parallel_convolution_seal(const TensorCipher &cnn_in, TensorCipher &cnn_out, int co, int st, int fh,
                                           int fw, const std::vector<double> &data, std::vector<double> running_var,
                                           std::vector<double> constant_weight, double epsilon, CKKSEncoder &encoder,
                                           Encryptor &encryptor, Evaluator &evaluator, GaloisKeys &gal_keys,
                                           std::vector<Ciphertext> &cipher_pool, bool end)
{
    // cnn_seal.cpp:284-530
    const int ki = cnn_in.k(), hi = cnn_in.h(), wi = cnn_in.w(), ci = cnn_in.c(), ti = cnn_in.t(), pi = cnn_in.p(),
              logn = cnn_in.logn();
    if (st != 1 && st != 2) throw std::invalid_argument("supported st is only 1 or 2");
    if (static_cast<int>(data.size()) != fh * fw * ci * co)
        throw std::invalid_argument("the size of data vector is not ker x ker x h x h");
    if (log2_long(ki) == -1) throw std::invalid_argument("ki is not power of two");
    if (static_cast<int>(running_var.size()) != co || static_cast<int>(constant_weight.size()) != co)
        throw std::invalid_argument("the size of running_var or weight is not correct");
    for (double v : running_var)
        if (v < 1e-16 && v > -1e-16) throw std::invalid_argument("the size of running_var is too small. nearly zero.");
    if (fh % 2 == 0 || fw % 2 == 0) throw std::invalid_argument("fh and fw should be odd");
    int ho = hi, wo = wi, ko = ki;
    if (st == 2)
    {
        if (hi % 2 == 1 || wi % 2 == 1) throw std::invalid_argument("hi or wi is not even");
        ho = hi / 2;
        wo = wi / 2;
        ko = 2 * ki;
    }
    const long n = 1L << logn;
    const int to = (co + ko * ko - 1) / (ko * ko);
    const int po = static_cast<int>(
        pow2(floor_to_int(std::log(static_cast<double>(n) / static_cast<double>(ko * ko * ho * wo * to)) / std::log(2.0))));
    const int q = (co + pi - 1) / pi;
    if (n % pi != 0) throw std::out_of_range("n is not divisible by pi");
    if (n % po != 0) throw std::out_of_range("n is not divisible by po");
    if ((long)ki * ki * hi * wi * ti * pi > n) throw std::out_of_range("ki^2 hi wi ti pi is larger than n");
    if ((long)ko * ko * ho * wo * to * po > n) throw std::out_of_range("ko^2 ho wo to po is larger than n");

    // kernel tap (i1, i2), input channel a, output channel b: data[((b*ci + a)*fh + i1)*fw + i2]
    auto tap = [&](int i1, int i2, int a, int b) { return data[((size_t)(b * ci + a) * fh + i1) * fw + i2]; };
    const Mux in{ n, ki, hi, wi, ti, pi };
    const int ch = (fh - 1) / 2, cw = (fw - 1) / 2;

    // weights of output-channel block i9 for tap (i1, i2): slot of replica i8 carries output
    // channel i8 + pi*i9 (cnn_seal.cpp:350-368)
    auto weight_vec = [&](int i1, int i2, int i9) {
        std::vector<double> v(n, 0.0);
        for (long s = 0; s < n; s++)
        {
            const Mux::Slot r = in.at(s);
            const int out_ch = static_cast<int>(r.copy) + pi * i9;
            const int y = r.row - ch + i1, x = r.col - cw + i2;
            if (!in.in_tensor(r) || out_ch >= co || r.channel >= ci || y < 0 || y > hi - 1 || x < 0 || x > wi - 1)
                continue;
            v[s] = tap(i1, i2, r.channel, out_ch);
        }
        return v;
    };
    // per output channel: BN-folded scale at the slots that hold that channel after the
    // channel sum (cnn_seal.cpp:370-397)
    auto select_vec = [&](int j4) {
        std::vector<double> v(n, 0.0);
        const double g = constant_weight[j4] / std::sqrt(running_var[j4] + epsilon);
        for (int u3 = 0; u3 < to; u3++)
            for (int v1 = 0; v1 < ko * ho; v1++)
                for (int v2 = 0; v2 < ko * wo; v2++)
                    if (ko * ko * u3 + ko * (v1 % ko) + v2 % ko == j4) v[(size_t)ko * ko * ho * wo * u3 + ko * wo * v1 + v2] = g;
        return v;
    };

    if (cipher_pool.size() < static_cast<size_t>(6 + fh * fw - 1)) cipher_pool.resize(6 + fh * fw - 1);
    Ciphertext &ctxt_in = cipher_pool[0], &ct_zero = cipher_pool[1], &sum = cipher_pool[3],
               &total_sum = cipher_pool[4], &var = cipher_pool[5];
    ctxt_in = cnn_in.cipher();

    // the fh*fw shifted copies of the input (centre tap is the input itself)
    std::vector<Ciphertext *> rot((size_t)fh * fw);
    for (int i1 = 0; i1 < fh; i1++)
        for (int i2 = 0; i2 < fw; i2++)
        {
            const int idx = fw * i1 + i2, centre = fw * ch + cw;
            rot[idx] = idx == centre ? &ctxt_in : &cipher_pool[6 + (idx > centre ? idx - 1 : idx)];
        }
    {
        // the fh*fw - 1 input rotations are independent: batched launches
        std::vector<int> steps;
        for (int i1 = 0; i1 < fh; i1++)
            for (int i2 = 0; i2 < fw; i2++) steps.push_back(ki * ki * wi * (i1 - ch) + ki * (i2 - cw));
        rotate_copies(ctxt_in, steps, rot, evaluator, gal_keys);
    }

    // encryption of zero at the input scale (cnn_seal.cpp:423-427)
    {
        Plaintext plain;
        encoder.encode(std::vector<double>(n, 0.0), ctxt_in.scale(), plain);
        encryptor.encrypt(plain, ct_zero);
    }

    // the tap weights and select vectors are static: their encodings are cached by the evaluator
    // under a hash of what they are built from (bit-identical to encoding them per call)
    Recipe conv_id;
    conv_id.add((std::uint64_t)0x636f6e76u).add(data).ints({ ki, hi, wi, ci, ti, pi, logn, co, st, fh, fw });
    Recipe sel_id;
    sel_id.add((std::uint64_t)0x73656c63u).add(constant_weight).add(running_var).add(epsilon).ints(
        { ko, ho, wo, to, n });

    const int d = static_cast<int>(log2_long(ki)), c = static_cast<int>(log2_long(ti));
    // The q output-channel blocks i9 are independent until they are summed into total_sum, and
    // each runs the same operation sequence (cnn_seal.cpp:435-493): they advance together, so each
    // step -- the rescale of the tap sum, every channel-fold rotation (one key for all blocks), the
    // gathering rotations -- is one batched launch over the blocks.  Every ciphertext sees the
    // reference's operations in the reference's order, and total_sum is accumulated in (i9, i8)
    // order, so the words are those of the block-by-block loop.
    std::vector<Ciphertext> sums(q), vars(q), tmps(q);
    std::vector<Ciphertext *> sp(q), vp(q), tp(q);
    std::vector<const Ciphertext *> vc(q);
    for (int i9 = 0; i9 < q; i9++)
    {
        sp[i9] = &sums[i9];
        vp[i9] = &vars[i9];
        tp[i9] = &tmps[i9];
        vc[i9] = &vars[i9];
        // filter taps: multiply_vector_reduced_error + add_inplace_reduced_error over the fh x fw taps,
        // every product and the sum in one pass (Evaluator::multiply_plain_sum; bit-identical, every
        // tap is at the input's level)
        std::vector<Plaintext> scratch((size_t)fh * fw);
        std::vector<const Ciphertext *> taps;
        std::vector<const Plaintext *> wps;
        for (int i1 = 0; i1 < fh; i1++)
            for (int i2 = 0; i2 < fw; i2++)
            {
                const Ciphertext &tap = *rot[fw * i1 + i2];
                Recipe id = conv_id;
                id.ints({ i1, i2, i9 });
                wps.push_back(&evaluator.cached_vector_plain(tap, id.a, id.b, [&] { return weight_vec(i1, i2, i9); },
                                                              scratch[(size_t)fw * i1 + i2]));
                taps.push_back(&tap);
            }
        evaluator.multiply_plain_sum(taps, wps, sums[i9]);
    }
    evaluator.rescale_to_next_inplace_many(sp);
    for (int i9 = 0; i9 < q; i9++) vars[i9] = std::move(sums[i9]);

    // sum over the input channels held in one replica
    auto fold = [&](long step) {
        rotate_copies(vc, std::vector<int>(q, static_cast<int>(step)), tp, evaluator, gal_keys);
        for (int i9 = 0; i9 < q; i9++) evaluator.add_inplace_reduced_error(vars[i9], tmps[i9]);
    };
    for (int x = 0; x < d; x++) fold(pow2(x));
    for (int x = 0; x < d; x++) fold(pow2(x) * ki * wi);
    if (c == -1)
    {
        std::vector<std::vector<Ciphertext>> parts(q, std::vector<Ciphertext>(ti));
        std::vector<const Ciphertext *> pin;
        std::vector<Ciphertext *> pout;
        std::vector<int> steps;
        for (int i9 = 0; i9 < q; i9++)
            for (int x = 0; x < ti; x++)
            {
                pin.push_back(&vars[i9]);
                pout.push_back(&parts[i9][x]);
                steps.push_back(ki * ki * hi * wi * x);
            }
        rotate_copies(pin, steps, pout, evaluator, gal_keys);
        for (int i9 = 0; i9 < q; i9++)
        {
            Ciphertext acc = ct_zero;
            for (int x = 0; x < ti; x++) evaluator.add_inplace_reduced_error(acc, parts[i9][x]);
            vars[i9] = std::move(acc);
        }
    }
    else
        for (int x = 0; x < c; x++) fold(pow2(x) * ki * ki * hi * wi);

    // gather each output channel into its slots of the output layout (the rotations of every block
    // are independent: batched launches, then the products and sums in the reference's order)
    std::vector<std::vector<Ciphertext>> gathered(q, std::vector<Ciphertext>(pi));
    {
        std::vector<const Ciphertext *> gin;
        std::vector<Ciphertext *> gp;
        std::vector<int> gsteps;
        for (int i9 = 0; i9 < q; i9++)
            for (int i8 = 0; i8 < pi && pi * i9 + i8 < co; i8++)
            {
                const int j4 = pi * i9 + i8;
                gin.push_back(&vars[i9]);
                gp.push_back(&gathered[i9][i8]);
                gsteps.push_back((int)((n / pi) * (j4 % pi) - j4 % ko - (j4 / (ko * ko)) * ko * ko * ho * wo -
                                       ((j4 % (ko * ko)) / ko) * ko * wo));
            }
        rotate_copies(gin, gsteps, gp, evaluator, gal_keys);
    }
    for (int i9 = 0; i9 < q; i9++)
        for (int i8 = 0; i8 < pi && pi * i9 + i8 < co; i8++)
        {
            const int j4 = pi * i9 + i8;
            Ciphertext &g = gathered[i9][i8];
            Recipe id = sel_id;
            id.ints({ j4 });
            multiply_static_vector(evaluator, g, id, [&] { return select_vec(j4); });
            if (i8 == 0 && i9 == 0)
                total_sum = std::move(g);
            else
                evaluator.add_inplace_reduced_error(total_sum, g);
        }
    gathered.clear();
    evaluator.rescale_to_next_inplace(total_sum);
    var = std::move(total_sum);

    // po replicas of the output
    if (!end)
    {
        sum = ct_zero;
        std::vector<Ciphertext> reps(po);
        std::vector<Ciphertext *> rp;
        std::vector<int> rsteps;
        for (int u6 = 0; u6 < po; u6++)
        {
            rp.push_back(&reps[u6]);
            rsteps.push_back(static_cast<int>(-u6 * (n / po)));
        }
        rotate_copies(var, rsteps, rp, evaluator, gal_keys);
        for (int u6 = 0; u6 < po; u6++) evaluator.add_inplace_reduced_error(sum, reps[u6]);
        var = std::move(sum);
    }
    cnn_out = TensorCipher(logn, ko, ho, wo, co, to, po, std::move(var));
}

// ------------------------------------------------------------------------ batch norm
void multiplexed_parallel_batch_norm_seal(const TensorCipher &cnn_in, TensorCipher &cnn_out, std::vector<double> bias,
                                          std::vector<double> running_mean, std::vector<double> running_var,
                                          std::vector<double> weight, double epsilon, CKKSEncoder &encoder,
                                          Encryptor &encryptor, Evaluator &evaluator, double B, bool)
{
    // cnn_seal.cpp:531-576: subtract the encrypted per-channel offset (mean*w/sqrt(var+eps) - bias)/B
    // (the multiplicative part is folded into the preceding convolution's select vector)
    const int ki = cnn_in.k(), hi = cnn_in.h(), wi = cnn_in.w(), ci = cnn_in.c(), ti = cnn_in.t(), pi = cnn_in.p(),
              logn = cnn_in.logn();
    if (static_cast<int>(bias.size()) != ci || static_cast<int>(running_mean.size()) != ci ||
        static_cast<int>(running_var.size()) != ci || static_cast<int>(weight.size()) != ci)
        throw std::invalid_argument("the size of bias, running_mean, running_var, or weight are not correct");
    for (double v : running_var)
        if (v < 1e-16 && v > -1e-16) throw std::invalid_argument("the size of running_var is too small. nearly zero.");
    if ((long)hi * wi * ci > (1L << logn)) throw std::invalid_argument("hi*wi*ci should not be larger than n");
    const long n = 1L << logn;
    if (n % pi != 0) throw std::out_of_range("n is not divisible by pi");
    const Mux in{ n, ki, hi, wi, ti, pi };
    std::vector<double> g(n, 0.0);
    for (long s = 0; s < n; s++)
    {
        const Mux::Slot r = in.at(s);
        if (r.channel >= ci || !in.in_tensor(r)) continue;
        const int i = r.channel;
        g[s] = (running_mean[i] * weight[i] / std::sqrt(running_var[i] + epsilon) - bias[i]) / B;
    }
    Ciphertext temp = cnn_in.cipher(), cipher_g;
    Plaintext plain;
    encoder.encode(g, temp.scale(), plain);
    encryptor.encrypt(plain, cipher_g);
    evaluator.sub_inplace_reduced_error(temp, cipher_g);
    cnn_out = TensorCipher(logn, ki, hi, wi, ci, ti, pi, std::move(temp));
}

// ------------------------------------------------------------------------ ReLU
void ReLU_seal(const TensorCipher &cnn_in, TensorCipher &cnn_out, long comp_no, std::vector<int> deg, long alpha,
               std::vector<Tree> &tree, double scaled_val, long scalingfactor, Encryptor &encryptor,
               Evaluator &evaluator, Decryptor &decryptor, CKKSEncoder &encoder, PublicKey &public_key,
               SecretKey &secret_key, RelinKeys &relin_keys, double)
{
    // cnn_seal.cpp:577-592
    if ((long)cnn_in.h() * cnn_in.w() * cnn_in.c() > (1L << cnn_in.logn()))
        throw std::invalid_argument("hi*wi*ci should not be larger than n");
    Ciphertext temp = cnn_in.cipher();
    minimax_ReLU_seal(comp_no, deg, alpha, tree, scaled_val, scalingfactor, encryptor, evaluator, decryptor, encoder,
                      public_key, secret_key, relin_keys, temp, temp);
    cnn_out = TensorCipher(cnn_in.logn(), cnn_in.k(), cnn_in.h(), cnn_in.w(), cnn_in.c(), cnn_in.t(), cnn_in.p(), std::move(temp));
}

// ------------------------------------------------------------------------ residual add
void cnn_add_seal(const TensorCipher &cnn1, const TensorCipher &cnn2, TensorCipher &destination, Evaluator &evaluator)
{
    // cnn_seal.cpp:593-609
    if (cnn1.k() != cnn2.k() || cnn1.h() != cnn2.h() || cnn1.w() != cnn2.w() || cnn1.c() != cnn2.c() ||
        cnn1.t() != cnn2.t() || cnn1.p() != cnn2.p() || cnn1.logn() != cnn2.logn())
        throw std::invalid_argument("the parameters of cnn1 and cnn2 are not the same");
    Ciphertext a = cnn1.cipher();
    const Ciphertext b = cnn2.cipher();
    evaluator.add_inplace_reduced_error(a, b);
    destination = TensorCipher(cnn1.logn(), cnn1.k(), cnn1.h(), cnn1.w(), cnn1.c(), cnn1.t(), cnn1.p(), std::move(a));
}

// ------------------------------------------------------------------------ downsampling
void multiplexed_parallel_downsampling_seal(const TensorCipher &cnn_in, TensorCipher &cnn_out, Evaluator &evaluator,
                                            GaloisKeys &gal_keys)
{
    // cnn_seal.cpp:610-679: keep even pixels, re-multiplex into gap 2k with half the height/width
    const int ki = cnn_in.k(), hi = cnn_in.h(), wi = cnn_in.w(), ci = cnn_in.c(), ti = cnn_in.t(), logn = cnn_in.logn();
    const long n = 1L << logn;
    const int ko = 2 * ki, ho = hi / 2, wo = wi / 2, to = ti / 2, co = 2 * ci;
    const int po = static_cast<int>(
        pow2(floor_to_int(std::log(static_cast<double>(n) / static_cast<double>(ko * ko * ho * wo * to)) / std::log(2.0))));
    if (ti % 8 != 0) throw std::invalid_argument("ti is not multiple of 8");
    if (hi % 2 != 0) throw std::invalid_argument("hi is not even");
    if (wi % 2 != 0) throw std::invalid_argument("wi is not even");
    if (n % po != 0) throw std::out_of_range("n is not divisible by po");
    const Mux in{ n, ki, hi, wi, ti, 1 };
    const Ciphertext ct = cnn_in.cipher();
    Ciphertext sum, temp;
    // the ki*ti select products, then their (independent) rotations in batched launches, then the
    // sum in the reference's order
    std::vector<Ciphertext> prod((size_t)ki * ti), rotd((size_t)ki * ti);
    std::vector<const Ciphertext *> pin;
    std::vector<Ciphertext *> pout;
    std::vector<int> psteps;
    for (int w1 = 0; w1 < ki; w1++)
        for (int w2 = 0; w2 < ti; w2++)
        {
            auto make_sel = [&] {
                std::vector<double> sel(n, 0.0);
                for (long s = 0; s < (long)ki * ki * hi * wi * ti; s++)
                {
                    const Mux::Slot r = in.at(s);
                    if (r.row % 2 == 0 && r.col % 2 == 0 && r.rb % ki == w1 && r.u == w2) sel[s] = 1.0;
                }
                return sel;
            };
            Recipe id;
            id.add((std::uint64_t)0x646f776eu).ints({ n, ki, hi, wi, ti, w1, w2 });
            Ciphertext &pr = prod[(size_t)w1 * ti + w2];
            pr = ct;
            multiply_static_vector(evaluator, pr, id, make_sel);
            const int w3 = ((ki * w2 + w1) % (2 * ko)) / 2, w4 = (ki * w2 + w1) % 2, w5 = (ki * w2 + w1) / (2 * ko);
            pin.push_back(&pr);
            pout.push_back(&rotd[(size_t)w1 * ti + w2]);
            psteps.push_back(ki * ki * hi * wi * w2 + ki * wi * w1 - ko * ko * ho * wo * w5 - ko * wo * w3 - ki * w4 -
                             ko * ko * ho * wo * (ti / 8));
        }
    rotate_copies(pin, psteps, pout, evaluator, gal_keys);
    for (std::size_t k = 0; k < rotd.size(); k++)
    {
        if (k == 0)
            sum = rotd[k];
        else
            evaluator.add_inplace_reduced_error(sum, rotd[k]);
    }
    evaluator.rescale_to_next_inplace(sum);
    const Ciphertext packed = sum;
    {
        std::vector<Ciphertext> reps(po > 1 ? po - 1 : 0);
        std::vector<Ciphertext *> rp;
        std::vector<int> rsteps;
        for (int u6 = 1; u6 < po; u6++)
        {
            rp.push_back(&reps[u6 - 1]);
            rsteps.push_back(static_cast<int>(-(n / po) * u6));
        }
        rotate_copies(packed, rsteps, rp, evaluator, gal_keys);
        for (auto &r : reps) evaluator.add_inplace_reduced_error(sum, r);
    }
    cnn_out = TensorCipher(logn, ko, ho, wo, co, to, po, std::move(sum));
}

// ------------------------------------------------------------------------ average pooling
void averagepooling_seal_scale(const TensorCipher &cnn_in, TensorCipher &cnn_out, Evaluator &evaluator,
                               GaloisKeys &gal_keys, double B, CKKSEncoder &, Decryptor &, std::ofstream &)
{
    // cnn_seal.cpp:680-746: sum the h*w pixels of every channel, then gather channel means
    // (times B) into consecutive slots
    const int ki = cnn_in.k(), hi = cnn_in.h(), wi = cnn_in.w(), ci = cnn_in.c(), ti = cnn_in.t(), logn = cnn_in.logn();
    if (log2_long(hi) == -1) throw std::invalid_argument("hi is not power of two");
    if (log2_long(wi) == -1) throw std::invalid_argument("wi is not power of two");
    const long n = 1L << logn;
    Ciphertext ct = cnn_in.cipher(), temp, sum;
    for (int x = 0; x < log2_long(wi); x++)
    {
        rotate_copy(ct, temp, static_cast<int>(pow2(x) * ki), evaluator, gal_keys);
        evaluator.add_inplace_reduced_error(ct, temp);
    }
    for (int x = 0; x < log2_long(hi); x++)
    {
        rotate_copy(ct, temp, static_cast<int>(pow2(x) * ki * ki * wi), evaluator, gal_keys);
        evaluator.add_inplace_reduced_error(ct, temp);
    }
    std::vector<Ciphertext> gath((size_t)ki * ti);
    {
        std::vector<Ciphertext *> gp;
        std::vector<int> gs;
        for (int s = 0; s < ki; s++)
            for (int u = 0; u < ti; u++)
            {
                gp.push_back(&gath[(size_t)s * ti + u]);
                gs.push_back(-(ki * u + s) * ki + ki * ki * hi * wi * u + ki * wi * s);
            }
        rotate_copies(ct, gs, gp, evaluator, gal_keys);
    }
    for (int s = 0; s < ki; s++)
        for (int u = 0; u < ti; u++)
        {
            Ciphertext &temp = gath[(size_t)s * ti + u];
            Recipe id;
            id.add((std::uint64_t)0x61766770u).add(B).ints({ n, ki, hi, wi, u, s });
            multiply_static_vector(evaluator, temp, id, [&] {
                std::vector<double> sel(n, 0.0);
                for (int i = 0; i < ki; i++) sel[(size_t)(ki * u + s) * ki + i] = B / static_cast<double>(hi * wi);
                return sel;
            });
            if (u == 0 && s == 0)
                sum = temp;
            else
                evaluator.add_inplace_reduced_error(sum, temp);
        }
    evaluator.rescale_to_next_inplace(sum);
    cnn_out = TensorCipher(logn, 1, 1, 1, ci, ti, 1, std::move(sum));
}

// ------------------------------------------------------------------------ fully connected
void matrix_multiplication_seal(const TensorCipher &cnn_in, TensorCipher &cnn_out, std::vector<double> matrix,
                                std::vector<double> bias, int q, int r, Evaluator &evaluator, GaloisKeys &gal_keys)
{
    // cnn_seal.cpp:747-787: diagonal method, q x r matrix over the first r slots
    if (static_cast<int>(matrix.size()) != q * r) throw std::invalid_argument("the size of matrix is not q*r");
    if (static_cast<int>(bias.size()) != q) throw std::invalid_argument("the size of bias is not q");
    const long n = 1L << cnn_in.logn();
    // diagonal s of the matrix: diag[i] = matrix[i][i + s - (r - 1)] (cached encodings)
    Recipe fc_id;
    fc_id.add((std::uint64_t)0x66636d6du).add(matrix).ints({ n, q, r });
    const Ciphertext ct = cnn_in.cipher();
    Ciphertext sum;
    std::vector<Ciphertext> rots((size_t)(q + r - 1));
    {
        std::vector<Ciphertext *> rp;
        std::vector<int> rs;
        for (int s = 0; s < q + r - 1; s++)
        {
            rp.push_back(&rots[s]);
            rs.push_back(r - 1 - s);
        }
        rotate_copies(ct, rs, rp, evaluator, gal_keys);
    }
    for (int s = 0; s < q + r - 1; s++)
    {
        Ciphertext &temp = rots[s];
        Recipe id = fc_id;
        id.ints({ s });
        multiply_static_vector(evaluator, temp, id, [&] {
            std::vector<double> diag(n, 0.0);
            for (int i = 0; i < q; i++)
            {
                const int j = i + r - 1 - s;
                if (j >= 0 && j < r) diag[i] = matrix[(size_t)i * r + j];
            }
            return diag;
        });
        if (s == 0)
            sum = temp;
        else
            evaluator.add_inplace_reduced_error(sum, temp);
    }
    evaluator.rescale_to_next_inplace(sum);
    cnn_out = TensorCipher(cnn_in.logn(), cnn_in.k(), cnn_in.h(), cnn_in.w(), cnn_in.c(), cnn_in.t(), cnn_in.p(), std::move(sum));
}
