// random.cpp -- SEAL's randomness for the seal:: surface: OS entropy, Blake2xbPRNG and its
// factory (SEAL/randomgen.h:200-560, randomgen.cpp:23-195), and the samplers of
// SEAL/util/rlwe.cpp driven on the device (csrc/sample.hip) with the host doing only what is
// sequential: the sparse ternary secret key (rlwe.cpp:40-70) and the ordering of the few
// rejected uniform words (rlwe.cpp:148-160).
#include "random_internal.h"

#include "../../include/mhe.h"
#include "../csrc/blake2b.h"

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <sys/random.h>

namespace seal
{
// ----------------------------------------------------------------------------- OS entropy
void random_bytes(seal_byte *buf, std::size_t count)
{
    // randomgen.cpp:23-50 reads /dev/urandom through std::random_device; getrandom(2) is the
    // same kernel CSPRNG without the file descriptor
    auto *p = reinterpret_cast<unsigned char *>(buf);
    while (count)
    {
        const ssize_t got = getrandom(p, count, 0);
        if (got < 0)
        {
            if (errno == EINTR) continue;
            throw std::runtime_error("failed to read OS entropy");
        }
        p += got;
        count -= (std::size_t)got;
    }
}

// ----------------------------------------------------------------------------- Blake2xbPRNG
UniformRandomGenerator::UniformRandomGenerator(prng_seed_type seed) : seed_(seed) {}
UniformRandomGenerator::~UniformRandomGenerator()
{
    std::fill(buffer_.begin(), buffer_.end(), 0);
    std::fill(seed_.begin(), seed_.end(), 0);
}

void UniformRandomGenerator::refill_buffer()
{
    // Blake2xbPRNG::refill_buffer (randomgen.cpp:185-195): blake2xb(buffer, 4096, &counter, 8, seed, 64)
    std::uint64_t root[8], blk[8];
    b2b::xof_root(seed_.data(), counter_, b2b::kPrngBuffer, root);
    for (std::uint32_t i = 0; i < b2b::kPrngBuffer / 64; i++)
    {
        b2b::xof_block(root, i, b2b::kPrngBuffer, 64, blk);
        std::memcpy(buffer_.data() + 64 * i, blk, 64);
    }
    counter_++;
}

void UniformRandomGenerator::generate(std::size_t byte_count, seal_byte *destination)
{
    // UniformRandomGenerator::generate (randomgen.cpp:160-177), including its eager refill
    std::lock_guard<std::mutex> lock(mutex_);
    auto *dst = reinterpret_cast<unsigned char *>(destination);
    while (byte_count)
    {
        const std::size_t cur = std::min(byte_count, buffer_.size() - head_);
        std::memcpy(dst, buffer_.data() + head_, cur);
        head_ += cur;
        dst += cur;
        byte_count -= cur;
        if (head_ == buffer_.size())
        {
            refill_buffer();
            head_ = 0;
        }
    }
}

std::uint32_t UniformRandomGenerator::generate()
{
    std::uint32_t r;
    generate(sizeof(r), reinterpret_cast<seal_byte *>(&r));
    return r;
}

void UniformRandomGenerator::refresh()
{
    std::lock_guard<std::mutex> lock(mutex_);
    refill_buffer();
    head_ = 0;
}

std::shared_ptr<UniformRandomGeneratorFactory> UniformRandomGeneratorFactory::DefaultFactory()
{
    static std::shared_ptr<UniformRandomGeneratorFactory> f = std::make_shared<Blake2xbPRNGFactory>();
    return f;
}

prng_seed_type UniformRandomGeneratorFactory::next_seed() const
{
    if (!use_random_seed_) return default_seed_;
    prng_seed_type s;
    random_bytes(reinterpret_cast<seal_byte *>(s.data()), prng_seed_byte_count);
    return s;
}

namespace rnd
{
// Stream words from a byte offset (a multiple of 8) on: the tail of sample_poly_uniform.
class StreamReader
{
public:
    StreamReader(const prng_seed_type &seed, std::uint64_t byte_offset) : seed_(seed), pos_(byte_offset) {}
    std::uint64_t next()
    {
        const std::uint64_t buf = pos_ / b2b::kPrngBuffer;
        if (buf != cur_)
        {
            std::uint64_t root[8];
            b2b::xof_root(seed_.data(), buf, b2b::kPrngBuffer, root);
            for (std::uint32_t i = 0; i < b2b::kPrngBuffer / 64; i++) b2b::xof_block(root, i, b2b::kPrngBuffer, 64, words_ + 8 * i);
            cur_ = buf;
        }
        const std::uint64_t w = words_[(pos_ % b2b::kPrngBuffer) / 8];
        pos_ += 8;
        return w;
    }

private:
    prng_seed_type seed_;
    std::uint64_t pos_, cur_ = ~0ULL;
    std::uint64_t words_[b2b::kPrngBuffer / 8];
};

prng_seed_type stream_prefix_seed(const prng_seed_type &seed)
{
    // bootstrap_prng->generate(prng_seed_byte_count, public_prng_seed) (rlwe.cpp:317-318): the
    // first 64 bytes of the stream
    std::uint64_t root[8], blk[8];
    b2b::xof_root(seed.data(), 0, b2b::kPrngBuffer, root);
    b2b::xof_block(root, 0, b2b::kPrngBuffer, 64, blk);
    prng_seed_type s;
    std::copy(blk, blk + 8, s.begin());
    return s;
}

namespace
{
std::uint64_t max_multiple(std::uint64_t q)
{
    // rlwe.cpp:152: max_random - barrett_reduce_64(max_random, modulus) - 1
    return ~0ULL - (~0ULL % q) - 1;
}

void check(int rc)
{
    if (rc != MHE_OK) throw std::runtime_error(mhe_last_error());
}

struct Scratch
{
    mhe_ctx *eng;
    void *s;
    void *p = nullptr;
    Scratch(mhe_ctx *e, void *st, std::size_t bytes) : eng(e), s(st) { check(mhe_malloc_async(eng, &p, bytes, s)); }
    ~Scratch() { (void)mhe_free_async(eng, p, s); }
};
} // namespace

void sample_uniform_dev(mhe_ctx *eng, const prng_seed_type &seed, const std::vector<std::uint64_t> &moduli,
                        const std::vector<int> &prime_of_limb, const std::vector<int> &slot_of_limb, std::size_t n,
                        std::uint64_t *out, void *s)
{
    const std::size_t limbs = prime_of_limb.size();
    constexpr std::uint32_t cap = 1u << 16;
    Scratch rej(eng, s, cap * 8 + 8);
    auto *rej_list = static_cast<std::uint64_t *>(rej.p);
    auto *rej_count = reinterpret_cast<std::uint32_t *>(rej_list + cap);
    const std::uint32_t zero = 0;
    check(mhe_memcpy_h2d(eng, rej_count, &zero, 4, s));
    check(mhe_prng_uniform_bulk(eng, seed.data(), (int)limbs, prime_of_limb.data(), slot_of_limb.data(), out, rej_list,
                                rej_count, cap, s));
    std::uint32_t count = 0;
    check(mhe_memcpy_d2h(eng, &count, rej_count, 4, s));
    check(mhe_stream_sync(eng, s));
    if (count > cap) throw std::runtime_error("sample_poly_uniform: rejection list overflow");
    if (!count) return;
    std::vector<std::uint64_t> idx(count);
    check(mhe_memcpy_d2h(eng, idx.data(), rej_list, count * 8, s));
    check(mhe_stream_sync(eng, s));
    std::sort(idx.begin(), idx.end());
    // redraw in index order from the words after the bulk (rlwe.cpp:153-157)
    StreamReader tail(seed, (std::uint64_t)limbs * n * 8);
    std::vector<std::uint64_t> fixes;
    for (std::uint64_t g : idx)
    {
        const std::size_t l = g / n;
        const std::uint64_t q = moduli[prime_of_limb[l]];
        const std::uint64_t mm = max_multiple(q);
        std::uint64_t w;
        do w = tail.next();
        while (w >= mm);
        if (slot_of_limb[l] >= 0)
        {
            fixes.push_back((std::uint64_t)slot_of_limb[l] * n + (g % n));
            fixes.push_back(w % q);
        }
    }
    if (fixes.empty()) return;
    Scratch fx(eng, s, fixes.size() * 8);
    check(mhe_memcpy_h2d(eng, fx.p, fixes.data(), fixes.size() * 8, s));
    check(mhe_prng_apply_fixes(eng, static_cast<const std::uint64_t *>(fx.p), (std::uint32_t)(fixes.size() / 2), out, s));
    check(mhe_stream_sync(eng, s)); // the host fix list is temporary
}

void sample_uniform_dev(mhe_ctx *eng, const prng_seed_type &seed, const std::vector<std::uint64_t> &moduli,
                        std::size_t limbs, std::size_t n, std::uint64_t *out, void *s)
{
    std::vector<int> prime(limbs), slot(limbs);
    for (std::size_t l = 0; l < limbs; l++) prime[l] = slot[l] = (int)l;
    sample_uniform_dev(eng, seed, moduli, prime, slot, n, out, s);
}

void sample_uniform_host(mhe_ctx *eng, const prng_seed_type &seed, const std::vector<std::uint64_t> &moduli,
                         const std::vector<int> &prime_of_limb, const std::vector<int> &slot_of_limb, std::size_t n,
                         std::uint64_t *out, void *s)
{
    int kept = 0;
    for (int v : slot_of_limb) kept = std::max(kept, v + 1);
    if (!kept) return;
    Scratch dev(eng, s, (std::size_t)kept * n * 8);
    sample_uniform_dev(eng, seed, moduli, prime_of_limb, slot_of_limb, n, static_cast<std::uint64_t *>(dev.p), s);
    check(mhe_memcpy_d2h(eng, out, dev.p, (std::size_t)kept * n * 8, s));
    check(mhe_stream_sync(eng, s));
}

void sample_cbd_dev(mhe_ctx *eng, const prng_seed_type &seed, std::uint64_t byte_offset, std::size_t limbs,
                    std::uint64_t *out, void *s)
{
    check(mhe_prng_small(eng, seed.data(), byte_offset, MHE_SAMPLE_CBD, (int)limbs, out, nullptr, s));
}

// host restatements of the small samplers (the fallback when a ternary word must be redrawn)
namespace
{
void put_small(std::int64_t v, const std::vector<std::uint64_t> &moduli, std::size_t limbs, std::size_t n,
               std::size_t i, std::uint64_t *out)
{
    for (std::size_t l = 0; l < limbs; l++) out[l * n + i] = v >= 0 ? (std::uint64_t)v : moduli[l] - (std::uint64_t)(-v);
}
} // namespace

void sample_ternary_host(UniformRandomGenerator &prng, const std::vector<std::uint64_t> &moduli, std::size_t limbs,
                         std::size_t n, std::uint64_t *out)
{
    // rlwe.cpp:21-38
    RandomToStandardAdapter engine(prng);
    std::uniform_int_distribution<std::uint64_t> dist(0, 2);
    for (std::size_t i = 0; i < n; i++) put_small((std::int64_t)dist(engine) - 1, moduli, limbs, n, i, out);
}

void sample_cbd_host(UniformRandomGenerator &prng, const std::vector<std::uint64_t> &moduli, std::size_t limbs,
                     std::size_t n, std::uint64_t *out)
{
    // rlwe.cpp:101-133
    for (std::size_t i = 0; i < n; i++)
    {
        unsigned char x[6];
        prng.generate(6, reinterpret_cast<seal_byte *>(x));
        x[2] &= 0x1F;
        x[5] &= 0x1F;
        const int noise = __builtin_popcount(x[0]) + __builtin_popcount(x[1]) + __builtin_popcount(x[2]) -
                          __builtin_popcount(x[3]) - __builtin_popcount(x[4]) - __builtin_popcount(x[5]);
        put_small(noise, moduli, limbs, n, i, out);
    }
}

void sample_sparse_ternary_host(UniformRandomGenerator &prng, const std::vector<std::uint64_t> &moduli,
                                std::size_t n, std::size_t hamming_weight, std::uint64_t *out)
{
    // modified SEAL sample_poly_sparse_ternary (rlwe.cpp:40-70).  dist_non_zero_position is
    // (0, coeff_count) inclusive, so index == n can be drawn: SEAL then tests destination[n]
    // (limb 1, coefficient 0) and writes limb j+1's coefficient 0 with the value reduced for q_j
    // (not a residue of q_{j+1} when q_j > q_{j+1}, and the last write lands one word past the
    // array): the secret is then not a ring element and decryption breaks (a test saw it: hw 64 at
    // n 4096 draws n with probability 1.6 % per key).  Here a draw of n is redrawn, so keys equal
    // SEAL's for every seed whose draws never hit n (probability 1 - hw/(n+1) per key).
    const std::size_t K = moduli.size();
    std::fill(out, out + K * n, 0);
    RandomToStandardAdapter engine(prng);
    std::uniform_int_distribution<std::uint64_t> dist(0, 1), pos(0, n);
    std::size_t w = 0;
    while (w < hamming_weight)
    {
        const std::size_t index = (std::size_t)pos(engine);
        if (index >= n || out[index] != 0) continue;
        const std::uint64_t r = 2 * dist(engine);
        for (std::size_t j = 0; j < K; j++) out[index + j * n] = r == 0 ? moduli[j] - 1 : r - 1;
        w++;
    }
}
} // namespace rnd
} // namespace seal
