// seal/seal.h -- SEAL-3.6-compatible C++ surface of the MI355X engine (libmhe_seal.so).
//
// Drop-in for the subset of the modified Microsoft SEAL 3.6.6 API that the reference's
// callers use: EncryptionParameters, CoeffModulus, SEALContext (+ chain),
// Ciphertext / Plaintext, keys, KeyGenerator, CKKSEncoder, Encryptor, Decryptor and the
// Evaluator, including the modified `Evaluator(context, encoder)` constructor and the
// `*_const`, `multiply_vector*`, `*_reduced_error` methods (SEAL/evaluator.h:1186-1285).
//
// Every ciphertext operation runs on the GPU through the C ABI of include/mhe.h; polynomial
// data lives in HBM in SEAL's layout ([poly][limb][n] u64, NTT form).  Ciphertext/Plaintext
// keep a host mirror that is synchronised only when data() is touched, so the usual
// value-semantics code (copies, temporaries) never crosses PCIe.  Each calling host thread
// gets its own HIP stream (the reference calls one shared Evaluator from 50 OpenMP threads,
// cnn/infer_seal.cpp:404).
//
// Differences from SEAL, by design:
//  * randomness is SEAL's: Blake2xbPRNG seeded from OS entropy (or a factory's default seed),
//    SEAL's samplers (run on the GPU where they are parallel), so keys and encryptions are SEAL's
//    bits for the same seed;
//  * SEAL's memory pools (MemoryPoolHandle) are accepted and ignored;
//  * serialization (save/load) is not provided yet.
#pragma once

#include <atomic>
#include <algorithm>
#include <array>
#include <complex>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <iosfwd>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

struct mhe_ctx;
struct mhe_encoder;

namespace seal
{
enum class scheme_type : std::uint8_t
{
    none = 0x0,
    bfv = 0x1,
    ckks = 0x2
};

enum class sec_level_type : int
{
    none = 0,
    tc128 = 128,
    tc192 = 192,
    tc256 = 256
};

using parms_id_type = std::array<std::uint64_t, 4>;
extern const parms_id_type parms_id_zero;

using seal_byte = std::byte;

// SEAL/serialization.h: only uncompressed streams are produced and accepted (the reference builds
// SEAL with ZLIB/ZSTD off for its drivers; a compressed stream is rejected as SEAL does).
enum class compr_mode_type : std::uint8_t
{
    none = 0,
    zlib = 1,
    zstd = 2
};

class Serialization
{
public:
    static constexpr std::uint16_t seal_magic = 0xA15E;
    static constexpr std::uint8_t seal_header_size = 0x10;
    static constexpr compr_mode_type compr_mode_default = compr_mode_type::none;
    struct SEALHeader
    {
        std::uint16_t magic = seal_magic;
        std::uint8_t header_size = seal_header_size;
        std::uint8_t version_major = 3;
        std::uint8_t version_minor = 6;
        compr_mode_type compr_mode = compr_mode_type::none;
        std::uint16_t reserved = 0;
        std::uint64_t size = 0;
    };
    static_assert(sizeof(SEALHeader) == 16, "");
    static bool IsValidHeader(const SEALHeader &header) noexcept;
};

class MemoryPoolHandle
{
public:
    static MemoryPoolHandle Global() { return {}; }
    static MemoryPoolHandle New(bool = false) { return {}; }
    explicit operator bool() const noexcept { return true; }
};

class MemoryManager
{
public:
    static MemoryPoolHandle GetPool() { return {}; }
};

// Modulus (SEAL/modulus.h)
class Modulus
{
public:
    Modulus(std::uint64_t value = 0) : value_(value) {}
    std::uint64_t value() const noexcept { return value_; }
    int bit_count() const noexcept;
    bool is_zero() const noexcept { return value_ == 0; }
    bool operator==(const Modulus &o) const noexcept { return value_ == o.value_; }
    bool operator!=(const Modulus &o) const noexcept { return value_ != o.value_; }
    bool operator<(const Modulus &o) const noexcept { return value_ < o.value_; }
    bool operator<=(const Modulus &o) const noexcept { return value_ <= o.value_; }

private:
    std::uint64_t value_;
};

// CoeffModulus::Create (SEAL/modulus.cpp:143-185)
class CoeffModulus
{
public:
    static std::vector<Modulus> Create(std::size_t poly_modulus_degree, std::vector<int> bit_sizes);
    static int MaxBitCount(std::size_t poly_modulus_degree, sec_level_type sec_level = sec_level_type::tc128) noexcept;
};

// Randomness (SEAL/randomgen.h): OS entropy, the Blake2xb PRNG and its factories, as in SEAL.
constexpr std::size_t prng_seed_uint64_count = 8;
constexpr std::size_t prng_seed_byte_count = prng_seed_uint64_count * 8;
using prng_seed_type = std::array<std::uint64_t, prng_seed_uint64_count>;
enum class prng_type : std::uint8_t
{
    unknown = 0,
    blake2xb = 1,
    shake256 = 2
};

// (not SEAL API) the PRNG seeds a Serializable<T> writes in place of the second polynomial of its
// symmetric encryptions: key index -> one seed per digit (a ciphertext or public key: index 0)
using SeedMap = std::map<std::size_t, std::vector<prng_seed_type>>;

// randomgen.cpp:23-50: bytes from the kernel CSPRNG (getrandom)
void random_bytes(seal_byte *buf, std::size_t count);
inline std::uint64_t random_uint64()
{
    std::uint64_t r;
    random_bytes(reinterpret_cast<seal_byte *>(&r), sizeof(r));
    return r;
}

// Blake2xbPRNG (randomgen.h:200-270, randomgen.cpp:160-195): 4096-byte buffers, buffer c =
// BLAKE2Xb(4096 bytes, message = u64 counter c, key = the 64-byte seed)
class UniformRandomGenerator
{
public:
    explicit UniformRandomGenerator(prng_seed_type seed);
    virtual ~UniformRandomGenerator();
    prng_seed_type seed() const noexcept { return seed_; }
    prng_type type() const noexcept { return prng_type::blake2xb; }
    void generate(std::size_t byte_count, seal_byte *destination);
    std::uint32_t generate();
    void refresh();

private:
    void refill_buffer();
    prng_seed_type seed_;
    std::array<std::uint8_t, 4096> buffer_{};
    std::size_t head_ = 4096; // buffer_head_ starts at buffer_end_ (randomgen.h:224)
    std::uint64_t counter_ = 0;
    std::mutex mutex_;
};

class Blake2xbPRNG : public UniformRandomGenerator
{
public:
    using UniformRandomGenerator::UniformRandomGenerator;
};

// randomgen.h:405-470: a factory seeds every generator it creates from fresh OS entropy, or --
// constructed with a default seed, for debugging -- always with that seed.
class UniformRandomGeneratorFactory
{
public:
    UniformRandomGeneratorFactory() : use_random_seed_(true) {}
    explicit UniformRandomGeneratorFactory(prng_seed_type default_seed)
        : default_seed_(default_seed), use_random_seed_(false)
    {}
    virtual ~UniformRandomGeneratorFactory() = default;
    std::shared_ptr<UniformRandomGenerator> create() { return std::make_shared<Blake2xbPRNG>(next_seed()); }
    std::shared_ptr<UniformRandomGenerator> create(prng_seed_type seed) { return std::make_shared<Blake2xbPRNG>(seed); }
    bool use_random_seed() const noexcept { return use_random_seed_; }
    const prng_seed_type &default_seed() const noexcept { return default_seed_; }
    static std::shared_ptr<UniformRandomGeneratorFactory> DefaultFactory();
    // (not SEAL API) the seed create() gives its generator: 512 fresh bits, or the default seed
    virtual prng_seed_type next_seed() const;

private:
    prng_seed_type default_seed_{};
    bool use_random_seed_;
};

class Blake2xbPRNGFactory : public UniformRandomGeneratorFactory
{
public:
    Blake2xbPRNGFactory() = default;
    explicit Blake2xbPRNGFactory(prng_seed_type default_seed) : UniformRandomGeneratorFactory(default_seed) {}
};

// (not SEAL API) A reproducible factory for debugging runs.  Blake2xbPRNGFactory(default_seed)
// hands every generator the same seed, so every key would share its uniform polynomial and error.
// While counting, generator i gets `base` with its last word XOR-ed by i + 1: keys drawn one after
// the other are independent and the same sequence repeats from run to run.  Once frozen, create()
// gives `base` itself, SEAL's debugging behaviour, so encryptions issued by concurrent threads or
// fibers stay reproducible whatever their order.  Never for real use.
class Blake2xbSeedSequence : public UniformRandomGeneratorFactory
{
public:
    explicit Blake2xbSeedSequence(prng_seed_type base) : UniformRandomGeneratorFactory(base) {}
    prng_seed_type next_seed() const override
    {
        prng_seed_type s = default_seed();
        if (!frozen_.load()) s[prng_seed_uint64_count - 1] ^= count_.fetch_add(1) + 1;
        return s;
    }
    void freeze() { frozen_.store(true); }
    std::uint64_t generators() const { return count_.load(); }

private:
    mutable std::atomic<std::uint64_t> count_{ 0 };
    std::atomic<bool> frozen_{ false };
};

// randomtostd.h: a UniformRandomGenerator as a 32-bit standard URBG
class RandomToStandardAdapter
{
public:
    using result_type = std::uint32_t;
    explicit RandomToStandardAdapter(UniformRandomGenerator &g) : g_(&g) {}
    result_type operator()() { return g_->generate(); }
    static constexpr result_type min() noexcept { return 0; }
    static constexpr result_type max() noexcept { return 0xFFFFFFFFu; }

private:
    UniformRandomGenerator *g_;
};

// EncryptionParameters (SEAL/encryptionparams.h, with the modified hamming weight / sparse slots)
class EncryptionParameters
{
public:
    EncryptionParameters(scheme_type scheme = scheme_type::none) : scheme_(scheme) {}
    void set_poly_modulus_degree(std::size_t n) { n_ = n; }
    void set_coeff_modulus(const std::vector<Modulus> &cm) { coeff_modulus_ = cm; }
    void set_secret_key_hamming_weight(std::size_t hw) { hamming_weight_ = hw; }
    void set_sparse_slots(std::size_t s) { sparse_slots_ = s; }
    void set_random_generator(std::shared_ptr<UniformRandomGeneratorFactory> g) { rng_ = std::move(g); }
    scheme_type scheme() const noexcept { return scheme_; }
    std::size_t poly_modulus_degree() const noexcept { return n_; }
    const std::vector<Modulus> &coeff_modulus() const noexcept { return coeff_modulus_; }
    std::size_t secret_key_hamming_weight() const noexcept { return hamming_weight_; }
    std::size_t sparse_slots() const noexcept { return sparse_slots_; }
    std::shared_ptr<UniformRandomGeneratorFactory> random_generator() const { return rng_; }
    // (not SEAL API) random_generator(), or SEAL's default factory when none was set (context.cpp:464-467)
    std::shared_ptr<UniformRandomGeneratorFactory> random_generator_or_default() const
    {
        return rng_ ? rng_ : UniformRandomGeneratorFactory::DefaultFactory();
    }
    parms_id_type parms_id() const;

private:
    scheme_type scheme_;
    std::size_t n_ = 0;
    std::vector<Modulus> coeff_modulus_;
    std::size_t hamming_weight_ = 0;
    std::size_t sparse_slots_ = 0;
    std::shared_ptr<UniformRandomGeneratorFactory> rng_;
};

class Ciphertext;
class Plaintext;

// SEALContext (SEAL/context.h): the modulus switching chain
class SEALContext
{
public:
    class ContextData
    {
    public:
        const EncryptionParameters &parms() const noexcept { return parms_; }
        const parms_id_type &parms_id() const noexcept { return parms_id_; }
        std::size_t chain_index() const noexcept { return chain_index_; }
        int total_coeff_modulus_bit_count() const noexcept { return total_bits_; }
        std::shared_ptr<const ContextData> next_context_data() const noexcept { return next_.lock(); }
        std::shared_ptr<const ContextData> prev_context_data() const noexcept { return prev_.lock(); }

    private:
        friend class SEALContext;
        EncryptionParameters parms_;
        parms_id_type parms_id_{};
        std::size_t chain_index_ = 0;
        int total_bits_ = 0;
        std::weak_ptr<const ContextData> next_, prev_;
    };

    SEALContext(const EncryptionParameters &parms, bool expand_mod_chain = true,
                sec_level_type sec_level = sec_level_type::tc128);
    std::shared_ptr<const ContextData> get_context_data(const parms_id_type &id) const;
    std::shared_ptr<const ContextData> key_context_data() const;
    std::shared_ptr<const ContextData> first_context_data() const;
    std::shared_ptr<const ContextData> last_context_data() const;
    const parms_id_type &key_parms_id() const;
    const parms_id_type &first_parms_id() const;
    const parms_id_type &last_parms_id() const;
    // false when the coefficient modulus exceeds CoeffModulus::MaxBitCount for the requested
    // security level (context.cpp:207-220); keys, encoders, encryptors then refuse the context
    bool parameters_set() const noexcept;
    sec_level_type sec_level() const noexcept;
    bool using_keyswitching() const noexcept;

    // engine plumbing (not SEAL API)
    mhe_ctx *engine() const;
    void *stream() const;         // this host thread's HIP stream on the engine
    std::size_t key_size() const; // primes at the key level (data + special)
    std::shared_ptr<void> handle() const;
    static void *stream_of(void *handle);

private:
    struct Impl;
    std::shared_ptr<Impl> impl_;
};

// Device polynomial storage with a lazily synchronised host mirror.
//
// Cross-thread ordering: every access names the HIP stream it is issued on (the calling
// thread's stream).  A read waits for the last writer if that was another stream; a write waits
// for the readers and the writer on other streams.  This keeps the reference's pattern -- one
// Evaluator shared by an OpenMP team, inputs produced by one thread and consumed by others --
// correct while every thread's work stays asynchronous on its own stream.
class PolyStore
{
public:
    PolyStore() = default;
    PolyStore(const PolyStore &o);
    PolyStore &operator=(const PolyStore &o);
    PolyStore(PolyStore &&o) noexcept;
    PolyStore &operator=(PolyStore &&o) noexcept;
    ~PolyStore();

    void bind(const SEALContext &ctx);
    bool bound() const noexcept { return eng_ != nullptr; }
    // resize to `words` u64; keeps the common prefix when `preserve`
    void resize_words(std::size_t words, bool preserve = true);
    std::size_t words() const noexcept { return words_; }
    const std::uint64_t *dev_read(void *stream) const;
    std::uint64_t *dev_write(void *stream, bool overwrite = false);
    std::uint64_t *host();             // host mirror, device marked stale
    const std::uint64_t *host() const; // host mirror, device stays current
    void *thread_stream() const;       // the calling thread's stream on the bound engine
    mhe_ctx *engine() const noexcept { return eng_; }

private:
    void release();
    void wait_writer(void *stream) const;
    void wait_all(void *stream) const;
    void copy_from(const PolyStore &o);
    std::shared_ptr<void> hold_; // SEALContext::Impl: keeps the engine and its streams alive
    mhe_ctx *eng_ = nullptr;
    std::uint64_t *dev_ = nullptr;
    std::size_t words_ = 0, cap_ = 0;
    mutable std::vector<std::uint64_t> host_;
    mutable bool host_valid_ = true, dev_valid_ = true;
    mutable std::unique_ptr<std::mutex> mu_ = std::make_unique<std::mutex>();
    mutable void *writer_ = nullptr;
    mutable bool writer_done_ = true;
    mutable std::vector<void *> readers_;
};

class Ciphertext
{
public:
    Ciphertext(MemoryPoolHandle = {}) {}
    Ciphertext(const SEALContext &context, MemoryPoolHandle = {});
    Ciphertext(const SEALContext &context, parms_id_type parms_id, MemoryPoolHandle = {});

    void resize(const SEALContext &context, parms_id_type parms_id, std::size_t size);
    void resize(const SEALContext &context, std::size_t size);
    void resize(std::size_t size);
    std::size_t size() const noexcept { return size_; }
    std::size_t coeff_modulus_size() const noexcept { return coeff_modulus_size_; }
    std::size_t poly_modulus_degree() const noexcept { return poly_modulus_degree_; }
    parms_id_type &parms_id() noexcept { return parms_id_; }
    const parms_id_type &parms_id() const noexcept { return parms_id_; }
    double &scale() noexcept { return scale_; }
    double scale() const noexcept { return scale_; }
    bool &is_ntt_form() noexcept { return is_ntt_form_; }
    bool is_ntt_form() const noexcept { return is_ntt_form_; }
    bool is_transparent() const;
    std::uint64_t *data() { return store_.host(); }
    const std::uint64_t *data() const { return store_.host(); }
    std::uint64_t *data(std::size_t poly) { return store_.host() + poly * coeff_modulus_size_ * poly_modulus_degree_; }
    const std::uint64_t *data(std::size_t poly) const
    {
        return store_.host() + poly * coeff_modulus_size_ * poly_modulus_degree_;
    }
    std::size_t dyn_array_size() const noexcept { return store_.words(); }

    // SEAL/ciphertext.h save/load (byte-compatible with SEAL 3.6, compr_mode_type::none)
    std::streamoff save_size(compr_mode_type compr_mode = Serialization::compr_mode_default) const;
    std::streamoff save(std::ostream &stream, compr_mode_type compr_mode = Serialization::compr_mode_default) const;
    std::streamoff save(seal_byte *out, std::size_t size,
                        compr_mode_type compr_mode = Serialization::compr_mode_default) const;
    std::streamoff load(const SEALContext &context, std::istream &stream);
    std::streamoff load(const SEALContext &context, const seal_byte *in, std::size_t size);
    std::streamoff unsafe_load(const SEALContext &context, std::istream &stream) { return load(context, stream); }
    // (not SEAL API; Serializable) the seeded form when seeds[0] holds c1's seed: c0 only, then the
    // UniformRandomGeneratorInfo (ciphertext.cpp:148-239); load() expands it
    std::streamoff save_size_seeded(const SeedMap &seeds, compr_mode_type compr_mode) const;
    std::streamoff save_seeded(std::ostream &stream, const SeedMap &seeds, compr_mode_type compr_mode) const;

    // engine plumbing
    PolyStore &store() noexcept { return store_; }
    const PolyStore &store() const noexcept { return store_; }

private:
    PolyStore store_;
    parms_id_type parms_id_{};
    std::size_t size_ = 0, coeff_modulus_size_ = 0, poly_modulus_degree_ = 0;
    double scale_ = 1.0;
    bool is_ntt_form_ = false;
};

class Plaintext
{
public:
    Plaintext(MemoryPoolHandle = {}) {}
    std::size_t coeff_count() const noexcept { return store_.words(); }
    parms_id_type &parms_id() noexcept { return parms_id_; }
    const parms_id_type &parms_id() const noexcept { return parms_id_; }
    double &scale() noexcept { return scale_; }
    double scale() const noexcept { return scale_; }
    bool is_ntt_form() const noexcept { return parms_id_ != parms_id_zero; }
    std::uint64_t *data() { return store_.host(); }
    const std::uint64_t *data() const { return store_.host(); }
    std::uint64_t &operator[](std::size_t i) { return store_.host()[i]; }
    std::size_t limbs() const noexcept { return limbs_; }

    // SEAL/plaintext.h save/load (byte-compatible with SEAL 3.6, compr_mode_type::none)
    std::streamoff save_size(compr_mode_type compr_mode = Serialization::compr_mode_default) const;
    std::streamoff save(std::ostream &stream, compr_mode_type compr_mode = Serialization::compr_mode_default) const;
    std::streamoff save(seal_byte *out, std::size_t size,
                        compr_mode_type compr_mode = Serialization::compr_mode_default) const;
    std::streamoff load(const SEALContext &context, std::istream &stream);
    std::streamoff load(const SEALContext &context, const seal_byte *in, std::size_t size);

    // engine plumbing
    void set_level(const SEALContext &ctx, const parms_id_type &id, std::size_t limbs);
    PolyStore &store() noexcept { return store_; }
    const PolyStore &store() const noexcept { return store_; }

private:
    PolyStore store_;
    parms_id_type parms_id_ = parms_id_zero;
    double scale_ = 1.0;
    std::size_t limbs_ = 0;
};

class SecretKey
{
public:
    const Plaintext &data() const noexcept { return sk_; }
    Plaintext &data() noexcept { return sk_; }
    const parms_id_type &parms_id() const noexcept { return sk_.parms_id(); }

private:
    Plaintext sk_; // NTT form over the key level
};

class PublicKey
{
public:
    const Ciphertext &data() const noexcept { return pk_; }
    Ciphertext &data() noexcept { return pk_; }
    const parms_id_type &parms_id() const noexcept { return pk_.parms_id(); }
    // SEAL/publickey.h: the key's ciphertext in SEAL's format
    std::streamoff save(std::ostream &stream, compr_mode_type m = Serialization::compr_mode_default) const
    {
        return pk_.save(stream, m);
    }
    std::streamoff load(const SEALContext &context, std::istream &stream) { return pk_.load(context, stream); }
    std::streamoff save_size(compr_mode_type m = Serialization::compr_mode_default) const { return pk_.save_size(m); }
    std::streamoff save_size_seeded(const SeedMap &seeds, compr_mode_type m) const
    {
        return pk_.save_size_seeded(seeds, m);
    }
    std::streamoff save_seeded(std::ostream &stream, const SeedMap &seeds, compr_mode_type m) const
    {
        return pk_.save_seeded(stream, seeds, m);
    }

private:
    Ciphertext pk_;
};

// KSwitchKeys (SEAL/kswitchkeys.h): one device buffer [digits][2][key_limbs][n] per key index.
//
// Keys are SEAL's: KeyGenerator draws them with SEAL's randomness and the evaluator owns no
// secret.  Level-truncated keys (MI355X memory budget): the reference's ResNet driver asks for
// 284 Galois keys at the key level, 284 x 1.04 GB = 295 GB, more than one GPU's 288 GB HBM, yet
// most are only used at <= 3 limbs, where the key switch reads L digits over L+1 primes
// (SEAL/evaluator.cpp:2345-2371).  KeyGenerator::create_galois_keys(elt_limbs) stores, per element,
// SEAL's key restricted to the digits and primes its level needs (stored limbs = limbs_of(i)); a
// ciphertext above that level is refused.  Client side only, opt-in:
// KeyGenerator::create_deferred_galois_keys gives a key provider that keeps the secret key and
// materialises each key on first use at the level of that use; usage() then reports the levels,
// from which the client makes the truncated set the server holds.  Deferred keys cannot be saved.
struct KeyMaker;
class KSwitchKeys
{
public:
    std::size_t size() const;
    const parms_id_type &parms_id() const noexcept { return parms_id_; }
    parms_id_type &parms_id() noexcept { return parms_id_; }
    bool has_index(std::size_t i) const;
    const PolyStore &key(std::size_t i) const;
    PolyStore &key_mut(std::size_t i) { return keys_[i]; }
    std::size_t key_limbs() const noexcept { return key_limbs_; }
    void set_key_limbs(std::size_t k) { key_limbs_ = k; }
    // stored limbs of key i (digits + 1): key_limbs() for a full key
    std::size_t limbs_of(std::size_t i) const;
    void insert(std::size_t index, PolyStore &&key, std::size_t limbs);
    // device key for index i usable by an L-limb ciphertext (a deferred key is materialised on
    // demand, thread-safe); key_limbs receives the key's limb stride
    const std::uint64_t *key_for(std::size_t i, std::size_t L, void *stream, std::size_t &key_limbs) const;
    bool deferred() const noexcept { return maker_ != nullptr; }
    void set_maker(std::shared_ptr<KeyMaker> m) { maker_ = std::move(m); }
    const std::shared_ptr<KeyMaker> &maker() const noexcept { return maker_; }
    // index -> stored limbs of every materialised key (for a deferred set: the levels it was used at)
    std::map<std::size_t, std::size_t> usage() const;
    // bytes of device memory held by materialised keys
    std::size_t device_bytes() const;

    // SEAL/kswitchkeys.cpp:42-140 byte format: parms_id | u64 dim1 | per index: u64 dim2 | dim2
    // PublicKey (Ciphertext) objects at the key level.  Truncated keys are written with their
    // stored primes; deferred key providers are not serialisable.
    std::streamoff save_size(compr_mode_type compr_mode = Serialization::compr_mode_default) const;
    std::streamoff save(std::ostream &stream, compr_mode_type compr_mode = Serialization::compr_mode_default) const;
    std::streamoff load(const SEALContext &context, std::istream &stream);
    // (not SEAL API; Serializable) every PublicKey record whose index has seeds written seeded
    std::streamoff save_size_seeded(const SeedMap &seeds, compr_mode_type compr_mode) const;
    std::streamoff save_seeded(std::ostream &stream, const SeedMap &seeds, compr_mode_type compr_mode) const;

private:
    mutable std::map<std::size_t, PolyStore> keys_;
    mutable std::map<std::size_t, std::size_t> limbs_of_; // stored limbs per index
    mutable std::vector<PolyStore> retired_;               // outgrown deferred keys (may be in flight)
    parms_id_type parms_id_ = parms_id_zero;
    std::size_t key_limbs_ = 0;
    std::shared_ptr<KeyMaker> maker_;
};

class RelinKeys : public KSwitchKeys
{
public:
    static std::size_t get_index(std::size_t key_power) { return key_power - 2; } // relinkeys.h:58
    bool has_key(std::size_t key_power) const { return has_index(get_index(key_power)); }
};

class GaloisKeys : public KSwitchKeys
{
public:
    static std::size_t get_index(std::uint32_t galois_elt) { return (galois_elt - 1) >> 1; } // galoiskeys.h:48
    bool has_key(std::uint32_t galois_elt) const { return has_index(get_index(galois_elt)); }
};

// Serializable<T> (SEAL/serializable.h): what SEAL's seeded creators return -- create_public_key(),
// create_relin_keys(), create_galois_keys(...), Encryptor::encrypt_symmetric(plain) /
// encrypt_zero_symmetric() -- an object that can only be saved.  The second polynomial of every
// symmetric encryption of zero inside it is written as the seed of the Blake2xb PRNG that drew it
// (SEAL: seed marker in c1, ciphertext.cpp:183-239), halving the bytes; T::load expands the seed into
// the same words (ciphertext.cpp:305-335).  encrypt(plain) carries no seed and saves in full.
template <class T>
class Serializable
{
public:
    std::streamoff save_size(compr_mode_type compr_mode = Serialization::compr_mode_default) const
    {
        return obj_.save_size_seeded(seeds_, compr_mode);
    }
    std::streamoff save(std::ostream &stream, compr_mode_type compr_mode = Serialization::compr_mode_default) const
    {
        return obj_.save_seeded(stream, seeds_, compr_mode);
    }
    std::streamoff save(seal_byte *out, std::size_t size,
                        compr_mode_type compr_mode = Serialization::compr_mode_default) const
    {
        const std::streamoff need = save_size(compr_mode);
        if (!out || (std::streamoff)size < need) throw std::invalid_argument("insufficient size");
        std::ostringstream ss(std::ios::binary);
        save(ss, compr_mode);
        const std::string b = ss.str();
        std::copy(b.begin(), b.end(), reinterpret_cast<char *>(out));
        return (std::streamoff)b.size();
    }

private:
    friend class KeyGenerator;
    friend class Encryptor;
    Serializable(T obj, SeedMap seeds) : obj_(std::move(obj)), seeds_(std::move(seeds)) {}
    T obj_;
    SeedMap seeds_;
};

class KeyGenerator
{
public:
    explicit KeyGenerator(const SEALContext &context);
    KeyGenerator(const SEALContext &context, const SecretKey &secret_key);
    const SecretKey &secret_key() const { return sk_; }
    void create_public_key(PublicKey &destination);
    // keygenerator.h:83-135, 250-310: the seeded forms, only for saving
    Serializable<PublicKey> create_public_key();
    void create_relin_keys(RelinKeys &destination);
    Serializable<RelinKeys> create_relin_keys();
    void create_galois_keys(const std::vector<int> &steps, GaloisKeys &destination);
    Serializable<GaloisKeys> create_galois_keys(const std::vector<int> &steps);
    void create_galois_keys(GaloisKeys &destination);
    Serializable<GaloisKeys> create_galois_keys();
    void create_galois_keys_from_elts(const std::vector<std::uint32_t> &elts, GaloisKeys &destination);
    // (not SEAL API) SEAL's Galois keys truncated per element to the ciphertext level (limbs) it
    // will be used at: digits min(limbs, K-1), primes q_0..q_{digits-1} and P (see KSwitchKeys)
    void create_galois_keys(const std::vector<std::pair<std::uint32_t, std::size_t>> &elt_limbs,
                            GaloisKeys &destination);
    // (not SEAL API) client-side deferred key provider (see KSwitchKeys): holds the secret key
    void create_deferred_galois_keys(const std::vector<int> &steps, GaloisKeys &destination);
    void create_deferred_galois_keys(GaloisKeys &destination);
    void create_deferred_galois_keys_from_elts(const std::vector<std::uint32_t> &elts, GaloisKeys &destination);
    // (not SEAL API) a deferred provider of the +-2^i rotation keys (i < log2(n/2)), made once per
    // generator: rotations by any step through SEAL's NAF decomposition (evaluator.cpp:2244-2276)
    const GaloisKeys &power_of_two_keys();

private:
    // seeds (optional) receives each digit's public seed (the PRNG seed of its c1)
    void kswitch_key(const std::uint64_t *new_key_dev, PolyStore &dest, std::size_t digits,
                     std::vector<prng_seed_type> *seeds = nullptr);
    void relin_keys_into(RelinKeys &destination, SeedMap *seeds);
    void galois_keys_into(const std::vector<std::uint32_t> &elts, GaloisKeys &destination, SeedMap *seeds);
    SEALContext ctx_;
    SecretKey sk_;
    std::shared_ptr<UniformRandomGeneratorFactory> rng_;
    std::shared_ptr<GaloisKeys> pow2_;
    std::shared_ptr<std::mutex> pow2_mu_ = std::make_shared<std::mutex>();
};

class CKKSEncoder
{
public:
    explicit CKKSEncoder(const SEALContext &context);
    ~CKKSEncoder();
    std::size_t slot_count() const noexcept { return slots_; }
    const mhe_encoder *handle() const noexcept { return enc_; } // engine plumbing
    void set_sparse_slots(std::size_t sparse_slots) { sparse_slots_ = sparse_slots; }
    void encode(const std::vector<double> &values, parms_id_type parms_id, double scale, Plaintext &destination,
                MemoryPoolHandle = {});
    void encode(const std::vector<std::complex<double>> &values, parms_id_type parms_id, double scale,
                Plaintext &destination, MemoryPoolHandle = {});
    void encode(const std::vector<double> &values, double scale, Plaintext &destination, MemoryPoolHandle = {});
    void encode(const std::vector<std::complex<double>> &values, double scale, Plaintext &destination,
                MemoryPoolHandle = {});
    void encode(double value, parms_id_type parms_id, double scale, Plaintext &destination, MemoryPoolHandle = {});
    void encode(double value, double scale, Plaintext &destination, MemoryPoolHandle = {});
    void decode(const Plaintext &plain, std::vector<double> &destination, MemoryPoolHandle = {});
    void decode(const Plaintext &plain, std::vector<std::complex<double>> &destination, MemoryPoolHandle = {});

private:
    void encode_internal(const double *re, const double *im, std::size_t count, parms_id_type parms_id,
                         double scale, Plaintext &destination);
    void decode_internal(const Plaintext &plain, std::vector<std::complex<double>> &out);
    SEALContext ctx_;
    mhe_encoder *enc_ = nullptr;
    std::size_t slots_ = 0, sparse_slots_ = 0;
    std::vector<std::size_t> index_map_;
    std::vector<std::complex<double>> root_powers_;
};

class Encryptor
{
public:
    Encryptor(const SEALContext &context, const PublicKey &public_key);
    Encryptor(const SEALContext &context, const SecretKey &secret_key);
    Encryptor(const SEALContext &context, const PublicKey &public_key, const SecretKey &secret_key);
    void set_public_key(const PublicKey &public_key);
    void set_secret_key(const SecretKey &secret_key);
    // encryptor.h:130-420: encrypt / encrypt_zero use the public key when one is set (else the
    // secret key, as this library's secret-key-only Encryptor always has); the *_symmetric forms
    // use the secret key; the Serializable forms are for saving (seeded when symmetric)
    void encrypt(const Plaintext &plain, Ciphertext &destination, MemoryPoolHandle = {}) const;
    Serializable<Ciphertext> encrypt(const Plaintext &plain, MemoryPoolHandle = {}) const;
    void encrypt_zero(Ciphertext &destination, MemoryPoolHandle = {}) const;
    void encrypt_zero(parms_id_type parms_id, Ciphertext &destination, MemoryPoolHandle = {}) const;
    void encrypt_symmetric(const Plaintext &plain, Ciphertext &destination, MemoryPoolHandle = {}) const;
    Serializable<Ciphertext> encrypt_symmetric(const Plaintext &plain, MemoryPoolHandle = {}) const;
    void encrypt_zero_symmetric(Ciphertext &destination, MemoryPoolHandle = {}) const;
    void encrypt_zero_symmetric(parms_id_type parms_id, Ciphertext &destination, MemoryPoolHandle = {}) const;
    Serializable<Ciphertext> encrypt_zero_symmetric(MemoryPoolHandle = {}) const;
    Serializable<Ciphertext> encrypt_zero_symmetric(parms_id_type parms_id, MemoryPoolHandle = {}) const;

private:
    // symmetric: secret key; public_seed (symmetric only) receives c1's PRNG seed
    void encrypt_zero_at(std::size_t limbs, Ciphertext &dest, bool symmetric,
                         prng_seed_type *public_seed = nullptr) const;
    void encrypt_plain(const Plaintext &plain, Ciphertext &destination, bool symmetric,
                       prng_seed_type *public_seed) const;
    void zero_at(parms_id_type parms_id, Ciphertext &destination, bool symmetric, prng_seed_type *public_seed) const;
    SEALContext ctx_;
    PublicKey pk_;
    SecretKey sk_;
    bool asymmetric_;
    bool has_sk_ = false;
    std::shared_ptr<UniformRandomGeneratorFactory> rng_;
};

class Decryptor
{
public:
    Decryptor(const SEALContext &context, const SecretKey &secret_key);
    void decrypt(const Ciphertext &encrypted, Plaintext &destination);

private:
    SEALContext ctx_;
    SecretKey sk_;
};

// (not SEAL API) Batched launches of the *_many / rotate_vectors calls, on by default.  Off, every
// entry runs as its own call (the words are the same either way: tests compare the two).
void set_batched_launches(bool on);
bool batched_launches();

// (not SEAL API) How many merged Lockstep / FiberBatch calls failed and were re-run member by
// member (Evaluator::lockstep_execute), process-wide; reset: return the count and start from 0.
// A healthy run reports 0: the engine's allocation retries and failures are in mhe_alloc_stats.
std::uint64_t merged_call_fallbacks(bool reset = false);

// (not SEAL API) True when `addr` lies in the guard page below a live seal::FiberBatch fiber stack
// (a stack overflow).  Reads a lock-free list, so a SIGSEGV handler may call it; FiberBatch::run
// gives its thread an alternate signal stack for handlers installed with SA_ONSTACK.
bool fiber_stack_guard(const void *addr);

// (not SEAL API) Lockstep: threads that evaluate the same operation sequence on different data (the
// images of a batch) join one group.  While joined, every top-level rotation (rotate_vector[s],
// rotate_vector_inplace), relinearization (relinearize_inplace, and the one inside
// multiply_[inplace_]reduced_error) and rescale_to_next_inplace of a member waits for the
// same-numbered call of every other member, and all of them run as one batched launch sequence on
// one stream: entries of one rotation key together, so k_ks_row_mac reads each key once for all
// members, and at low levels one launch fills the chip that one image's could not.  Results are
// word for word those of the unbatched calls.  A member that leaves (scope end, exception) is no
// longer waited for; calls whose kinds differ within a round run one by one.
struct LsOp;
// (not SEAL API) FiberBatch: the same merging as Lockstep, but the members are fibers on the calling
// host thread instead of threads: run(count, work) runs work(0) .. work(count - 1) as fibers that
// switch only at the merge points (rotations, relinearizations, reduced-error products, rescales),
// so every round is collected without thread wake-ups, and every member's kernels -- merged or not
// -- go to the calling thread's one stream, in order, with no cross-stream waits.  Exceptions are
// per fiber; the first one is rethrown once every fiber has finished.
class FiberBatch
{
public:
    struct Impl;
    static void run(std::size_t count, const std::function<void(std::size_t)> &work,
                    std::size_t stack_bytes = (std::size_t)8 << 20);
    static std::size_t last_rounds();  // merged rounds of the calling thread's last run()
    static std::size_t last_merged();  // member calls those rounds merged
    // index of the fiber running on the calling thread, -1 outside a FiberBatch (state that the
    // reference keeps per thread must be kept per fiber: the fibers of a thread interleave)
    static long current();
};
class Lockstep
{
public:
    struct Impl;
    explicit Lockstep(std::size_t members);
    ~Lockstep();
    Lockstep(const Lockstep &) = delete;
    Lockstep &operator=(const Lockstep &) = delete;
    // RAII membership of the calling thread; an inactive member's calls run directly except inside
    // an Active scope (all members must open and close their Active scopes at the same points of
    // their operation sequences)
    class Member
    {
    public:
        explicit Member(Lockstep &group, bool active = true);
        ~Member();
        Member(const Member &) = delete;
        Member &operator=(const Member &) = delete;

    private:
        Lockstep &g_;
    };
    // merge the calling member's operations for this scope (no-op outside a group)
    class Active
    {
    public:
        Active();
        ~Active();
        Active(const Active &) = delete;
        Active &operator=(const Active &) = delete;

    private:
        Impl *saved_;
    };
    std::size_t rounds() const;        // batched rounds run so far
    std::size_t merged_calls() const;  // member calls that ran inside a merged round

private:
    std::unique_ptr<Impl> impl_;
};

class Evaluator
{
public:
    Evaluator(const SEALContext &context, CKKSEncoder &encoder);

    void negate_inplace(Ciphertext &encrypted) const;
    void negate(const Ciphertext &encrypted, Ciphertext &destination) const;
    void add_inplace(Ciphertext &encrypted1, const Ciphertext &encrypted2) const;
    void add(const Ciphertext &encrypted1, const Ciphertext &encrypted2, Ciphertext &destination) const;
    void add_many(const std::vector<Ciphertext> &encrypteds, Ciphertext &destination) const;
    void sub_inplace(Ciphertext &encrypted1, const Ciphertext &encrypted2) const;
    void sub(const Ciphertext &encrypted1, const Ciphertext &encrypted2, Ciphertext &destination) const;
    void multiply_inplace(Ciphertext &encrypted1, const Ciphertext &encrypted2, MemoryPoolHandle = {}) const;
    void multiply_many(const std::vector<Ciphertext> &encrypteds, const RelinKeys &relin_keys,
                       Ciphertext &destination, MemoryPoolHandle = {}) const;
    void exponentiate_inplace(Ciphertext &encrypted, std::uint64_t exponent, const RelinKeys &relin_keys,
                              MemoryPoolHandle = {}) const;
    void multiply(const Ciphertext &encrypted1, const Ciphertext &encrypted2, Ciphertext &destination,
                  MemoryPoolHandle = {}) const;
    void square_inplace(Ciphertext &encrypted, MemoryPoolHandle = {}) const;
    void square(const Ciphertext &encrypted, Ciphertext &destination, MemoryPoolHandle = {}) const;
    void relinearize_inplace(Ciphertext &encrypted, const RelinKeys &relin_keys, MemoryPoolHandle = {}) const;
    void relinearize(const Ciphertext &encrypted, const RelinKeys &relin_keys, Ciphertext &destination,
                     MemoryPoolHandle = {}) const;
    void mod_switch_to_next_inplace(Ciphertext &encrypted, MemoryPoolHandle = {}) const;
    void mod_switch_to_next(const Ciphertext &encrypted, Ciphertext &destination, MemoryPoolHandle = {}) const;
    void mod_switch_to_next_inplace(Plaintext &plain) const;
    void mod_switch_to_inplace(Ciphertext &encrypted, parms_id_type parms_id, MemoryPoolHandle = {}) const;
    void mod_switch_to(const Ciphertext &encrypted, parms_id_type parms_id, Ciphertext &destination,
                       MemoryPoolHandle = {}) const;
    void mod_switch_to_inplace(Plaintext &plain, parms_id_type parms_id) const;
    void rescale_to_next_inplace(Ciphertext &encrypted, MemoryPoolHandle = {}) const;
    void rescale_to_next(const Ciphertext &encrypted, Ciphertext &destination, MemoryPoolHandle = {}) const;
    void rescale_to_inplace(Ciphertext &encrypted, parms_id_type parms_id, MemoryPoolHandle = {}) const;
    void multiply_plain_inplace(Ciphertext &encrypted, const Plaintext &plain, MemoryPoolHandle = {}) const;
    void multiply_plain(const Ciphertext &encrypted, const Plaintext &plain, Ciphertext &destination,
                        MemoryPoolHandle = {}) const;
    void add_plain_inplace(Ciphertext &encrypted, const Plaintext &plain) const;
    void add_plain(const Ciphertext &encrypted, const Plaintext &plain, Ciphertext &destination) const;
    void sub_plain_inplace(Ciphertext &encrypted, const Plaintext &plain) const;
    void sub_plain(const Ciphertext &encrypted, const Plaintext &plain, Ciphertext &destination) const;
    void transform_to_ntt_inplace(Ciphertext &encrypted) const;
    void transform_from_ntt_inplace(Ciphertext &encrypted) const;
    void apply_galois_inplace(Ciphertext &encrypted, std::uint32_t galois_elt, const GaloisKeys &galois_keys,
                              MemoryPoolHandle = {}) const;
    void rotate_vector_inplace(Ciphertext &encrypted, int steps, const GaloisKeys &galois_keys,
                               MemoryPoolHandle = {}) const;
    // (not SEAL API) apply_galois reading encrypted, writing destination (no copy)
    void apply_galois_to(const Ciphertext &encrypted, std::uint32_t galois_elt, const GaloisKeys &galois_keys,
                         Ciphertext &destination) const;
    void rotate_vector(const Ciphertext &encrypted, int steps, const GaloisKeys &galois_keys,
                       Ciphertext &destination, MemoryPoolHandle = {}) const;
    // (not SEAL API) independent rotations in batched launches: *destinations[i] =
    // rotate_vector(*encrypted[i], steps[i]) for every i, bit-identical to the one-by-one calls.
    // Entries of one level with a key present run together (mhe_apply_galois_batch); a zero step,
    // a missing key (NAF decomposition) or a lone level falls back to rotate_vector.  Destinations
    // must be distinct objects, none of them an input.
    void rotate_vectors(const std::vector<const Ciphertext *> &encrypted, const std::vector<int> &steps,
                        const GaloisKeys &galois_keys, const std::vector<Ciphertext *> &destinations) const;
    // (not SEAL API) rescale_to_next_inplace of independent ciphertexts in batched launches
    void rescale_to_next_inplace_many(const std::vector<Ciphertext *> &encrypted) const;
    // (not SEAL API) relinearize_inplace of independent size-3 ciphertexts: entries of one level run
    // their key switches as one batched launch (mhe_switch_key_batch), bit-identical
    void relinearize_inplace_many(const std::vector<Ciphertext *> &encrypted, const RelinKeys &relin_keys) const;
    // (not SEAL API) *destinations[i] = multiply_reduced_error(*encrypted1[i], *encrypted2[i]) for
    // every i, the relinearizations batched (relinearize_inplace_many); destinations distinct and
    // none of them an input
    void multiply_reduced_error_many(const std::vector<const Ciphertext *> &encrypted1,
                                     const std::vector<const Ciphertext *> &encrypted2, const RelinKeys &relin_keys,
                                     const std::vector<Ciphertext *> &destinations) const;
    void complex_conjugate_inplace(Ciphertext &encrypted, const GaloisKeys &galois_keys, MemoryPoolHandle = {}) const;
    void complex_conjugate(const Ciphertext &encrypted, const GaloisKeys &galois_keys, Ciphertext &destination,
                           MemoryPoolHandle = {}) const;

    // modified SEAL (evaluator.h:1186-1285)
    void add_const_inplace(Ciphertext &encrypted, double value) const;
    void add_const(const Ciphertext &encrypted, double value, Ciphertext &destination) const;
    void multiply_const_inplace(Ciphertext &encrypted, double value) const;
    void multiply_const(const Ciphertext &encrypted, double value, Ciphertext &destination) const;
    template <typename T>
    void multiply_vector_inplace(Ciphertext &encrypted, const std::vector<T> &value) const;
    // (not SEAL API) the plaintext multiply_vector_inplace multiplies by: value encoded at the
    // first level with scale encrypted.scale(), kept at the ciphertext's level
    template <typename T>
    void encode_vector_for(const Ciphertext &encrypted, const std::vector<T> &value, Plaintext &plain) const;
    template <typename T>
    void multiply_vector(Ciphertext &encrypted, const std::vector<T> &value, Ciphertext &destination) const
    {
        Plaintext plain;
        encode_vector_for(encrypted, value, plain);
        multiply_plain(encrypted, plain, destination);
    }
    void add_inplace_reduced_error(Ciphertext &encrypted1, const Ciphertext &encrypted2) const;
    // (not SEAL API) multiply_plain(encrypted, plain, t) + add_inplace_reduced_error(acc, t) for acc at
    // encrypted's level, fused into one pass with bit-identical output
    void multiply_plain_add_reduced_error(Ciphertext &acc, const Ciphertext &encrypted, const Plaintext &plain) const;
    // (not SEAL API) multiply_plain(encrypted[0], plain[0], destination), then
    // multiply_plain_add_reduced_error(destination, encrypted[k], plain[k]) for k = 1, 2, ... (all at one
    // level and size): the same words and scale, one pass per 16 terms (mhe_multiply_plain_sum)
    void multiply_plain_sum(const std::vector<const Ciphertext *> &encrypted, const std::vector<const Plaintext *> &plain,
                            Ciphertext &destination) const;
    void add_reduced_error(const Ciphertext &encrypted1, const Ciphertext &encrypted2, Ciphertext &destination) const
    {
        // evaluator.h: operands swap when destination aliases encrypted2
        if (&encrypted2 == &destination)
            add_inplace_reduced_error(destination, encrypted1);
        else
            reduced_error_out(encrypted1, encrypted2, destination, Rmode::add, nullptr);
    }
    void double_inplace(Ciphertext &encrypted) const { add_inplace(encrypted, encrypted); }
    void sub_inplace_reduced_error(Ciphertext &encrypted1, const Ciphertext &encrypted2) const;
    void sub_reduced_error(const Ciphertext &encrypted1, const Ciphertext &encrypted2, Ciphertext &destination) const
    {
        // As the modified SEAL (evaluator.h): with destination aliasing encrypted2 the result is
        // encrypted2 - encrypted1.  Kept for drop-in equality of results.
        if (&encrypted2 == &destination)
            sub_inplace_reduced_error(destination, encrypted1);
        else
            reduced_error_out(encrypted1, encrypted2, destination, Rmode::sub, nullptr);
    }
    void multiply_inplace_reduced_error(Ciphertext &encrypted1, const Ciphertext &encrypted2,
                                        const RelinKeys &relin_keys) const;
    void multiply_reduced_error(const Ciphertext &encrypted1, const Ciphertext &encrypted2,
                                const RelinKeys &relin_keys, Ciphertext &destination) const
    {
        if (&encrypted2 == &destination)
            multiply_inplace_reduced_error(destination, encrypted1, relin_keys);
        else
            reduced_error_out(encrypted1, encrypted2, destination, Rmode::mul, &relin_keys);
    }
    template <typename T>
    void multiply_vector_inplace_reduced_error(Ciphertext &encrypted, const std::vector<T> &value)
    {
        multiply_vector_inplace(encrypted, value);
    }
    template <typename T>
    void multiply_vector_reduced_error(Ciphertext &encrypted, const std::vector<T> &value, Ciphertext &destination)
    {
        // copy + multiply_vector_inplace in SEAL; the product written straight to destination here
        Plaintext plain;
        encode_vector_for(encrypted, value, plain);
        multiply_plain(encrypted, plain, destination);
    }

    // (not SEAL API) encode_vector_for of static operands (network weights, masks), cached: the
    // caller names the vector by a 128-bit recipe id (a hash of everything that determines it) and
    // make() builds it on a miss only.  Entries are keyed by (id, level, scale), are bit-identical
    // to a fresh encode_vector_for, and live as long as the evaluator (and its copies).  Returns the
    // cached plaintext, or `scratch` holding a fresh encoding when the cache is full or off
    // (MHE_VEC_CACHE_GB, default 48; 0 disables).
    const Plaintext &cached_vector_plain(const Ciphertext &encrypted, std::uint64_t id_hi, std::uint64_t id_lo,
                                         const std::function<std::vector<double>()> &make, Plaintext &scratch) const;
    std::size_t vector_cache_entries() const;
    std::size_t vector_cache_bytes() const;

private:
    enum class Rmode
    {
        add,
        sub,
        mul
    };
    void reduced_error_op(Ciphertext &encrypted1, const Ciphertext &encrypted2, Rmode mode) const;
    // destination = encrypted1 (op)_reduced_error encrypted2 without the copy of encrypted1 when the
    // levels match (the copy + in-place op of the modified SEAL, same words)
    void reduced_error_out(const Ciphertext &encrypted1, const Ciphertext &encrypted2, Ciphertext &destination,
                           Rmode mode, const RelinKeys *relin_keys) const;
    void switch_key(Ciphertext &encrypted, const std::uint64_t *target_dev, const KSwitchKeys &keys,
                    std::size_t index) const;
    void rotate_internal(Ciphertext &encrypted, int steps, const GaloisKeys &galois_keys) const;
    // Lockstep: hand `op` to the calling thread's group (false: no group, run it directly)
    bool lockstep_submit(LsOp &op) const;
    friend struct Lockstep::Impl;
    friend class FiberBatch;
    void lockstep_execute(std::vector<LsOp *> &ops) const;
    std::size_t limbs_of(const parms_id_type &id) const;
    SEALContext context_;
    CKKSEncoder &encoder_;
    struct VecCache;
    std::shared_ptr<VecCache> vcache_;
};

extern template void Evaluator::multiply_vector_inplace<double>(Ciphertext &, const std::vector<double> &) const;
extern template void Evaluator::multiply_vector_inplace<std::complex<double>>(
    Ciphertext &, const std::vector<std::complex<double>> &) const;
// seal::util::iter -- the iterator helpers the reference's bootstrapper uses for coefficient access
// (modraise_inplace, BOOT/Bootstrapper.cpp:2894-2948; SEAL/util/iterator.h): iter(ciphertext)[poly]
// [limb][coeff] over the host mirror (non-const access marks the device copy stale, so the next GPU
// operation uploads it), iter(plaintext)[limb][coeff], and iter(coeff_modulus)[j].
namespace util
{
template <class T>
class CoeffIterT
{
public:
    explicit CoeffIterT(T *p) : p_(p) {}
    T &operator[](std::size_t i) const { return p_[i]; }
    T *ptr() const noexcept { return p_; }
    operator T *() const noexcept { return p_; }

private:
    T *p_;
};
template <class T>
class RNSIterT
{
public:
    RNSIterT(T *p, std::size_t n) : p_(p), n_(n) {}
    CoeffIterT<T> operator[](std::size_t limb) const { return CoeffIterT<T>(p_ + limb * n_); }
    std::size_t poly_modulus_degree() const noexcept { return n_; }

private:
    T *p_;
    std::size_t n_;
};
template <class T>
class PolyIterT
{
public:
    PolyIterT(T *p, std::size_t n, std::size_t limbs) : p_(p), n_(n), limbs_(limbs) {}
    RNSIterT<T> operator[](std::size_t poly) const { return RNSIterT<T>(p_ + poly * limbs_ * n_, n_); }
    std::size_t coeff_modulus_size() const noexcept { return limbs_; }

private:
    T *p_;
    std::size_t n_, limbs_;
};
using CoeffIter = CoeffIterT<std::uint64_t>;
using ConstCoeffIter = CoeffIterT<const std::uint64_t>;
using RNSIter = RNSIterT<std::uint64_t>;
using ConstRNSIter = RNSIterT<const std::uint64_t>;
using PolyIter = PolyIterT<std::uint64_t>;
using ConstPolyIter = PolyIterT<const std::uint64_t>;

inline PolyIter iter(Ciphertext &c)
{
    return PolyIter(c.data(), c.poly_modulus_degree(), c.coeff_modulus_size());
}
inline ConstPolyIter iter(const Ciphertext &c)
{
    return ConstPolyIter(c.data(), c.poly_modulus_degree(), c.coeff_modulus_size());
}
inline const std::vector<Modulus> &iter(const std::vector<Modulus> &coeff_modulus) { return coeff_modulus; }
} // namespace util
} // namespace seal
