// serialize.cpp -- SEAL 3.6 byte format for Ciphertext / Plaintext and SEAL's parms_id hash.
//
// Formats (SEAL/serialization.h:60-120, SEAL/ciphertext.cpp:183-345, SEAL/plaintext.cpp:204-300,
// SEAL/dynarray.h:652-720):
//   object    = SEALHeader(16 B: magic 0xA15E, header size 0x10, version 3.6, compr mode, 0, total
//               size in bytes incl. the header) + members
//   Ciphertext members = parms_id (4 x u64) | is_ntt_form (1 byte) | size u64 | poly_modulus_degree
//               u64 | coeff_modulus_size u64 | scale f64 | DynArray
//   Plaintext members  = parms_id | coeff_count u64 | scale f64 | DynArray
//   DynArray  = SEALHeader + element count u64 + elements (u64, [poly][limb][n])
// Only compr_mode_type::none is written or accepted.
//
// Seeded objects (Serializable<T>: encrypt_symmetric, create_public_key(), create_relin_keys(),
// create_galois_keys(...)): a size-2 ciphertext written with only c0 in its DynArray, followed by a
// UniformRandomGeneratorInfo (SEALHeader + prng_type byte + 64-byte seed, randomgen.cpp:99-121) --
// ciphertext.cpp:148-239; on load a DynArray of exactly n * L words means "seeded" and c1 is
// sample_poly_uniform(Blake2xbPRNG(seed)) over the ciphertext's primes (ciphertext.cpp:305-335,
// rlwe.cpp:133-162).  A key's PublicKey records are seeded the same way, per digit.
//
// parms_id (SEAL/encryptionparams.cpp:124-158, util/hash.h:30-37) is BLAKE2b with a 32-byte digest
// over the u64 words [scheme, poly_modulus_degree, coeff moduli..., plain modulus (0 for CKKS)].
// BLAKE2b itself follows RFC 7693 (12 rounds, SHA-512 IV, no key).
#include "seal/seal.h"

#include "random_internal.h"

#include <cstring>
#include <istream>
#include <ostream>
#include <sstream>

namespace seal
{
namespace
{
// ----------------------------------------------------------------------- BLAKE2b (RFC 7693)
constexpr std::uint64_t kIV[8] = { 0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                   0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                   0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL };
constexpr std::uint8_t kSigma[12][16] = {
    { 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15 }, { 14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3 },
    { 11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4 }, { 7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8 },
    { 9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13 }, { 2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9 },
    { 12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11 }, { 13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10 },
    { 6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5 }, { 10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0 },
    { 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15 }, { 14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3 },
};

inline std::uint64_t rotr(std::uint64_t x, int r) { return (x >> r) | (x << (64 - r)); }

void blake2b_compress(std::uint64_t h[8], const std::uint8_t block[128], std::uint64_t t, bool last)
{
    std::uint64_t m[16], v[16];
    std::memcpy(m, block, 128); // little-endian host (x86-64 / gfx950 hosts)
    for (int i = 0; i < 8; i++)
    {
        v[i] = h[i];
        v[i + 8] = kIV[i];
    }
    v[12] ^= t; // the byte counter never exceeds 2^64 here
    if (last) v[14] = ~v[14];
    auto G = [&](int a, int b, int c, int d, std::uint64_t x, std::uint64_t y) {
        v[a] = v[a] + v[b] + x;
        v[d] = rotr(v[d] ^ v[a], 32);
        v[c] = v[c] + v[d];
        v[b] = rotr(v[b] ^ v[c], 24);
        v[a] = v[a] + v[b] + y;
        v[d] = rotr(v[d] ^ v[a], 16);
        v[c] = v[c] + v[d];
        v[b] = rotr(v[b] ^ v[c], 63);
    };
    for (int r = 0; r < 12; r++)
    {
        const std::uint8_t *s = kSigma[r];
        G(0, 4, 8, 12, m[s[0]], m[s[1]]);
        G(1, 5, 9, 13, m[s[2]], m[s[3]]);
        G(2, 6, 10, 14, m[s[4]], m[s[5]]);
        G(3, 7, 11, 15, m[s[6]], m[s[7]]);
        G(0, 5, 10, 15, m[s[8]], m[s[9]]);
        G(1, 6, 11, 12, m[s[10]], m[s[11]]);
        G(2, 7, 8, 13, m[s[12]], m[s[13]]);
        G(3, 4, 9, 14, m[s[14]], m[s[15]]);
    }
    for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[i + 8];
}

template <class T>
void put(std::ostream &s, const T &v)
{
    s.write(reinterpret_cast<const char *>(&v), sizeof(T));
}
template <class T>
T get(std::istream &s)
{
    T v{};
    s.read(reinterpret_cast<char *>(&v), sizeof(T));
    if (!s) throw std::runtime_error("I/O error");
    return v;
}

Serialization::SEALHeader read_header(std::istream &s)
{
    auto h = get<Serialization::SEALHeader>(s);
    if (!Serialization::IsValidHeader(h)) throw std::logic_error("loaded SEALHeader is invalid");
    if (h.compr_mode != compr_mode_type::none) throw std::logic_error("unsupported compression mode");
    return h;
}

void write_header(std::ostream &s, std::uint64_t total, compr_mode_type mode)
{
    if (mode != compr_mode_type::none) throw std::invalid_argument("unsupported compression mode");
    Serialization::SEALHeader h;
    h.size = total;
    put(s, h);
}

constexpr std::streamoff kHeader = sizeof(Serialization::SEALHeader);

// DynArray<u64>: header + count + words
std::streamoff dynarray_size(std::size_t words) { return kHeader + 8 + (std::streamoff)(8 * words); }
void write_dynarray(std::ostream &s, const std::uint64_t *p, std::size_t words)
{
    write_header(s, (std::uint64_t)dynarray_size(words), compr_mode_type::none);
    put<std::uint64_t>(s, words);
    if (words) s.write(reinterpret_cast<const char *>(p), (std::streamsize)(8 * words));
}
// reads the count (bounded by `max_words`, SEAL's in_size check) into `out`
void read_dynarray(std::istream &s, std::vector<std::uint64_t> &out, std::size_t max_words)
{
    const auto h = read_header(s);
    const auto words = get<std::uint64_t>(s);
    if (words > max_words || h.size != (std::uint64_t)dynarray_size(words))
        throw std::logic_error("ciphertext data is invalid");
    out.resize(words);
    if (words) s.read(reinterpret_cast<char *>(out.data()), (std::streamsize)(8 * words));
    if (!s) throw std::runtime_error("I/O error");
}

template <class Obj>
std::streamoff save_to_buffer(const Obj &o, seal_byte *out, std::size_t size, compr_mode_type mode)
{
    const std::streamoff need = o.save_size(mode);
    if (!out || (std::streamoff)size < need) throw std::invalid_argument("insufficient size");
    std::ostringstream ss(std::ios::binary);
    o.save(ss, mode);
    const std::string b = ss.str();
    std::memcpy(out, b.data(), b.size());
    return (std::streamoff)b.size();
}

template <class Obj>
std::streamoff load_from_buffer(Obj &o, const SEALContext &ctx, const seal_byte *in, std::size_t size)
{
    if (!in) throw std::invalid_argument("in cannot be null");
    std::istringstream ss(std::string(reinterpret_cast<const char *>(in), size), std::ios::binary);
    return o.load(ctx, ss);
}

// UniformRandomGeneratorInfo (randomgen.cpp:99-158): header + prng_type + seed
constexpr std::streamoff kInfo = kHeader + 1 + (std::streamoff)prng_seed_byte_count;
void write_info(std::ostream &s, const prng_seed_type &seed)
{
    write_header(s, (std::uint64_t)kInfo, compr_mode_type::none);
    put<std::uint8_t>(s, (std::uint8_t)prng_type::blake2xb);
    s.write(reinterpret_cast<const char *>(seed.data()), (std::streamsize)prng_seed_byte_count);
}
prng_seed_type read_info(std::istream &s)
{
    const auto h = read_header(s);
    if (h.size != (std::uint64_t)kInfo) throw std::logic_error("ciphertext data is invalid");
    const auto t = get<std::uint8_t>(s);
    if (t == (std::uint8_t)prng_type::shake256) throw std::logic_error("unsupported prng_type");
    if (t != (std::uint8_t)prng_type::blake2xb) throw std::logic_error("prng_type is invalid");
    prng_seed_type seed;
    s.read(reinterpret_cast<char *>(seed.data()), (std::streamsize)prng_seed_byte_count);
    if (!s) throw std::runtime_error("I/O error");
    return seed;
}
// c1 = sample_poly_uniform(Blake2xbPRNG(seed)) drawn over the key-level primes listed in `prime`
// (limb order of the draw), limb l kept at out[slot[l]][n] when slot[l] >= 0 (host memory)
void expand_uniform(const SEALContext &ctx, const prng_seed_type &seed, const std::vector<int> &prime,
                    const std::vector<int> &slot, std::size_t n, std::uint64_t *out)
{
    std::vector<std::uint64_t> moduli;
    for (const auto &m : ctx.key_context_data()->parms().coeff_modulus()) moduli.push_back(m.value());
    rnd::sample_uniform_host(ctx.engine(), seed, moduli, prime, slot, n, out, ctx.stream());
}
std::vector<int> iota_limbs(std::size_t L)
{
    std::vector<int> v(L);
    for (std::size_t i = 0; i < L; i++) v[i] = (int)i;
    return v;
}
const prng_seed_type *seed_of(const SeedMap &seeds, std::size_t index, std::size_t digit)
{
    auto it = seeds.find(index);
    if (it == seeds.end() || digit >= it->second.size()) return nullptr;
    return &it->second[digit];
}

// residues of a [polys][limbs][n] block must be canonical (SEAL: is_data_valid_for)
bool residues_valid(const std::vector<std::uint64_t> &w, const std::vector<Modulus> &cm, std::size_t n)
{
    const std::size_t L = cm.size();
    for (std::size_t i = 0; i < w.size(); i++)
        if (w[i] >= cm[(i / n) % L].value()) return false;
    return true;
}
} // namespace

parms_id_type blake2b_parms_id(const std::uint64_t *words, std::size_t count)
{
    std::uint64_t h[8];
    for (int i = 0; i < 8; i++) h[i] = kIV[i];
    h[0] ^= 0x01010000ULL ^ 32; // no key, 32-byte digest
    const std::size_t bytes = count * 8;
    const auto *p = reinterpret_cast<const std::uint8_t *>(words);
    std::uint8_t block[128];
    std::size_t off = 0;
    while (bytes - off > 128)
    {
        std::memcpy(block, p + off, 128);
        off += 128;
        blake2b_compress(h, block, off, false);
    }
    std::memset(block, 0, 128);
    std::memcpy(block, p + off, bytes - off);
    blake2b_compress(h, block, bytes, true);
    parms_id_type id;
    for (int i = 0; i < 4; i++) id[i] = h[i];
    return id;
}

bool Serialization::IsValidHeader(const SEALHeader &h) noexcept
{
    return h.magic == seal_magic && h.header_size == seal_header_size && h.version_major == 3 &&
           (h.version_minor == 6 || h.version_minor == 5 || h.version_minor == 4) &&
           (std::uint8_t)h.compr_mode <= 2 && h.size >= seal_header_size;
}

// ------------------------------------------------------------------------------ Ciphertext
std::streamoff Ciphertext::save_size(compr_mode_type) const
{
    return kHeader + 32 + 1 + 8 * 3 + 8 + dynarray_size(store_.words());
}

std::streamoff Ciphertext::save(std::ostream &stream, compr_mode_type mode) const
{
    const std::streamoff total = save_size(mode);
    write_header(stream, (std::uint64_t)total, mode);
    put(stream, parms_id_);
    put<std::uint8_t>(stream, is_ntt_form_ ? 1 : 0);
    put<std::uint64_t>(stream, size_);
    put<std::uint64_t>(stream, poly_modulus_degree_);
    put<std::uint64_t>(stream, coeff_modulus_size_);
    put<double>(stream, scale_);
    write_dynarray(stream, store_.words() ? data() : nullptr, store_.words());
    if (!stream) throw std::runtime_error("I/O error");
    return total;
}

std::streamoff Ciphertext::save(seal_byte *out, std::size_t size, compr_mode_type mode) const
{
    return save_to_buffer(*this, out, size, mode);
}

std::streamoff Ciphertext::save_size_seeded(const SeedMap &seeds, compr_mode_type mode) const
{
    if (!seed_of(seeds, 0, 0)) return save_size(mode);
    if (size_ != 2) throw std::logic_error("a seeded ciphertext has size 2");
    return kHeader + 32 + 1 + 8 * 3 + 8 + dynarray_size(coeff_modulus_size_ * poly_modulus_degree_) + kInfo;
}

std::streamoff Ciphertext::save_seeded(std::ostream &stream, const SeedMap &seeds, compr_mode_type mode) const
{
    const prng_seed_type *seed = seed_of(seeds, 0, 0);
    if (!seed) return save(stream, mode);
    const std::streamoff total = save_size_seeded(seeds, mode);
    write_header(stream, (std::uint64_t)total, mode);
    put(stream, parms_id_);
    put<std::uint8_t>(stream, is_ntt_form_ ? 1 : 0);
    put<std::uint64_t>(stream, size_);
    put<std::uint64_t>(stream, poly_modulus_degree_);
    put<std::uint64_t>(stream, coeff_modulus_size_);
    put<double>(stream, scale_);
    write_dynarray(stream, data(), coeff_modulus_size_ * poly_modulus_degree_); // c0
    write_info(stream, *seed);
    if (!stream) throw std::runtime_error("I/O error");
    return total;
}

std::streamoff Ciphertext::load(const SEALContext &context, std::istream &stream)
{
    const auto h = read_header(stream);
    const auto id = get<parms_id_type>(stream);
    const auto ntt = get<std::uint8_t>(stream);
    const auto size = get<std::uint64_t>(stream);
    const auto n = get<std::uint64_t>(stream);
    const auto L = get<std::uint64_t>(stream);
    const auto scale = get<double>(stream);
    // metadata validity (SEAL: is_metadata_valid_for, pure key levels allowed)
    auto cd = context.get_context_data(id);
    if (!cd || ntt > 1 || cd->parms().poly_modulus_degree() != n || cd->parms().coeff_modulus().size() != L ||
        (size != 0 && (size < 2 || size > 16)))
        throw std::logic_error("ciphertext data is invalid");
    std::vector<std::uint64_t> w;
    read_dynarray(stream, w, (std::size_t)(size * n * L));
    std::streamoff expect = kHeader + 32 + 1 + 24 + 8 + dynarray_size(w.size());
    if (size == 2 && w.size() == n * L)
    {
        // seeded: c0 loaded, c1 expanded from the UniformRandomGeneratorInfo that follows
        const prng_seed_type seed = read_info(stream);
        w.resize(2 * n * L);
        expand_uniform(context, seed, iota_limbs((std::size_t)L), iota_limbs((std::size_t)L), (std::size_t)n,
                       w.data() + n * L);
        expect += kInfo;
    }
    if (w.size() != size * n * L || !residues_valid(w, cd->parms().coeff_modulus(), n) ||
        h.size != (std::uint64_t)expect)
        throw std::logic_error("ciphertext data is invalid");
    resize(context, id, (std::size_t)size);
    is_ntt_form_ = ntt != 0;
    scale_ = scale;
    if (!w.empty()) std::memcpy(data(), w.data(), 8 * w.size());
    return (std::streamoff)h.size;
}

std::streamoff Ciphertext::load(const SEALContext &context, const seal_byte *in, std::size_t size)
{
    return load_from_buffer(*this, context, in, size);
}

// ------------------------------------------------------------------------------ KSwitchKeys
// Every key index holds `digits` PublicKeys: a size-2 NTT-form ciphertext over the key level, which
// is exactly the [digit][2][K][n] slice of the device buffer (keygenerator.cpp:384-414).
namespace
{
std::streamoff pk_size(std::size_t K, std::size_t n) { return kHeader + 32 + 1 + 24 + 8 + dynarray_size(2 * K * n); }
// a seeded PublicKey record: c0 only, then the seed
std::streamoff pk_size_seeded(std::size_t K, std::size_t n)
{
    return kHeader + 32 + 1 + 24 + 8 + dynarray_size(K * n) + kInfo;
}
} // namespace

// A level-truncated key (KSwitchKeys, digits D < K-1) is written as D PublicKeys of D+1 limbs
// (primes q_0..q_{D-1}, P): the same record layout, an extension SEAL itself does not read.
std::streamoff KSwitchKeys::save_size(compr_mode_type mode) const { return save_size_seeded(SeedMap{}, mode); }

std::streamoff KSwitchKeys::save(std::ostream &stream, compr_mode_type mode) const
{
    return save_seeded(stream, SeedMap{}, mode);
}

std::streamoff KSwitchKeys::save_size_seeded(const SeedMap &seeds, compr_mode_type) const
{
    if (maker_) throw std::logic_error("deferred Galois keys cannot be serialized");
    const std::size_t dim1 = keys_.empty() ? 0 : keys_.rbegin()->first + 1;
    std::streamoff total = kHeader + 32 + 8 + (std::streamoff)(8 * dim1);
    for (const auto &kv : keys_)
    {
        const std::size_t KL = limbs_of(kv.first), words = kv.second.words();
        const std::size_t n = KL > 1 ? words / (2 * KL * (KL - 1)) : 0;
        if (!n || words != (KL - 1) * 2 * KL * n) throw std::logic_error("key data is invalid");
        for (std::size_t d = 0; d + 1 < KL; d++)
            total += seed_of(seeds, kv.first, d) ? pk_size_seeded(KL, n) : pk_size(KL, n);
    }
    return total;
}

std::streamoff KSwitchKeys::save_seeded(std::ostream &stream, const SeedMap &seeds, compr_mode_type mode) const
{
    const std::streamoff total = save_size_seeded(seeds, mode);
    write_header(stream, (std::uint64_t)total, mode);
    put(stream, parms_id_);
    const std::size_t dim1 = keys_.empty() ? 0 : keys_.rbegin()->first + 1;
    put<std::uint64_t>(stream, dim1);
    for (std::size_t i = 0; i < dim1; i++)
    {
        auto it = keys_.find(i);
        if (it == keys_.end())
        {
            put<std::uint64_t>(stream, 0);
            continue;
        }
        const std::size_t KL = limbs_of(i), digits = KL - 1, n = it->second.words() / (2 * KL * digits);
        put<std::uint64_t>(stream, digits);
        const std::uint64_t *p = it->second.host();
        for (std::size_t d = 0; d < digits; d++)
        {
            const prng_seed_type *seed = seed_of(seeds, i, d);
            write_header(stream, (std::uint64_t)(seed ? pk_size_seeded(KL, n) : pk_size(KL, n)), compr_mode_type::none);
            put(stream, parms_id_);
            put<std::uint8_t>(stream, 1);
            put<std::uint64_t>(stream, 2);
            put<std::uint64_t>(stream, n);
            put<std::uint64_t>(stream, KL);
            put<double>(stream, 1.0);
            if (seed)
            {
                write_dynarray(stream, p + d * 2 * KL * n, KL * n); // c0; c1 is the seed's
                write_info(stream, *seed);
            }
            else
                write_dynarray(stream, p + d * 2 * KL * n, 2 * KL * n);
        }
    }
    if (!stream) throw std::runtime_error("I/O error");
    return total;
}

std::streamoff KSwitchKeys::load(const SEALContext &context, std::istream &stream)
{
    const auto h = read_header(stream);
    const auto id = get<parms_id_type>(stream);
    if (id != context.key_parms_id()) throw std::logic_error("KSwitchKeys data is invalid");
    const auto cd = context.key_context_data();
    const std::size_t K = cd->parms().coeff_modulus().size(), n = cd->parms().poly_modulus_degree();
    const auto &cm = cd->parms().coeff_modulus();
    const auto dim1 = get<std::uint64_t>(stream);
    if (dim1 > 4 * n) throw std::logic_error("KSwitchKeys data is invalid");
    std::map<std::size_t, PolyStore> keys;
    std::map<std::size_t, std::size_t> limbs;
    std::streamoff total = kHeader + 32 + 8;
    for (std::size_t i = 0; i < dim1; i++)
    {
        const auto digits = get<std::uint64_t>(stream);
        total += 8;
        if (!digits) continue;
        if (digits > K - 1) throw std::logic_error("KSwitchKeys data is invalid");
        const std::size_t KL = digits + 1;
        std::vector<Modulus> stored(cm.begin(), cm.begin() + digits);
        stored.push_back(cm.back());
        PolyStore &ps = keys[i];
        limbs[i] = KL;
        ps.bind(context);
        ps.resize_words(digits * 2 * KL * n, false);
        std::uint64_t *dst = ps.host();
        for (std::size_t d = 0; d < digits; d++)
        {
            // one PublicKey record (Ciphertext::save_members layout) over the stored primes
            const auto rh = read_header(stream);
            const auto pid = get<parms_id_type>(stream);
            const auto ntt = get<std::uint8_t>(stream);
            const auto size = get<std::uint64_t>(stream);
            const auto deg = get<std::uint64_t>(stream);
            const auto cms = get<std::uint64_t>(stream);
            (void)get<double>(stream);
            if (pid != id || ntt != 1 || size != 2 || deg != n || cms != KL)
                throw std::logic_error("KSwitchKeys data is invalid");
            std::vector<std::uint64_t> w;
            read_dynarray(stream, w, 2 * KL * n);
            std::streamoff expect = pk_size(KL, n);
            if (w.size() == KL * n)
            {
                // seeded digit: c1 is SEAL's draw over every key-level prime, restricted to the
                // stored ones (q_0..q_{digits-1}, P) for a level-truncated key
                const prng_seed_type seed = read_info(stream);
                std::vector<int> slot(K, -1);
                for (std::size_t l = 0; l < digits; l++) slot[l] = (int)l;
                slot[K - 1] = (int)digits;
                w.resize(2 * KL * n);
                expand_uniform(context, seed, iota_limbs(K), slot, n, w.data() + KL * n);
                expect = pk_size_seeded(KL, n);
            }
            if (w.size() != 2 * KL * n || !residues_valid(w, stored, n) || rh.size != (std::uint64_t)expect)
                throw std::logic_error("KSwitchKeys data is invalid");
            std::memcpy(dst + d * 2 * KL * n, w.data(), 8 * w.size());
            total += (std::streamoff)rh.size;
        }
    }
    if ((std::uint64_t)total != h.size) throw std::logic_error("KSwitchKeys data is invalid");
    keys_ = std::move(keys);
    limbs_of_ = std::move(limbs);
    parms_id_ = id;
    key_limbs_ = K;
    maker_.reset();
    return total;
}

// ------------------------------------------------------------------------------ Plaintext
std::streamoff Plaintext::save_size(compr_mode_type) const { return kHeader + 32 + 8 + 8 + dynarray_size(store_.words()); }

std::streamoff Plaintext::save(std::ostream &stream, compr_mode_type mode) const
{
    const std::streamoff total = save_size(mode);
    write_header(stream, (std::uint64_t)total, mode);
    put(stream, parms_id_);
    put<std::uint64_t>(stream, store_.words());
    put<double>(stream, scale_);
    write_dynarray(stream, store_.words() ? data() : nullptr, store_.words());
    if (!stream) throw std::runtime_error("I/O error");
    return total;
}

std::streamoff Plaintext::save(seal_byte *out, std::size_t size, compr_mode_type mode) const
{
    return save_to_buffer(*this, out, size, mode);
}

std::streamoff Plaintext::load(const SEALContext &context, std::istream &stream)
{
    const auto h = read_header(stream);
    const auto id = get<parms_id_type>(stream);
    const auto count = get<std::uint64_t>(stream);
    const auto scale = get<double>(stream);
    // CKKS plaintexts are in NTT form at a chain level (parms_id_zero marks BFV-style coefficient
    // plaintexts, which the CKKS-only surface does not carry)
    auto cd = context.get_context_data(id);
    if (!cd) throw std::logic_error("plaintext data is invalid");
    const std::size_t n = cd->parms().poly_modulus_degree(), L = cd->parms().coeff_modulus().size();
    if (count != n * L) throw std::logic_error("plaintext data is invalid");
    std::vector<std::uint64_t> w;
    read_dynarray(stream, w, (std::size_t)count);
    if (w.size() != count || !residues_valid(w, cd->parms().coeff_modulus(), n) ||
        h.size != (std::uint64_t)(kHeader + 32 + 8 + 8 + dynarray_size(w.size())))
        throw std::logic_error("plaintext data is invalid");
    set_level(context, id, L);
    scale_ = scale;
    std::memcpy(data(), w.data(), 8 * w.size());
    return (std::streamoff)h.size;
}

std::streamoff Plaintext::load(const SEALContext &context, const seal_byte *in, std::size_t size)
{
    return load_from_buffer(*this, context, in, size);
}
} // namespace seal
