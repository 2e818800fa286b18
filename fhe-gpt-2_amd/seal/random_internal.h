// random_internal.h -- samplers of SEAL/util/rlwe.cpp for the seal:: surface (random.cpp).
#pragma once
#include "seal/seal.h"

#include <cstdint>
#include <vector>

namespace seal
{
namespace rnd
{
// The first 64 bytes of the stream of `seed`: the public seed encrypt_zero_symmetric draws from its
// bootstrap PRNG before anything else (rlwe.cpp:317-321).
prng_seed_type stream_prefix_seed(const prng_seed_type &seed);

// sample_poly_uniform(Blake2xbPRNG(seed)) over limbs 0..L-1 (limb l reduced mod
// moduli[prime_of_limb[l]]); limbs with slot_of_limb[l] >= 0 are written to out[slot][n] on the
// device.  Synchronises stream s (the rejected words are ordered on the host).
void sample_uniform_dev(mhe_ctx *eng, const prng_seed_type &seed, const std::vector<std::uint64_t> &moduli,
                        const std::vector<int> &prime_of_limb, const std::vector<int> &slot_of_limb, std::size_t n,
                        std::uint64_t *out, void *s);
// ... over limbs 0..limbs-1 of the context, all kept
void sample_uniform_dev(mhe_ctx *eng, const prng_seed_type &seed, const std::vector<std::uint64_t> &moduli,
                        std::size_t limbs, std::size_t n, std::uint64_t *out, void *s);
// sample_uniform_dev into host memory out[slot][n] (the expansion of a saved seed on load)
void sample_uniform_host(mhe_ctx *eng, const prng_seed_type &seed, const std::vector<std::uint64_t> &moduli,
                         const std::vector<int> &prime_of_limb, const std::vector<int> &slot_of_limb, std::size_t n,
                         std::uint64_t *out, void *s);
// sample_poly_cbd from stream byte `byte_offset` (64-aligned) over limbs 0..limbs-1, on the device
void sample_cbd_dev(mhe_ctx *eng, const prng_seed_type &seed, std::uint64_t byte_offset, std::size_t limbs,
                    std::uint64_t *out, void *s);

// host samplers writing [limbs][n] residues
void sample_ternary_host(UniformRandomGenerator &prng, const std::vector<std::uint64_t> &moduli, std::size_t limbs,
                         std::size_t n, std::uint64_t *out);
void sample_cbd_host(UniformRandomGenerator &prng, const std::vector<std::uint64_t> &moduli, std::size_t limbs,
                     std::size_t n, std::uint64_t *out);
void sample_sparse_ternary_host(UniformRandomGenerator &prng, const std::vector<std::uint64_t> &moduli,
                                std::size_t n, std::size_t hamming_weight, std::uint64_t *out);
} // namespace rnd
} // namespace seal
