/*
 * mhe.h -- C ABI of the MI355X-native RNS-CKKS engine (libmhe.so).
 *
 * This is the drop-in boundary under the SEAL-compatible C++ surface: every entry point
 * replaces one step of the modified SEAL 3.6.6 evaluator path in the reference
 * (paths relative to /root/reference/cnn_ckks/cpu-ckks/single-key/seal-modified-3.6.6/native/src/seal/).
 *
 * Conventions
 *  - Polynomials are u64 residues laid out exactly like SEAL's Ciphertext/Plaintext/
 *    PublicKey data: [poly][limb][n], limb-major, NTT form for CKKS.  Uploading a SEAL
 *    object is one memcpy.
 *  - All data pointers passed to compute calls are DEVICE pointers (from mhe_malloc or any
 *    HIP allocation on the context's device).  Sizes are in limbs / polys; n = 2^log_n.
 *  - `stream` is a hipStream_t passed as void* (NULL = default stream).  Every call is
 *    stream-ordered and asynchronous; concurrent calls on different streams are safe
 *    (each stream gets its own scratch workspace).
 *  - Return value: MHE_OK (0) or a negative MHE_ERR_*; mhe_last_error() gives the message,
 *    worded like SEAL's exceptions so the C++ shim can rethrow them verbatim.
 *  - The modulus chain passed to mhe_ctx_create is the KEY level chain of a SEALContext
 *    (context.cpp:422-523): data primes q_0..q_{L-1} then the special prime P.  A ciphertext
 *    "at L limbs" uses q_0..q_{L-1}.
 */
#ifndef MHE_H
#define MHE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MHE_OK 0
#define MHE_ERR_ARG (-1)     /* std::invalid_argument in SEAL */
#define MHE_ERR_DEVICE (-2)  /* HIP runtime failure */
#define MHE_ERR_RANGE (-3)   /* std::out_of_range / end of modulus switching chain */
#define MHE_ERR_MEMORY (-4)  /* allocation failure */

typedef struct mhe_ctx mhe_ctx;

/* ---- diagnostics ---------------------------------------------------------------- */
const char *mhe_last_error(void);
int mhe_version(void);

/* ---- context ------------------------------------------------------------------------
 * Replaces SEALContext's per-prime precomputation: NTTTables::initialize
 * (util/ntt.cpp:30-89), RNSTool::inv_q_last_mod_q (util/rns.cpp:686-693), Modulus::const_ratio
 * (modulus.cpp:66-98).  log_n in [12,16]; moduli: key-level chain, special prime last;
 * count in [2,64]; each q < 2^61, q = 1 mod 2n. */
int mhe_ctx_create(mhe_ctx **ctx, int log_n, const uint64_t *moduli, int count, int device);
int mhe_ctx_destroy(mhe_ctx *ctx);
/* Pre-size the scratch workspace of `stream` for ciphertexts of up to max_limbs limbs so
 * that no allocation happens inside later calls (needed before hipGraph capture). */
int mhe_ctx_reserve(mhe_ctx *ctx, int max_limbs, void *stream);

/* CoeffModulus::Create (modulus.cpp:143-185 with get_primes, util/numth.cpp:279-317). */
int mhe_coeff_modulus_create(uint64_t poly_modulus_degree, const int *bit_sizes, int count, uint64_t *out);
/* GaloisTool::get_elt_from_step (util/galois.cpp:53-95); 0 on invalid step. */
uint32_t mhe_galois_elt_from_step(int log_n, int step);

/* ---- memory ----------------------------------------------------------------------- */
int mhe_malloc(mhe_ctx *ctx, void **dptr, size_t bytes);
int mhe_free(mhe_ctx *ctx, void *dptr);
/* Stream-ordered allocation from the device memory pool (kept cached: Ciphertext temporaries
 * are created and destroyed constantly by the reference's callers). */
int mhe_malloc_async(mhe_ctx *ctx, void **dptr, size_t bytes, void *stream);
int mhe_free_async(mhe_ctx *ctx, void *dptr, void *stream);
int mhe_memcpy_h2d(mhe_ctx *ctx, void *dst, const void *src, size_t bytes, void *stream);
int mhe_memcpy_d2h(mhe_ctx *ctx, void *dst, const void *src, size_t bytes, void *stream);
int mhe_memcpy_d2d(mhe_ctx *ctx, void *dst, const void *src, size_t bytes, void *stream);
int mhe_stream_sync(mhe_ctx *ctx, void *stream);
/* Device-side ordering without host blocking: work enqueued on `waiter` after the call runs after
 * everything already enqueued on `waitee` (event record + stream wait). */
int mhe_stream_wait(mhe_ctx *ctx, void *waiter, void *waitee);
/* Key-switching key bytes streamed by the key switches run on the context since the last reset
 * (L digits x 2 x (L+1) primes x n x 8 per switch): the algorithmic key traffic of a workload. */
int mhe_key_traffic(mhe_ctx *ctx, uint64_t *bytes, int reset);
/* The same key slices counted as a prepared key streams them (8 B per residue for the doubles
 * format, as in SEAL's layout). */
int mhe_key_traffic_prepared(mhe_ctx *ctx, uint64_t *bytes, int reset);
/* Operations run on the context since the last reset, by kind and level (limbs): counts[l] for
 * l < levels (reset != 0 zeroes every level of the kind).  Units: one key switch per entry
 * (relinearization, rotation, switch_key), one polynomial for the rest (a 2-poly rescale counts
 * 2, a plaintext product of a 2-poly ciphertext 2, an NTT of one poly 1).  The op mix of a
 * workload, e.g. for a CPU cost estimate from per-op CPU timings.  No SEAL counterpart. */
#define MHE_OPK_KEYSWITCH 0
#define MHE_OPK_RESCALE 1
#define MHE_OPK_TENSOR 2   /* ciphertext x ciphertext products (multiply / square), per product */
#define MHE_OPK_MULPLAIN 3 /* ciphertext x plaintext products */
#define MHE_OPK_ADDSUB 4   /* add / sub / negate (incl. the adds of fused product sums) */
#define MHE_OPK_SCALAR 5   /* per-limb scalar multiply / add / set */
#define MHE_OPK_NTT 6      /* forward or inverse NTT (encode, decode, transform_to/from_ntt) */
#define MHE_OPK_GALOIS 7   /* NTT-domain Galois permutation */
int mhe_op_counts(mhe_ctx *ctx, int kind, uint64_t *counts, int levels, int reset);

/* ---- launch coalescing (no SEAL counterpart) ----------------------------------------------------
 * With a hook set on the calling thread, the elementwise entry points mhe_add, mhe_sub, mhe_negate,
 * mhe_multiply_plain, mhe_multiply_plain_add, mhe_multiply_scalar, mhe_add_scalar, mhe_set_scalar,
 * mhe_ct_multiply, mhe_ct_square and mhe_memcpy_d2d check their arguments, then hand a descriptor of
 * their launch to the hook instead of launching.  The hook must get it run -- by mhe_launch_run,
 * alone or together with other descriptors -- and return; the entry point then returns l->rc.
 * mhe_launch_run runs descriptors of one context: entries of the same kind and shape (and scalars)
 * as one batched launch of up to 8, the rest one by one; each gets its rc.  seal::FiberBatch uses this
 * to turn the same-numbered elementwise calls of its fibers (the images of a batch) into one launch. */
#define MHE_LK_ADDSUB 1       /* op: 0 add, 1 sub, 2 negate */
#define MHE_LK_MULPLAIN 2
#define MHE_LK_MULPLAIN_ADD 3 /* out is the accumulator */
#define MHE_LK_SCALAR 4       /* op: 0 multiply, 1 add, 2 set; scalars per limb */
#define MHE_LK_TENSOR 5       /* op: 1 square (b unused); out gets 3 polys */
#define MHE_LK_COPY 6         /* bytes */
typedef struct mhe_launch
{
    int kind, op;
    const uint64_t *a, *b;
    uint64_t *out;
    int polys, limbs;
    size_t bytes;
    uint64_t scalars[64];
    void *stream;
    int rc;
} mhe_launch;
typedef void (*mhe_launch_hook)(mhe_ctx *ctx, mhe_launch *launch, void *user);
int mhe_set_launch_hook(mhe_launch_hook hook, void *user); /* the calling thread's hook; NULL = off */
int mhe_launch_run(mhe_ctx *ctx, mhe_launch *const *launches, int count);
/* A non-blocking HIP stream on the context's device (and its scratch workspace); the SEAL
 * shim gives every host thread its own, as the reference's OpenMP threads share one
 * Evaluator (cnn/infer_seal.cpp:404). */
/* Kernel timing for the benchmark: when on, HIP events are recorded on the launching stream
 * around every launch of the dominant key-switch kernels; mhe_kernel_time sums their durations
 * since the last call (kernel 0 = fused ModUp row pass + key inner products, 1 = ModUp column
 * pass) and resets. */
int mhe_ctx_set_timing(mhe_ctx *ctx, int on);
int mhe_kernel_time(mhe_ctx *ctx, int kernel, double *total_ms, int *launches);
/* Hoisted rotations (no SEAL counterpart; csrc/hoist.h): the rotations of an input that appears
 * more than once in one mhe_apply_galois_batch share one ModUp of the unrotated c1 (bit-identical
 * to SEAL's one-at-a-time switch_key_inplace).  on = 1 turns it on for this context (the default;
 * MHE_KS_HOIST=0 at context creation starts it off), 0 off.  check = 1 also recomputes every hoisted
 * rotation by the classic path on the same stream and compares the words (a debugging aid: one
 * host sync per hoisted pass; mismatches are counted and described on stderr).
 * mhe_hoist_stats: rotations that went through the hoisted path, launches of the hoisted key-MAC
 * kernels, and words that differed under check, since the last reset. */
int mhe_ctx_set_hoist(mhe_ctx *ctx, int on, int check);
int mhe_ctx_get_hoist(mhe_ctx *ctx, int *on, int *check);
int mhe_hoist_stats(mhe_ctx *ctx, uint64_t *rotations, uint64_t *mac_launches, uint64_t *check_mismatches, int reset);
/* Device scratch the context holds: per-stream workspaces (key-switch / rescale scratch for up to
 * 8 batch entries at the key level), hoisting buffers, Galois negation-mask tables, and the number
 * of streams with a workspace. */
int mhe_scratch_bytes(mhe_ctx *ctx, uint64_t *workspace, uint64_t *hoisting, uint64_t *masks, int *streams);
/* Fault injection for tests: the nth next device allocation of the context (mhe_malloc_async, or a
 * workspace / hoisting scratch growth) fails with MHE_ERR_MEMORY as if the device were out of
 * memory; 0 turns it off.  Used to check that a batched call that fails part way leaves its
 * operands as they were (tests/cpp/seal_batch_test.cpp). */
int mhe_debug_fail_alloc(mhe_ctx *ctx, int nth);
/* Fault injection for tests: the nth next batched key-switch launch sequence of the context (one
 * chunk of at most 8 entries of mhe_switch_key_batch, mhe_hmult_batch, ...) fails with MHE_ERR_MEMORY
 * before its first launch; 0 turns it off.  Used to fail the second chunk of a merged relinearization
 * (tests/cpp/seal_batch_test.cpp). */
int mhe_debug_fail_switch(mhe_ctx *ctx, int nth);
/* Process-wide allocation health, since the last reset: device allocations (ciphertext buffers and
 * scratch) that succeeded only after the caching allocator gave its cached blocks back to the device
 * and retried, and allocations that failed (injected failures included).  A healthy run reports 0
 * and 0; the SEAL surface's re-run merged calls are counted by seal::merged_call_fallbacks. */
int mhe_alloc_stats(uint64_t *retries, uint64_t *failures, int reset);
/* Give the device memory the engine's caching allocator holds for reuse (freed ciphertext / key
 * buffers, kept per size for the stream-ordered mhe_malloc_async) back to the device.  Synchronises
 * the device.  For after a setup phase that freed much more than the steady state reuses (e.g. the
 * ResNet runner's planning inference and its deferred keys). */
int mhe_trim(mhe_ctx *ctx);
int mhe_stream_create(mhe_ctx *ctx, void **stream);
int mhe_stream_destroy(mhe_ctx *ctx, void *stream);

/* ---- NTT ---------------------------------------------------------------------------
 * ntt_negacyclic_harvey(_lazy) / inverse_ntt_negacyclic_harvey(_lazy) on every limb l of
 * `polys` polynomials of `limbs` limbs each (limb l uses prime l of the chain):
 * util/ntt.cpp:183-209, util/ntt.h:235-296,336-396; ct version evaluator.cpp:2025-2118.
 * lazy=1 leaves forward outputs in [0,4q) and inverse outputs in [0,2q). */
int mhe_ntt_forward(mhe_ctx *ctx, uint64_t *data, int polys, int limbs, int lazy, void *stream);
int mhe_ntt_inverse(mhe_ctx *ctx, uint64_t *data, int polys, int limbs, int lazy, void *stream);

/* ---- coefficient-wise arithmetic ----------------------------------------------------
 * add/sub/negate_poly_coeffmod (util/polyarithsmallmod.h:190-300; Evaluator::add_inplace,
 * sub_inplace, negate_inplace evaluator.cpp:103-246); out may alias a or b. */
int mhe_add(mhe_ctx *ctx, const uint64_t *a, const uint64_t *b, uint64_t *out, int polys, int limbs, void *stream);
int mhe_sub(mhe_ctx *ctx, const uint64_t *a, const uint64_t *b, uint64_t *out, int polys, int limbs, void *stream);
int mhe_negate(mhe_ctx *ctx, const uint64_t *a, uint64_t *out, int polys, int limbs, void *stream);
/* dyadic_product_coeffmod per limb (util/polyarithsmallmod.cpp:111-165); b is [limbs][n] and
 * is broadcast over the polys of a: this is Evaluator::multiply_plain_ntt
 * (evaluator.cpp:1891-1930) when a is a ciphertext and b an NTT plaintext. */
int mhe_multiply_plain(mhe_ctx *ctx, const uint64_t *a, const uint64_t *b, uint64_t *out, int polys, int limbs,
                       void *stream);
/* acc += a * b (b broadcast over the polys of a): multiply_plain_ntt followed by add_inplace in one
 * pass, bit-identical to the two (evaluator.cpp:1891-1930, 78-120) */
int mhe_multiply_plain_add(mhe_ctx *ctx, const uint64_t *a, const uint64_t *b, uint64_t *acc, int polys, int limbs,
                           void *stream);
/* out = (accumulate ? out : 0) + sum_k a[k] * b[k] over `count` terms (each b[k] broadcast over the
 * polys of a[k]): one multiply_plain_ntt followed by count - 1 fused multiply_plain + add_inplace
 * steps of the same level, in one pass per 16 terms; the residues are those of the term-by-term
 * sequence (every partial sum is reduced mod q, and modular addition does not depend on order).
 * Used by the convolution's filter taps (cnn_seal.cpp:435-453) and the BSGS inner sums
 * (Bootstrapper.cpp:1975-1988). */
int mhe_multiply_plain_sum(mhe_ctx *ctx, int count, const uint64_t *const *a, const uint64_t *const *b, uint64_t *out,
                           int accumulate, int polys, int limbs, void *stream);
/* multiply_poly_scalar_coeffmod with one scalar per limb (scalars[l] < q_l), host array;
 * used by multiply_const (evaluator.cpp:287-301). */
int mhe_multiply_scalar(mhe_ctx *ctx, const uint64_t *a, const uint64_t *scalars, uint64_t *out, int polys,
                        int limbs, void *stream);
/* add_poly_scalar_coeffmod with one scalar per limb (add_const, evaluator.cpp:287-301). */
int mhe_add_scalar(mhe_ctx *ctx, const uint64_t *a, const uint64_t *scalars, uint64_t *out, int polys, int limbs,
                   void *stream);
/* out[p][l][*] = scalars[l]: the NTT form of a constant plaintext (CKKSEncoder::encode(double),
 * ckks.cpp:78-200, writes the same residue into every coefficient of limb l). */
int mhe_set_scalar(mhe_ctx *ctx, const uint64_t *scalars, uint64_t *out, int polys, int limbs, void *stream);

/* ---- ciphertext ops -------------------------------------------------------------------
 * Evaluator::ckks_multiply, size-2 x size-2 (evaluator.cpp:673-773): out3 = [3][L][n]. */
int mhe_ct_multiply(mhe_ctx *ctx, const uint64_t *a, const uint64_t *b, uint64_t *out3, int limbs, void *stream);
/* Evaluator::ckks_square (evaluator.cpp:1000-1059). */
int mhe_ct_square(mhe_ctx *ctx, const uint64_t *a, uint64_t *out3, int limbs, void *stream);

/* Key-switching key: one KSwitchKeys entry (vector<PublicKey>, keygenerator.cpp:384-414) laid
 * out [digit][2][key_limbs][n] on the device; the special prime is limb key_limbs-1 and data
 * limb i is limb i.  A full SEAL key has key_limbs = chain count and digits = count-1; a
 * level-truncated slice for L-limb ciphertexts may keep only L digits and L+1 limbs. */

/* Engine key formats (optional, no SEAL counterpart; the role of SEAL's KSwitchKeys
 * storage, keygenerator.cpp:384-414).  Converts a key of `digits` digits and `key_limbs` limbs
 * in place, and every key switch given it stays bit-identical:
 *   MHE_KEY_FMT_DOUBLE: each limb slot of a prime below 2^51 holds its residues as IEEE doubles
 *     (-0.0 for zero; every word >= 2^61, never a residue), the FP64 key MAC's operand with no
 *     unpacking -- for keys streamed by batched launches (the relinearization key of 8 HMults);
 *   MHE_KEY_FMT_PACK48: each limb slot of a prime below 2^48 holds a 32-bit plane [n], a 16-bit
 *     plane [n] and a tag word (>= 2^63) in its unused last quarter -- 6 instead of 8 bytes per
 *     residue, for keys streamed by one ciphertext at a time.
 * The key MAC recognises either format from the buffer itself.  The buffer is not a SEAL key again
 * until mhe_key_unprepare.  Preparing a prepared key (or unpreparing a SEAL key) fails with
 * MHE_ERR_ARG.  mhe_key_prepare makes MHE_KEY_FMT_DOUBLE (MHE_KEY_FMT=2 in the environment: PACK48). */
#define MHE_KEY_FMT_DOUBLE 1
#define MHE_KEY_FMT_PACK48 2
int mhe_key_prepare(mhe_ctx *ctx, uint64_t *key, int digits, int key_limbs, void *stream);
int mhe_key_prepare_as(mhe_ctx *ctx, uint64_t *key, int digits, int key_limbs, int format, void *stream);
int mhe_key_unprepare(mhe_ctx *ctx, uint64_t *key, int digits, int key_limbs, void *stream);
/* *prepared = the format of `key`: 0 SEAL's layout, MHE_KEY_FMT_DOUBLE or MHE_KEY_FMT_PACK48
 * (reads one or two words; host sync). */
int mhe_key_is_prepared(mhe_ctx *ctx, const uint64_t *key, int key_limbs, int *prepared, void *stream);

/* Evaluator::switch_key_inplace (evaluator.cpp:2281-2525): ct[2][L][n] += KS(target[L][n]). */
int mhe_switch_key(mhe_ctx *ctx, uint64_t *ct, const uint64_t *target, const uint64_t *key, int key_limbs,
                   int limbs, void *stream);
/* Evaluator::relinearize_internal for size 3 (evaluator.cpp:1061-1116): ct3[3][L][n] ->
 * first two polys hold the relinearised ciphertext. */
int mhe_relinearize(mhe_ctx *ctx, uint64_t *ct3, const uint64_t *key, int key_limbs, int limbs, void *stream);
/* Evaluator::apply_galois_inplace (evaluator.cpp:2120-2222) with GaloisTool::apply_galois_ntt
 * (util/galois.cpp:192-218): ct[2][L][n] in place. */
int mhe_apply_galois(mhe_ctx *ctx, uint64_t *ct, uint32_t galois_elt, const uint64_t *key, int key_limbs,
                     int limbs, void *stream);
/* The same with the input left untouched: out[2][L][n] = KS-rotated in (out must not alias in). */
int mhe_apply_galois_to(mhe_ctx *ctx, const uint64_t *in, uint64_t *out, uint32_t galois_elt, const uint64_t *key,
                        int key_limbs, int limbs, void *stream);
/* Batched launches: `count` independent operations of one level run as one launch per kernel
 * (up to 8 entries per launch; larger counts run in groups of 8), bit-identical to `count` calls
 * of the single-ciphertext entry point.  This is how independent rotations of the reference's
 * callers run on the GPU: the conv input rotations and output-channel gathers
 * (cnn/cnn_seal.cpp:423-430, 499-526), the BSGS baby and giant steps
 * (ckks_bootstrapping/Bootstrapper.cpp:1952-2087), and the same operation of several images
 * (cnn/infer_seal.cpp:404).  Pointer arrays are host arrays of device pointers. */
/* mhe_apply_galois_to for each i: out[i][2][L][n] = rotated in[i] with Galois element elts[i]
 * and key keys[i] (key_limbs[i]); outputs disjoint from every input and from each other. */
int mhe_apply_galois_batch(mhe_ctx *ctx, int count, const uint64_t *const *in, uint64_t *const *out,
                           const uint32_t *elts, const uint64_t *const *keys, const int *key_limbs, int limbs,
                           void *stream);
/* mhe_rescale_to_next for each i: in[i][size][L][n] -> out[i][size][L-1][n]. */
int mhe_rescale_batch(mhe_ctx *ctx, int count, const uint64_t *const *in, uint64_t *const *out, int size, int limbs,
                      void *stream);
/* mhe_switch_key for each i: ct[i][2][L][n] += KS(target[i][L][n]) with keys[i]. */
int mhe_switch_key_batch(mhe_ctx *ctx, int count, uint64_t *const *ct, const uint64_t *const *target,
                         const uint64_t *const *keys, const int *key_limbs, int limbs, void *stream);
/* GaloisTool::apply_galois_ntt alone on [polys][limbs][n] (out must not alias in). */
int mhe_permute_galois(mhe_ctx *ctx, const uint64_t *in, uint32_t galois_elt, uint64_t *out, int polys, int limbs,
                       void *stream);
/* Evaluator::mod_switch_scale_to_next / RNSTool::divide_and_round_q_last_ntt_inplace
 * (evaluator.cpp:1118-1181, util/rns.cpp:737-808): in[size][L][n] -> out[size][L-1][n].
 * L may be the full key level (special prime last), as Encryptor uses it to drop P. */
int mhe_rescale_to_next(mhe_ctx *ctx, const uint64_t *in, uint64_t *out, int size, int limbs, void *stream);
/* Evaluator::mod_switch_drop_to_next (evaluator.cpp:1183-1281): in[size][L][n] ->
 * out[size][L-1][n] (limb copy; out may equal in for an in-place compaction). */
int mhe_mod_switch_drop(mhe_ctx *ctx, const uint64_t *in, uint64_t *out, int size, int limbs, void *stream);
/* Bootstrapper::modraise_inplace (cnn_ckks/cpu-ckks/single-key/ckks_bootstrapping/Bootstrapper.cpp:
 * 2894-2948): in[size][1][n] in COEFFICIENT form mod q_0 -> out[size][limbs][n] coefficient form,
 * the centered lift of each coefficient reduced mod q_0..q_{limbs-1} (out must not alias in). */
int mhe_modraise(mhe_ctx *ctx, const uint64_t *in, uint64_t *out, int size, int limbs, void *stream);
/* One HMult: multiply + relinearize + rescale_to_next:
 * a, b: [2][L][n] -> out: [2][L-1][n]. */
int mhe_hmult(mhe_ctx *ctx, const uint64_t *a, const uint64_t *b, const uint64_t *relin_key, int key_limbs,
              uint64_t *out, int limbs, void *stream);
/* mhe_hmult for each i of `count` independent HMults sharing relin_key: out[i] = HMult(a[i], b[i]),
 * bit-identical to count mhe_hmult calls.  Up to 8 run per key switch, whose key stream is read
 * once per XCD for all of them (the independent multiply_inplace + relinearize_inplace +
 * rescale_to_next_inplace calls of the reference's callers, e.g. cnn_seal.cpp:423-430 products
 * of one layer, or the C2 microbenchmark's loop).  Outputs distinct; a[i] == b[i] squares. */
int mhe_hmult_batch(mhe_ctx *ctx, int count, const uint64_t *const *a, const uint64_t *const *b,
                    const uint64_t *relin_key, int key_limbs, uint64_t *const *out, int limbs, void *stream);

/* ---- CKKS encoding (SEAL/ckks.cpp:10-200, SEAL/ckks.h:457-640) ---------------------------
 * An encoder holds CKKSEncoder's constructor tables (index map 5^i, complex roots).  Encoding
 * is SEAL's host double-precision FFT in SEAL's operation order (no FMA, bit-identical),
 * then the RNS reduction and the per-limb NTT on the GPU. */
typedef struct mhe_encoder mhe_encoder;
int mhe_encoder_create(mhe_encoder **enc, int log_n);
int mhe_encoder_destroy(mhe_encoder *enc);
/* CKKSEncoder::encode(vector<double|complex<double>>, parms_id, scale, destination): re/im
 * host arrays (im may be NULL for real input), count <= n/2 slots; writes the NTT-form
 * plaintext [limbs][n] at device pointer out (limbs = coeff_modulus_size of the level). */
int mhe_ckks_encode(mhe_ctx *ctx, const mhe_encoder *enc, const double *re, const double *im, size_t count,
                    double scale, int limbs, uint64_t *out, void *stream);
/* CKKSEncoder::encode(double value, parms_id, scale, destination) (ckks.cpp:78-200): the
 * constant plaintext is one residue per limb, written to the host array residues[limbs]
 * (multiply_const / add_const feed it to mhe_multiply_scalar / mhe_add_scalar). */
int mhe_ckks_encode_scalar(mhe_ctx *ctx, double value, double scale, int limbs, uint64_t *residues);
/* The same, with SEAL's size checks made against the first `bound_limbs` primes while only the
 * first `limbs` residues are produced: encode at the first level followed by
 * mod_switch_to_inplace(plain, parms_id) (what Evaluator::add_const/multiply_const/
 * multiply_vector do, evaluator.cpp:287-310) without computing the dropped limbs. */
int mhe_ckks_encode_at(mhe_ctx *ctx, const mhe_encoder *enc, const double *re, const double *im, size_t count,
                       double scale, int bound_limbs, int limbs, uint64_t *out_dev, void *stream);
/* CKKSEncoder::decode (ckks.h:644-761): NTT-form plaintext [limbs][n] on the device ->
 * `sparse_slots` slot values (0 = n/2; the modified SEAL's sparse decode, ckks.h:704-713).
 * `im` may be NULL (decode to vector<double>).  Synchronous on `stream`. */
int mhe_ckks_decode(mhe_ctx *ctx, const mhe_encoder *enc, const uint64_t *plain_dev, int limbs, double scale,
                    size_t sparse_slots, double *re, double *im, void *stream);
int mhe_ckks_encode_scalar_at(mhe_ctx *ctx, double value, double scale, int bound_limbs, int limbs,
                              uint64_t *residues);

/* Random polynomials of key generation / encryption from SEAL's default PRNG (Blake2xbPRNG,
 * SEAL/randomgen.cpp:185-195: 4096-byte buffers, buffer c = BLAKE2Xb(4096, counter c, 64-byte seed))
 * through SEAL's samplers (SEAL/util/rlwe.cpp), bit-identical to SEAL for the same seed.
 *
 * sample_poly_uniform (rlwe.cpp:136-162), bulk part: the stream's first limbs*n words are the
 * draws of limbs 0..limbs-1 (limb l reduced mod prime prime_of_limb[l]); accepted words of limbs
 * with slot_of_limb[l] >= 0 are written, reduced, to out[slot][n]; the stream indices of rejected
 * words (w >= max_multiple) go to the device array rej (first rej_cap of them) and their count to
 * *rej_count (device, zeroed by the caller).  The caller sorts them and redraws each, in index
 * order, from the stream words after the bulk, then writes the results with
 * mhe_prng_apply_fixes (fixes_dev = pairs {out index, value}). */
int mhe_prng_uniform_bulk(mhe_ctx *ctx, const uint64_t seed[8], int limbs, const int *prime_of_limb,
                          const int *slot_of_limb, uint64_t *out, uint64_t *rej, uint32_t *rej_count,
                          uint32_t rej_cap, void *stream);
int mhe_prng_apply_fixes(mhe_ctx *ctx, const uint64_t *fixes_dev, uint32_t count, uint64_t *out, void *stream);
/* sample_poly_ternary (rlwe.cpp:21-38, kind MHE_SAMPLE_TERNARY, 4 stream bytes per coefficient) or
 * sample_poly_cbd (rlwe.cpp:101-133, kind MHE_SAMPLE_CBD, 6 bytes per coefficient), drawing from
 * stream byte `byte_offset` (a multiple of 64) of the PRNG seeded with `seed`, written as
 * canonical residues over limbs 0..limbs-1 of the context (coefficient form).  state_dev is a
 * device word pair: ternary sets state_dev[0] to the bytes its redraws consumed (a zero word is
 * redrawn, as libstdc++'s uniform_int_distribution does; usually 0) and CBD, given state_dev, reads
 * from byte_offset + state_dev[0] -- so the samples after a ternary one follow SEAL's stream with
 * no host synchronisation.  Async on stream. */
#define MHE_SAMPLE_TERNARY 1
#define MHE_SAMPLE_CBD 3
int mhe_prng_small(mhe_ctx *ctx, const uint64_t seed[8], uint64_t byte_offset, int kind, int limbs, uint64_t *out,
                   uint32_t *state_dev, void *stream);

#ifdef __cplusplus
}
#endif
#endif
