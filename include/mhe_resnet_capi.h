/* mhe_resnet_capi.h -- C ABI of the encrypted ResNet CIFAR-10 runner (libmhe_seal.so), for host
 * processes that are not C++ (one Python process per GPU under torch.distributed).
 *
 * It replaces the driver loop of cnn_ckks/cpu-ckks/single-key/cnn/infer_seal.cpp:234-577 (keys made
 * once, images fanned out over OpenMP threads sharing them, :404) with one runner per GPU: rank 0
 * generates the key set, every key buffer is exported as device memory, broadcast over RCCL (xGMI)
 * and imported on the other ranks, which then run their own images with the same keys.
 * Return values: 0 ok, -1 error (message from mhe_resnet_last_error, the C++ exception text).
 * Device pointers are on the runner's device (MHE_DEVICE / the calling process's GPU). */
#ifndef MHE_RESNET_CAPI_H
#define MHE_RESNET_CAPI_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mhe_resnet mhe_resnet;

/* layers: 20/32/44/56/110; params_bin: tests/golden/resnet/resnet{L}_params.* (make_resnet_params.py
 * format); comp_dir: holds d13.txt; generate_keys 1 = make the key set here (client + server),
 * 0 = keys follow through mhe_resnet_key_import + mhe_resnet_finish_import. */
int mhe_resnet_create(mhe_resnet **runner, int layers, const char *params_bin, const char *comp_dir, int generate_keys);
/* The same with the runner's PRNG seeded (keys, encryption randomness): seed != 0 makes every run
 * draw the same keys, so decrypted logits repeat run to run; 0 = a fresh random seed, as
 * mhe_resnet_create. */
int mhe_resnet_create_seeded(mhe_resnet **runner, int layers, const char *params_bin, const char *comp_dir,
                             int generate_keys, uint64_t seed);
int mhe_resnet_destroy(mhe_resnet *runner);
const char *mhe_resnet_last_error(void);

/* Key buffers (ResNetRunner::KeyBlob): kind 0 secret key [K][n], 1 public key [2][K][n],
 * 2 relinearization key [K-1][2][K][n], 3 Galois key `index` with `limbs` primes
 * ([limbs-1][2][limbs][n]); words = u64 count.  Export copies key i into dst_dev (synchronous). */
int mhe_resnet_key_count(mhe_resnet *runner, int *count);
int mhe_resnet_key_info(mhe_resnet *runner, int i, int *kind, uint64_t *index, uint64_t *limbs, uint64_t *words);
int mhe_resnet_key_export(mhe_resnet *runner, int i, void *dst_dev);
int mhe_resnet_key_import(mhe_resnet *runner, int kind, uint64_t index, uint64_t limbs, uint64_t words,
                          const void *src_dev);
int mhe_resnet_finish_import(mhe_resnet *runner);

/* count images (3 x 32 x 32 doubles each, before the /B of infer_seal.cpp:444) on `threads` host
 * threads (one HIP stream each).  logits: count x 10 (decrypted), labels: count, seconds: count
 * (per image, as the reference's total_time), boot/relu: count (time in bootstrapping / ReLU),
 * wall: the whole batch. */
int mhe_resnet_infer_batch(mhe_resnet *runner, const double *images, int count, int threads, double *logits,
                           int *labels, double *seconds, double *boot, double *relu, double *wall);
/* The same with `fibers` images per host thread at a time as one seal::FiberBatch (their key
 * switches, rescales and elementwise launches merged; boot / relu times are then not measured);
 * fibers 0 = MHE_RESNET_FIBERS (default 1, one image per thread). */
int mhe_resnet_infer_batch_fibers(mhe_resnet *runner, const double *images, int count, int threads, int fibers,
                                  double *logits, int *labels, double *seconds, double *boot, double *relu, double *wall);
int mhe_resnet_info(mhe_resnet *runner, double *setup_s, double *galois_key_gb, int *galois_keys);
/* key-switching key bytes the runner's key switches streamed since the last reset (reset != 0 zeroes) */
int mhe_resnet_key_traffic(mhe_resnet *runner, double *bytes, int reset);
/* operations of kind MHE_OPK_* (include/mhe.h) the runner ran since the last reset, counts[l] per
 * level l < 64 (reset != 0 zeroes them) */
int mhe_resnet_op_counts(mhe_resnet *runner, int kind, uint64_t *counts, int reset);
/* *prepared = 1 when the runner's evaluation keys are in the engine's prepared format
 * (mhe_key_prepare), 0 when they are in SEAL's layout (MHE_KEY_PREPARE=0). */
int mhe_resnet_key_format(mhe_resnet *runner, int *prepared);
/* Hoisted rotations of the runner's engine on / off (mhe_ctx_set_hoist; check: every hoisted rotation
 * recomputed by the classic path and compared), and stats[3] = hoisted rotations, hoisted key-MAC
 * launches, words that differed under check, since the last reset. */
int mhe_resnet_set_hoist(mhe_resnet *runner, int on, int check);
int mhe_resnet_hoist_stats(mhe_resnet *runner, uint64_t *stats, int reset);
/* Device scratch the runner's engine holds (per-stream workspaces, hoisting buffers, Galois mask
 * tables; mhe_scratch_bytes), beyond its keys and ciphertexts. */
int mhe_resnet_scratch_bytes(mhe_resnet *runner, double *bytes);
/* The same network in plain doubles with the exact ReLU (the check of a decrypted inference,
 * infer_seal.cpp:543-575 prints decrypted logits against the label): image 3 x 32 x 32 -> logits[10]. */
int mhe_resnet_plain_logits(mhe_resnet *runner, const double *image, double *logits);
/* The same network in plain doubles with the encrypted network's own ReLU, the minimax composite
 * polynomial on x / B restated on doubles (mhe_comp.h MinimaxReluPlain): a decrypted result differs
 * from it by the encryption's error alone (noise, rescaling, bootstrapping). */
int mhe_resnet_plain_logits_approx(mhe_resnet *runner, const double *image, double *logits);
/* stats[3]: merged FiberBatch / Lockstep calls that failed and were re-run member by member
 * (seal::merged_call_fallbacks), device allocations that succeeded only after the engine released
 * its cached blocks and retried, and allocations that failed (mhe_alloc_stats); process-wide, since
 * the last reset.  A healthy run reports 0, 0, 0. */
int mhe_resnet_fallback_stats(uint64_t *stats, int reset);

#ifdef __cplusplus
}
#endif
#endif
