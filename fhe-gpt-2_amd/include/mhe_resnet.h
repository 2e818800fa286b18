// mhe_resnet.h -- encrypted ResNet-20/32/44/56/110 CIFAR-10 inference of the reference
// (cnn_ckks/cpu-ckks/single-key/cnn/infer_seal.cpp: import_parameters_cifar10 :3-100,
// ResNet_cifar10_seal_sparse :234-577) over the MI355X seal:: surface, with the multiplexed
// layers of mhe_cnn.h, the approximate ReLU of mhe_comp.h and the bootstrapping of mhe_boot.h.
//
// ResNetRunner is the one-time setup of ResNet_cifar10_seal_sparse (parameters, keys, three
// sparse-slot bootstrappers, LT coefficients, ReLU trees) and infer() the per-image body, in the
// reference's operation order.  Galois keys are registered for every rotation step and
// materialised on first use at the level of that use (seal.h, KSwitchKeys), which replaces the
// reference's hand-listed rotation_kinds table (infer_seal.cpp:345-360).
#pragma once

#include <memory>
#include <string>
#include <chrono>
#include <complex>
#include <cstdint>
#include <iosfwd>
#include <functional>
#include <vector>

#include "mhe_boot.h"
#include "mhe_cnn.h"

struct ResNetParams
{
    std::vector<double> linear_weight, linear_bias;
    std::vector<std::vector<double>> conv_weight, bn_bias, bn_running_mean, bn_running_var, bn_weight;
};

// infer_seal.cpp:3-100: text files of the reference layout under <dir>/resnet<L>_new/
void import_parameters_cifar10(std::vector<double> &linear_weight, std::vector<double> &linear_bias,
                               std::vector<std::vector<double>> &conv_weight,
                               std::vector<std::vector<double>> &bn_bias,
                               std::vector<std::vector<double>> &bn_running_mean,
                               std::vector<std::vector<double>> &bn_running_var,
                               std::vector<std::vector<double>> &bn_weight, std::size_t layer_num,
                               std::size_t end_num, const std::string &dir = "../../pretrained_parameters");
// The same values from one float64 file in import order (tests/golden/make_resnet_params.py).
ResNetParams load_resnet_params_bin(const std::string &path, std::size_t layer_num);
// The network in plain doubles with the exact ReLU (the output check of an encrypted inference:
// the reference prints decrypted logits next to the label, infer_seal.cpp:543-575): image is
// 3 x 32 x 32 values before the /B of infer_seal.cpp:444; returns the 10 logits.
std::vector<double> resnet_plain_logits(const ResNetParams &p, const std::vector<double> &image, std::size_t layer_num);
// The same with `relu` applied in place at every ReLU (e.g. the minimax composite of the encrypted
// network, ResNetRunner::plain_logits_approx).
std::vector<double> resnet_plain_logits(const ResNetParams &p, const std::vector<double> &image, std::size_t layer_num,
                                        const std::function<void(std::vector<double> &)> &relu);

struct ResNetResult
{
    std::vector<double> logits; // 10 scores (real parts of the first 10 slots)
    std::vector<std::complex<double>> slots; // the first 10 decoded slots as the reference prints them
    std::size_t label = 0;      // argmax
    double seconds = 0;         // total_time of the reference: encryption excluded, decryption excluded
    double boot_seconds = 0, relu_seconds = 0, linear_seconds = 0;
    int bootstraps = 0;
    // 64-bit digest of the output ciphertext's words, level and scale (FNV-1a over the u64 words):
    // equal digests mean bit-identical ciphertexts (the FiberBatch check compares an image batched
    // with the same image run alone)
    std::uint64_t digest = 0;
};

class ResNetRunner
{
public:
    // Where the keys come from.  generate: this runner is the client too -- KeyGenerator, public and
    // relinearization keys, and the level-truncated Galois key set planned by one inference with a
    // deferred provider.  import: the keys arrive from another runner (export_keys -> broadcast over
    // RCCL -> import_key on every rank), then finish_import().
    enum class KeySource
    {
        generate,
        import
    };
    // comp_dir: directory holding d<alpha>.txt of the approximate ReLU (mhe_comp.h)
    // rng_seed != 0: a debugging mode (seal.h Blake2xbSeedSequence): every generator of the setup --
    // secret, public, relinearization and Galois keys -- gets its own seed derived from rng_seed, and
    // after the setup every encryption uses rng_seed itself, so two runs of one image give the same
    // words whatever the thread or fiber order; never for real use
    ResNetRunner(std::size_t layer_num, const ResNetParams &params, const std::string &comp_dir,
                 KeySource keys = KeySource::generate, std::uint64_t rng_seed = 0);
    ~ResNetRunner();
    // one image: 3 x 32 x 32 values (channel-major, the test_values.txt order), before /B
    ResNetResult infer(const std::vector<double> &image);
    // the same, writing the reference's per-stage log (op, time, remaining level, scale) to *log
    ResNetResult infer(const std::vector<double> &image, std::ostream *log);
    // stage_syncs false: no host synchronisation around each ReLU / bootstrap (their times are then
    // not measured; used by the FiberBatch images, whose fibers share one stream)
    ResNetResult infer(const std::vector<double> &image, std::ostream *log, bool stage_syncs);
    // images on `threads` host threads at once, each on its own HIP stream (the reference runs one
    // image per OpenMP thread, infer_seal.cpp:404); results in image order
    // fibers > 1: each host thread runs `fibers` images at a time as a seal::FiberBatch (one stream, their
    // rotations, relinearizations, products and rescales merged into batched launches); 0 takes
    // MHE_RESNET_FIBERS (default 1: one image per thread)
    std::vector<ResNetResult> infer_batch(const std::vector<std::vector<double>> &images, int threads, int fibers = 0);
    double setup_seconds() const { return setup_s_; }
    // setup breakdown: the client's planning inference (deferred keys) and the truncated-key generation
    double plan_seconds() const { return plan_s_; }
    double keygen_seconds() const { return keygen_s_; }
    std::size_t galois_keys() const { return galois_keys_; }
    // device bytes of the server's Galois key set (all resident in HBM: no key traffic per image)
    double galois_key_gb() const;
    // key-switching key bytes streamed by this runner's key switches since the last reset
    double key_traffic_bytes(bool reset);
    // operations of the runner's key-level context since the last reset, per level (mhe_op_counts)
    std::vector<std::uint64_t> op_counts(int kind, bool reset);
    // hoisted rotations of the runner's engine (mhe_ctx_set_hoist): on / off, with the classic-path
    // check; stats: (hoisted rotations, hoisted MAC launches, differing words under check) since reset
    void set_hoist(bool on, bool check = false);
    std::vector<std::uint64_t> hoist_stats(bool reset);
    // bytes of device scratch the engine holds (per-stream workspaces, hoisting buffers, Galois masks)
    std::size_t scratch_bytes() const;
    // the evaluation keys are in the engine's prepared format (mhe_key_prepare) rather than SEAL's
    bool keys_prepared() const { return keys_prepared_; }
    // resnet_plain_logits with this runner's parameters
    std::vector<double> plain_logits(const std::vector<double> &image) const;
    // the same with the encrypted network's own ReLU: the minimax composite polynomial of
    // minimax_ReLU_seal on x / B, restated in plain doubles (MinimaxReluPlain), so a decrypted result
    // differs from it by the encryption's error alone (noise, rescaling, bootstrapping)
    std::vector<double> plain_logits_approx(const std::vector<double> &image) const;

    // key buffers as device memory, for sharing one key set across GPUs: kind 0 secret key [K][n],
    // 1 public key [2][K][n], 2 relinearization key [K-1][2][K][n], 3 Galois key `index` with
    // `limbs` stored primes ([limbs-1][2][limbs][n]).  dev stays valid while the runner lives.
    struct KeyBlob
    {
        int kind;
        std::size_t index, limbs, words;
        const std::uint64_t *dev;
    };
    std::vector<KeyBlob> export_keys() const;
    void import_key(const KeyBlob &blob); // device-to-device copy from blob.dev (this runner's device)
    // blob -> dst_dev in SEAL's key layout (a prepared key is unprepared in dst), synchronous
    void copy_key(const KeyBlob &blob, void *dst_dev) const;
    void finish_import();                 // after the last import_key (KeySource::import)

private:
    void finish_setup(bool plan_galois_keys);
    void prepare_keys(); // relinearization and Galois keys -> the engine's prepared key format
    struct Impl;
    std::unique_ptr<Impl> impl_;
    std::chrono::steady_clock::time_point t0_;
    double setup_s_ = 0, plan_s_ = 0, keygen_s_ = 0;
    std::size_t galois_keys_ = 0;
    bool keys_prepared_ = false;
};

// infer_seal.cpp:234-577 entry point: images [start, end] from ../../../testFile/test_values.txt
// when present, else seeded synthetic images (uniform [-2.5, 2.5], seed = image id); parameters
// from ../../pretrained_parameters (or $MHE_RESNET_PARAMS, a .bin from make_resnet_params.py).
void ResNet_cifar10_seal_sparse(std::size_t layer_num, std::size_t start_image_id, std::size_t end_image_id);
