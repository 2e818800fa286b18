// resnet_capi.cpp -- the C ABI of include/mhe_resnet_capi.h over ResNetRunner (mhe_resnet.h).
#include <algorithm>
#include "../../include/mhe_resnet_capi.h"

#include "mhe_resnet.h"

#include <chrono>
#include <cstring>
#include <fstream>
#include <memory>
#include <string>
#include <vector>

#include "../../include/mhe.h"

struct mhe_resnet
{
    std::unique_ptr<ResNetRunner> runner;
    std::vector<ResNetRunner::KeyBlob> keys;
};

namespace
{
thread_local std::string g_err;

template <class F>
int guard(F f)
{
    try
    {
        f();
        return 0;
    }
    catch (const std::exception &e)
    {
        g_err = e.what();
    }
    catch (...)
    {
        g_err = "unknown error";
    }
    return -1;
}

ResNetParams load_params(const char *path, std::size_t layers)
{
    // the packed fixture of tests/golden/make_resnet_params.py (resnet20_params.bin: <f8 values;
    // resnet110_params.d7: 7 significant digits as text-free floats), read by the runner's own loader
    return load_resnet_params_bin(path, layers);
}
} // namespace

extern "C" {
const char *mhe_resnet_last_error(void)
{
    return g_err.c_str();
}

int mhe_resnet_create_seeded(mhe_resnet **out, int layers, const char *params_bin, const char *comp_dir,
                             int generate_keys, uint64_t seed)
{
    return guard([&] {
        if (!out || !params_bin || !comp_dir) throw std::invalid_argument("null argument");
        auto r = std::make_unique<mhe_resnet>();
        r->runner = std::make_unique<ResNetRunner>((std::size_t)layers, load_params(params_bin, (std::size_t)layers),
                                                   comp_dir,
                                                   generate_keys ? ResNetRunner::KeySource::generate
                                                                 : ResNetRunner::KeySource::import,
                                                   seed);
        if (generate_keys) r->keys = r->runner->export_keys();
        *out = r.release();
    });
}

int mhe_resnet_create(mhe_resnet **out, int layers, const char *params_bin, const char *comp_dir, int generate_keys)
{
    return mhe_resnet_create_seeded(out, layers, params_bin, comp_dir, generate_keys, 0);
}

int mhe_resnet_destroy(mhe_resnet *r)
{
    return guard([&] { delete r; });
}

int mhe_resnet_key_count(mhe_resnet *r, int *count)
{
    return guard([&] { *count = (int)r->keys.size(); });
}

int mhe_resnet_key_info(mhe_resnet *r, int i, int *kind, uint64_t *index, uint64_t *limbs, uint64_t *words)
{
    return guard([&] {
        const auto &b = r->keys.at((std::size_t)i);
        *kind = b.kind;
        *index = b.index;
        *limbs = b.limbs;
        *words = b.words;
    });
}

int mhe_resnet_key_export(mhe_resnet *r, int i, void *dst)
{
    return guard([&] {
        r->runner->copy_key(r->keys.at((std::size_t)i), dst);
    });
}

int mhe_resnet_key_import(mhe_resnet *r, int kind, uint64_t index, uint64_t limbs, uint64_t words, const void *src)
{
    return guard([&] {
        r->runner->import_key({ kind, (std::size_t)index, (std::size_t)limbs, (std::size_t)words,
                                static_cast<const std::uint64_t *>(src) });
    });
}

int mhe_resnet_finish_import(mhe_resnet *r)
{
    return guard([&] {
        r->runner->finish_import();
        r->keys = r->runner->export_keys();
    });
}

int mhe_resnet_infer_batch(mhe_resnet *r, const double *images, int count, int threads, double *logits, int *labels,
                           double *seconds, double *boot, double *relu, double *wall)
{
    return mhe_resnet_infer_batch_fibers(r, images, count, threads, 0, logits, labels, seconds, boot, relu, wall);
}

int mhe_resnet_infer_batch_fibers(mhe_resnet *r, const double *images, int count, int threads, int fibers,
                                  double *logits, int *labels, double *seconds, double *boot, double *relu, double *wall)
{
    return guard([&] {
        std::vector<std::vector<double>> imgs((std::size_t)count);
        for (int i = 0; i < count; i++) imgs[i].assign(images + (std::size_t)i * 3072, images + (std::size_t)(i + 1) * 3072);
        const auto t0 = std::chrono::steady_clock::now();
        auto res = r->runner->infer_batch(imgs, threads, fibers);
        if (wall) *wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        for (int i = 0; i < count; i++)
        {
            for (int k = 0; k < 10; k++) logits[i * 10 + k] = res[i].logits[k];
            if (labels) labels[i] = (int)res[i].label;
            if (seconds) seconds[i] = res[i].seconds;
            if (boot) boot[i] = res[i].boot_seconds;
            if (relu) relu[i] = res[i].relu_seconds;
        }
    });
}

int mhe_resnet_key_traffic(mhe_resnet *r, double *bytes, int reset)
{
    return guard([&] {
        const double b = r->runner->key_traffic_bytes(reset != 0);
        if (bytes) *bytes = b;
    });
}

int mhe_resnet_op_counts(mhe_resnet *r, int kind, uint64_t *counts, int reset)
{
    return guard([&] {
        if (!counts) throw std::invalid_argument("null argument");
        const auto c = r->runner->op_counts(kind, reset != 0);
        std::copy(c.begin(), c.end(), counts);
    });
}

int mhe_resnet_key_format(mhe_resnet *r, int *prepared)
{
    return guard([&] {
        if (!prepared) throw std::invalid_argument("null argument");
        *prepared = r->runner->keys_prepared() ? 1 : 0;
    });
}

int mhe_resnet_set_hoist(mhe_resnet *r, int on, int check)
{
    return guard([&] { r->runner->set_hoist(on != 0, check != 0); });
}

int mhe_resnet_hoist_stats(mhe_resnet *r, uint64_t *stats, int reset)
{
    return guard([&] {
        if (!stats) throw std::invalid_argument("null argument");
        const auto v = r->runner->hoist_stats(reset != 0);
        std::copy(v.begin(), v.end(), stats);
    });
}

int mhe_resnet_scratch_bytes(mhe_resnet *r, double *bytes)
{
    return guard([&] {
        if (!bytes) throw std::invalid_argument("null argument");
        *bytes = (double)r->runner->scratch_bytes();
    });
}

int mhe_resnet_plain_logits(mhe_resnet *r, const double *image, double *logits)
{
    return guard([&] {
        if (!image || !logits) throw std::invalid_argument("null argument");
        const std::vector<double> out = r->runner->plain_logits(std::vector<double>(image, image + 3072));
        for (int k = 0; k < 10; k++) logits[k] = out[k];
    });
}

int mhe_resnet_plain_logits_approx(mhe_resnet *r, const double *image, double *logits)
{
    return guard([&] {
        if (!image || !logits) throw std::invalid_argument("null argument");
        const std::vector<double> out = r->runner->plain_logits_approx(std::vector<double>(image, image + 3072));
        for (int k = 0; k < 10; k++) logits[k] = out[k];
    });
}

int mhe_resnet_fallback_stats(uint64_t *stats, int reset)
{
    return guard([&] {
        if (!stats) throw std::invalid_argument("null argument");
        stats[0] = seal::merged_call_fallbacks(reset != 0);
        if (mhe_alloc_stats(&stats[1], &stats[2], reset) != 0) throw std::runtime_error(mhe_last_error());
    });
}

int mhe_resnet_info(mhe_resnet *r, double *setup_s, double *gb, int *nkeys)
{
    return guard([&] {
        if (setup_s) *setup_s = r->runner->setup_seconds();
        if (gb) *gb = r->runner->galois_key_gb();
        if (nkeys) *nkeys = (int)r->runner->galois_keys();
    });
}
}
