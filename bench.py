"""Benchmark of the hot path: homomorphic multiplications per second (BASELINE.json metric)
on config 2 -- N=2^16, 45-prime chain (44 data limbs + 1 special prime), one HMult =
multiply_inplace + relinearize_inplace + rescale_to_next_inplace.

One step = BATCH independent HMults per GPU (same relin key, different ciphertexts), inputs
resident in HBM before the timed region, spread round-robin over 4 HIP streams (the hardware
queues of one process) so one HMult's small ModDown/rescale kernels overlap the next one's
key-switch kernels.  Multi-GPU: one process per GPU (torchrun), each
rank runs its own ciphertexts (images are independent in the reference), the relin key is
generated on rank 0 and broadcast over RCCL/xGMI once at setup; no collective in the data
path -> weak scaling.

Prints one JSON line (rank 0).  The cpu_baseline leg times the repo's CPU restatement of the
reference algorithm (oracle/, "port") on the host cores of the same box.
"""
import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fhe-gpt-2_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import mhe  # noqa: E402

LOG_N = 16
C2_BITS = [51] + [46] * 30 + [51] * 13 + [51]
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
MIB = 1 << 20


def hmult_bytes(L, key_bytes=None):
    """Algorithmic HBM bytes of one HMult: 2 input cts (2L MiB) + relin key
    slice (L(L+1) MiB in SEAL's layout) + output ct ((L-1) MiB) = L^2 + 4L - 1 MiB; with a
    prepared key the key term is the prepared slice's bytes (ks_row_mac_key_bytes)."""
    if key_bytes is None:
        return (L * L + 4 * L - 1) * MIB
    return (3 * L - 1) * MIB + key_bytes


def ks_row_mac_key_bytes(L, n, moduli=None, prepared=False):
    """Algorithmic HBM bytes of one k_ks_row_mac launch (SURVEY.md §8(d) key slice): every key
    limb it multiplies against is read once, 2 polys x L digits x (L+1) primes x n residues, 8 B
    each in SEAL's layout; a prepared key (mhe_key_prepare) holds the same limbs as doubles, also
    8 B per residue.  The ModUp intermediate the kernel also reads is not algorithmic."""
    return 2 * L * (L + 1) * n * 8


FP64_LANE_OPS_PEAK = 35e12  # v_fma_f64 lane-ops/s measured on MI355X (profiles/r01_ubench_valu.txt; spec 39.3e12)


def ks_row_mac_valu(L, n, moduli):
    """VALU model of one k_ks_row_mac launch (SURVEY.md §8(d) per-op work): the ModUp row pass of
    the L^2 digit/prime pairs with I != J (8 of the 16 stages: L^2 * 8 * n/2 butterflies) and the
    key inner products (2 * L * (L+1) * n multiply-accumulates).  FP64 lane-ops per butterfly: 8
    (lazy form, q < 2^47) or 11; per MAC: 7 (the FP64 mulmod's 6 and the accumulating add; a
    prepared key is already a double, so no conversion is counted -- up to round 5 the model
    counted 8, with the key word's conversion)."""
    primes = list(moduli[:L]) + [moduli[-1]]
    bfly = sum((L - (1 if I < L else 0)) * 8 * (n // 2) * (8 if q < (1 << 47) else 11) for I, q in enumerate(primes))
    macs = 2 * L * (L + 1) * n
    return {"butterflies": L * L * 8 * (n // 2), "macs": macs, "fp64_lane_ops": bfly + 7 * macs}


def rand_residues(shape, moduli_t, gen):
    """Uniform residues on device: last two dims [limbs][n], limb l uniform in [0, q_l)."""
    hi = torch.randint(0, 2**62, shape, generator=gen, device=moduli_t.device, dtype=torch.int64)
    return torch.remainder(hi, moduli_t.view(*([1] * (len(shape) - 2)), -1, 1))


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cgroup_cpu_max():
    """The cgroup v2 CPU quota of this process ("max" = none), as '<quota> <period>'."""
    try:
        return open("/sys/fs/cgroup/cpu.max").read().strip()
    except OSError:
        return None


def cpu_baseline(moduli, L_main, threads):
    """SURVEY.md §8(d) CPU baseline: the repo's CPU restatement of the reference algorithm (oracle/,
    "port", bit-exact with the GPU path), compiled on this host with -O3 -march=native, timed in
    this run on `threads` host cores (the box's CPU share for one GPU): single-thread HMult/s,
    B in {1, 8, 32} independent HMults (one per OpenMP thread) for L in {44, 31, 17, 3}, and the
    same on every host core this process may use at L in {44, 31} (`all_cores`)."""
    import tempfile

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # test infrastructure: only the baseline leg uses it

    tmp = tempfile.mkdtemp(prefix="mhe_oracle_")
    O.build_native(tmp)
    n = 1 << LOG_N
    oc = O.Context(LOG_N, moduli)
    rng = np.random.default_rng(20261015)
    K = len(moduli)
    qs = np.array(moduli, np.uint64)
    Lmax = max(L_main, 44)
    key = rng.integers(0, 2**62, size=(Lmax, 2, K, n), dtype=np.uint64) % qs[None, None, :, None]
    a_all = rng.integers(0, 2**62, size=(32, 2, Lmax, n), dtype=np.uint64) % qs[None, None, :Lmax, None]
    b_all = rng.integers(0, 2**62, size=(32, 2, Lmax, n), dtype=np.uint64) % qs[None, None, :Lmax, None]
    table, walls = {}, {}
    for L in (44, 31, 17, 3):
        kL = np.ascontiguousarray(key[:L])
        row = {}
        for B in (1, 8, 32):
            a = np.ascontiguousarray(a_all[:B, :, :L])
            b = np.ascontiguousarray(b_all[:B, :, :L])
            t0 = time.perf_counter()
            _, used = oc.hmult_batch(a, b, kL, threads=min(B, threads))
            dt = time.perf_counter() - t0
            row[str(B)] = round(B / dt, 4)
            walls[(L, B)] = (dt, used)
        table[str(L)] = row
    # all host cores: the cores this process may actually use -- the CPU
    # affinity capped by the cgroup quota (the GPU box gives one GPU's job 16 of its nproc CPUs; more
    # threads than that only time-share them: 256 threads measured 4.8 HMult/s at L=44 against 10.5
    # on 16, r03c) -- with B = 32 independent HMults on that many threads, at L = 44 and L = 31
    host = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = cgroup_cpu_max()
    usable = host
    try:
        q, per = quota.split()
        if q != "max":
            usable = max(1, min(host, -(-int(q) // int(per))))
    except (AttributeError, ValueError):
        pass
    all_cores = {"usable_cpus": usable, "affinity_cpus": host, "cgroup_cpu_max": quota, "batch": 32}
    for L in (44, 31):
        if usable == threads and str(L) in table:
            all_cores[str(L)] = {"hmult_per_s": table[str(L)]["32"], "threads": usable, "note": "= per_L[L][32]"}
            continue
        kL = np.ascontiguousarray(key[:L])
        a = np.ascontiguousarray(a_all[:, :, :L])
        b = np.ascontiguousarray(b_all[:, :, :L])
        t0 = time.perf_counter()
        _, used = oc.hmult_batch(a, b, kL, threads=usable)
        dt = time.perf_counter() - t0
        all_cores[str(L)] = {"hmult_per_s": round(32 / dt, 3), "wall_s": round(dt, 2), "threads": int(used)}
    a1 = np.ascontiguousarray(a_all[:1, :, :L_main])
    b1 = np.ascontiguousarray(b_all[:1, :, :L_main])
    t0 = time.perf_counter()
    oc.hmult_batch(a1, b1, np.ascontiguousarray(key[:L_main]), threads=1)
    single = 1.0 / (time.perf_counter() - t0)
    dt, used = walls[(L_main, 32)] if (L_main, 32) in walls else (None, threads)
    return {
        "value": table.get(str(L_main), {}).get("32", round(single, 4)),
        "unit": "HMult/s",
        "cores": int(used),
        "kind": "port",
        "nproc": os.cpu_count(),
        "model": cpu_model(),
        "build": "gcc -O3 -march=native -fopenmp (built on this host in this run)",
        "single_thread": round(single, 4),
        "all_cores": all_cores,
        "per_L": {"limbs": table, "batch_key": "independent HMults, one per OpenMP thread, min(B, cores) threads"},
        "sample": f"32 independent HMults (N=2^16, L={L_main}, 45-prime C2 chain) on {used} threads, "
                  f"oracle/mhe_oracle.c (restatement of SEAL's evaluator); {dt:.1f} s wall"
                  if dt else f"single HMult at L={L_main}",
    }


RESNET_BITS = [51] + [46] * 16 + [51] * 14 + [51]  # cnn/infer_seal.cpp:288-316: 31 data limbs + special
# The ResNet runner's keys are drawn from OS entropy as SEAL draws them (--resnet-seed N: the
# runner's reproducible debugging seed sequence instead).  The decrypted logits are checked against
# the plain network with the encrypted network's own minimax-composite ReLU (the encryption's error
# alone) and, as a labelled sanity check, with the exact ReLU; --resnet-key-draws extra key sets
# (fresh runners, 2 images each) report the error's spread over keys.
RESNET_CKKS_TOL = {20: 0.08, 110: 0.08}  # |decrypted - approx-ReLU plain| / max(1, max |logit|)
RESNET_EXACT_TOL = {20: 0.08, 110: 0.1}  # sanity: vs the exact-ReLU plain network


def logit_errors(runner, images, logits, layers):
    """Per image: max |decrypted - plain| against the approx-ReLU twin (the check) and the exact-ReLU
    network (sanity), and the twins' own distance; raises when an image leaves either band."""
    out = {"vs_approx_relu": [], "vs_exact_relu": [], "approx_vs_exact_relu": [], "rel_vs_approx_relu": []}
    for img, got in zip(images, logits):
        got = np.asarray(got)
        ap, ex = runner.plain_logits_approx(img), runner.plain_logits(img)
        e_ap, e_ex = float(np.max(np.abs(got - ap))), float(np.max(np.abs(got - ex)))
        m_ap, m_ex = max(1.0, float(np.max(np.abs(ap)))), max(1.0, float(np.max(np.abs(ex))))
        out["vs_approx_relu"].append(round(e_ap, 5))
        out["vs_exact_relu"].append(round(e_ex, 5))
        out["approx_vs_exact_relu"].append(round(float(np.max(np.abs(ap - ex))), 5))
        out["rel_vs_approx_relu"].append(round(e_ap / m_ap, 5))
        if not e_ap < RESNET_CKKS_TOL[layers] * m_ap:
            raise RuntimeError(f"encrypted ResNet-{layers} logits off the approx-ReLU plain network: {e_ap:.4g} >= "
                               f"{RESNET_CKKS_TOL[layers] * m_ap:.4g}")
        if not e_ex < RESNET_EXACT_TOL[layers] * m_ex:
            raise RuntimeError(f"encrypted ResNet-{layers} logits off the exact-ReLU plain network: {e_ex:.4g} >= "
                               f"{RESNET_EXACT_TOL[layers] * m_ex:.4g}")
    return out


def resnet_cpu_estimate(ops, threads):
    """Estimated CPU seconds per ResNet image on this host: the image's engine operations by kind
    and level (ops_per_image from the runner, mhe_op_counts) priced with the oracle's single-thread
    per-operation times (oracle/mhe_oracle.c, the CPU restatement of SEAL's evaluator, -O3 -march=native,
    built in this run) measured at L in {3, 10, 17, 24, 31} on the ResNet chain and interpolated (key
    switch: quadratic in L, the rest linear).  An estimate, not a run of the reference: it prices the
    same operations the GPU ran, one thread per image as the reference's OpenMP loop runs them."""
    import oracle as O  # test infrastructure: the cpu_baseline leg times it

    n = 1 << LOG_N
    moduli = mhe.coeff_modulus_create(n, RESNET_BITS)
    K = len(moduli)
    oc = O.Context(LOG_N, moduli)
    rng = np.random.default_rng(20261019)
    qs = np.array(moduli, np.uint64)
    levels = (3, 10, 17, 24, 31)
    Lmax = max(levels)
    key = rng.integers(0, 2**62, size=(Lmax, 2, K, n), dtype=np.uint64) % qs[None, None, :, None]
    ct = rng.integers(0, 2**62, size=(2, Lmax, n), dtype=np.uint64) % qs[None, :Lmax, None]
    ct2 = rng.integers(0, 2**62, size=(2, Lmax, n), dtype=np.uint64) % qs[None, :Lmax, None]
    elt = O.galois_elt_from_step(n, 5)

    def timed(f, reps=1):
        t0 = time.perf_counter()
        for _ in range(reps):
            f()
        return (time.perf_counter() - t0) / reps

    per = {k: [] for k in ("keyswitch", "rescale", "tensor", "mulplain", "addsub", "ntt", "galois")}
    for L in levels:
        a = np.ascontiguousarray(ct[:, :L])
        b = np.ascontiguousarray(ct2[:, :L])
        kL = np.ascontiguousarray(key[:L])
        tg = np.ascontiguousarray(b[1])
        pt = np.ascontiguousarray(b[0])
        reps = 1 if L >= 17 else 3
        per["keyswitch"].append(timed(lambda: oc.switch_key(a, tg, kL), reps))
        per["rescale"].append(timed(lambda: oc.rescale(a), 3) / 2)  # per polynomial
        per["tensor"].append(timed(lambda: oc.multiply(a, b), 3))
        per["mulplain"].append(timed(lambda: oc.multiply_plain(a, pt), 3) / 2)
        per["addsub"].append(timed(lambda: oc.add(a, b), 3) / 2)
        per["ntt"].append(timed(lambda: oc.ntt(a), 3) / 2)
        per["galois"].append(timed(lambda: O.apply_galois_ntt(a, LOG_N, elt), 3) / 2)
    fits = {k: np.polyfit(levels, v, 2 if k == "keyswitch" else 1) for k, v in per.items()}
    price = dict(fits, scalar=fits["mulplain"])
    total, by_kind = 0.0, {}
    for kind, lv in ops.items():
        f = price.get(kind)
        if f is None:
            continue
        s_ = sum(c * max(0.0, float(np.polyval(f, int(L)))) for L, c in lv.items())
        by_kind[kind] = round(s_, 2)
        total += s_
    return {
        "estimated_cpu_s_per_image": round(total, 1),
        "threads_per_image": 1,
        "throughput_images_per_s_on_host": round(threads / total, 5) if total > 0 else None,
        "host_cores": threads,
        "by_kind_s": by_kind,
        "per_op_s_at_levels": {k: dict(zip(map(str, levels), [round(x, 5) for x in v])) for k, v in per.items()},
        "kind": "estimate: oracle port (oracle/mhe_oracle.c) per-op CPU times x the GPU run's per-image op counts",
    }


RESNET20_CPU_S = 2188.8  # reference CPU SEAL, s/image, 1 thread per image (BASELINE.md / SURVEY.md §6)


def resnet_leg(device, images, streams, layers=20, fibers=1, seed=0, key_draws=0):
    """Second half of BASELINE.json's metric: seconds per image of encrypted ResNet-20 CIFAR-10
    (config C3: multiplexed conv + approximate ReLU + 18 bootstraps at N=2^16; config C4's network
    with layers=110), through the runner's C ABI (include/mhe_resnet_capi.h) in this process, with
    the reference's pretrained parameters on seeded synthetic images: single-stream images (latency), then
    `images` images on `streams` host threads (one HIP stream each).
    One key set for the whole job: rank 0 generates it (planning inference + SEAL
    keys truncated to their levels), every buffer is broadcast over RCCL/xGMI and imported by the
    other ranks; each rank then runs its own images.  Key traffic per image: none (all resident)."""
    from mhe import resnet as R

    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank() if world > 1 else 0
    os.environ["MHE_DEVICE"] = str(device)
    params = os.path.join(ROOT, "tests", "golden", "resnet",
                          "resnet20_params.bin" if layers == 20 else f"resnet{layers}_params.d7")
    comp = os.path.join(ROOT, "tests", "golden", "comp")
    mem = {}

    def used(tag):  # device-wide bytes in use (engine pools, keys, scratch, torch), GB
        free_b, total_b = torch.cuda.mem_get_info(device)
        mem[tag] = round((total_b - free_b) / 1e9, 1)

    used("before")
    t0 = time.perf_counter()
    R.Runner.fallback_stats(reset=True)
    runner = R.Runner(layers, params, comp, generate_keys=(rank == 0), seed=(seed + rank) if seed else 0)
    shared = None
    if world > 1:
        t1 = time.perf_counter()
        nbuf, nbytes = R.share_keys(dist, runner, torch.device("cuda", device), src=0)
        torch.cuda.synchronize(device)
        shared = {"buffers": nbuf, "GB": round(nbytes / 1e9, 2), "broadcast_s": round(time.perf_counter() - t1, 2)}
    setup = time.perf_counter() - t0
    used("after_setup")
    info = runner.info()
    rng = np.random.default_rng(1000 + rank)
    imgs = rng.uniform(-2.5, 2.5, size=(images, 3072))
    # latency: `lat` images one after another on one stream; the first also fills the runner's
    # static-operand encode cache, so the median of >= 3 is the warm per-image time (one image for
    # the deeper networks, where the batch below already is that single image)
    lat = 3 if layers <= 20 else 1
    lat_imgs = rng.uniform(-2.5, 2.5, size=(lat, 3072))
    runner.key_traffic(reset=True)
    runner.op_counts(reset=True)
    one = runner.infer_batch(lat_imgs, 1)
    used("after_latency_pass")
    key_bytes = runner.key_traffic(reset=True) / lat  # key-switching key bytes of one image
    # the engine operations of one image, by kind and level (mhe_op_counts): the op mix the CPU
    # estimate of the cpu_baseline leg prices
    ops = {k: {str(l): c / lat for l, c in enumerate(v) if c} for k, v in runner.op_counts(reset=True).items()}
    k_med = int(np.argsort(one["seconds"])[lat // 2])
    sec_one = float(one["seconds"][k_med])
    if world > 1:
        dist.barrier()
    t2 = time.perf_counter()
    runner.hoist_stats(reset=True)
    batch = runner.infer_batch(imgs, streams, fibers)
    batch_wall = time.perf_counter() - t2
    hoisted, hoist_macs, _ = runner.hoist_stats(reset=True)
    scratch = runner.scratch_bytes()
    used("after_batch")
    # every image's decrypted logits against the plain twins, on every rank -- the keys there may have
    # arrived over RCCL; a miss fails the leg
    errs = logit_errors(runner, np.concatenate([lat_imgs, imgs]), list(one["logits"]) + list(batch["logits"]), layers)
    prepared = runner.keys_prepared()
    runner.close()
    # merged calls re-run member by member and allocation retries / failures during the leg: 0 in a
    # healthy run (a fallback is where round 4's wrong image could hide)
    fb = R.Runner.fallback_stats(reset=True)
    fallbacks = {"merged_call_fallbacks": fb[0], "alloc_retries": fb[1], "alloc_failures": fb[2]}
    # the error's spread over key draws: fresh runners (new keys), two images each on one stream
    draws = []
    for k in range(key_draws if rank == 0 else 0):
        rk = R.Runner(layers, params, comp, generate_keys=True, seed=0)
        dimg = np.random.default_rng(5000 + k).uniform(-2.5, 2.5, size=(2, 3072))
        res = rk.infer_batch(dimg, 1)
        e = logit_errors(rk, dimg, res["logits"], layers)
        rk.close()
        draws.append({"draw": k + 1, "vs_approx_relu": e["vs_approx_relu"], "vs_exact_relu": e["vs_exact_relu"]})
    return {
        "workload": ("C3" if layers == 20 else "C4" if layers == 110 else "ResNet")
        + f": ResNet-{layers} CIFAR-10, N=2^16, 31+1 primes, sparse bootstrapping (logn 14/13/12)",
        "data": "reference pretrained parameters (tests/golden/resnet), seeded synthetic images",
        "sec_per_image_1stream": round(sec_one, 4),
        "sec_per_image_1stream_samples": [round(float(x), 4) for x in one["seconds"]],
        "latency_stat": f"median of {lat} images, one stream" if lat > 1 else "one image, one stream",
        "bootstrap_s_per_image": round(float(one["boot"][k_med]), 4),
        "relu_s_per_image": round(float(one["relu"][k_med]), 4),
        "batch_wall_s": round(batch_wall, 4),
        "batch_images": images,
        "streams": streams,
        "fibers_per_stream": fibers,
        "batch_mode": (f"{streams} host threads x {fibers} images as one seal::FiberBatch each (merged key switches, "
                       "rescales and elementwise launches)" if fibers > 1 else f"{streams} host threads, one image each"),
        "setup_s": round(setup, 2),
        # hoisted rotations (csrc/hoist.h, the engine default): rotations of one input in one batched
        # call share one ModUp; counted over the batch
        "hoisted_rotations_batch": hoisted,
        "hoisted_mac_launches_batch": hoist_macs,
        # device scratch the engine holds after the batch (per-stream workspaces, hoisting buffers,
        # Galois mask tables), beyond keys and ciphertexts (mhe_scratch_bytes)
        "scratch_GB": round(scratch / 1e9, 2),
        "device_mem_used_GB": mem,
        "galois_keys": info["galois_keys"],
        "galois_key_GB_resident": round(info["galois_key_gb"], 2),
        "key_format": ("prepared (mhe_key_prepare: residues of primes < 2^51 as doubles)" if prepared else "SEAL layout")
        + "; key bytes below in SEAL's layout",
        # design facts of the runner, not measurements: every planned key is made before the first
        # image and stays resident in HBM (no eviction tier at 65 GB of 288), and the evaluation keys
        # hold no secret key
        "key_residency": "design: all planned keys resident, none streamed from the host per image",
        "key_seed": seed if seed else "fresh keys from OS entropy (SEAL's default)",
        "logit_check": {
            "vs": "plain network with the encrypted network's minimax-composite ReLU (plain_logits_approx): the "
                  "encryption's error alone; sanity: the exact-ReLU plain network",
            "tol_rel_vs_approx_relu": RESNET_CKKS_TOL[layers],
            "tol_rel_vs_exact_relu": RESNET_EXACT_TOL[layers],
            "max_abs_err_per_image": errs,
            "other_key_draws": draws,
        },
        "fallbacks": fallbacks,
        # ResNet roofline: the key-switching key bytes one image streams (the algorithmic bytes of its
        # dominant work, every key switch reading its L x 2 x (L+1)-limb key slice) over its 1-stream time
        "roofline": {
            "bound": "hbm",
            "key_bytes_per_image": key_bytes,
            "achieved": round(key_bytes / sec_one / 1e9, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(key_bytes / sec_one / 1e9 / HBM_PEAK_GBS, 4),
        },
        "key_sharing": shared if shared else "single GPU: keys generated here",
        "ops_per_image": ops,
        "labels": [int(x) for x in batch["labels"]],
        "reference_cpu_sec_per_image": RESNET20_CPU_S if layers == 20 else None,
    }


def broadcast_key(key, src=0):
    """One-time evaluation-key broadcast from `src` to every rank (RCCL over xGMI on the GPU
    box; any backend works).  No-op on a single process."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(key, src=src)
    return key


def max_over_ranks(seconds, device):
    """Max of a per-rank elapsed time (the slowest GPU sets the job time)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.tensor([seconds], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())
    return seconds


class HMultWorkload:
    """The timed workload of the HMult leg, built exactly once and shared with
    tests/test_bench_path.py (which checks every output of these calls against the oracle):
    `batch` independent HMults at L limbs on the C2 chain, one relin key drawn on rank 0 (seeded) and
    broadcast, the engine's prepared key format (or SEAL's), calls of `group` HMults each
    (mhe_hmult_batch) dealt round robin over `streams` HIP streams."""

    def __init__(self, dev, rank=0, limbs=44, batch=32, group=8, streams=4, key_format="prepared", keep_host=False):
        self.dev, self.L, self.B = dev, limbs, batch
        self.moduli = mhe.coeff_modulus_create(1 << LOG_N, C2_BITS)
        K = self.K = len(self.moduli)
        L = limbs
        assert 2 <= L <= K - 1
        self.eng = eng = mhe.Engine(LOG_N, self.moduli, device=dev.index or 0)
        n = self.n = eng.n
        q_t = torch.tensor(self.moduli, dtype=torch.int64, device=dev)
        gen = torch.Generator(device=dev)
        gen.manual_seed(20261015 + rank)
        # relin key: rank 0 draws it, RCCL broadcast to every GPU
        self.key = key = torch.empty((K - 1, 2, K, n), dtype=torch.int64, device=dev)
        if rank == 0:
            g0 = torch.Generator(device=dev)
            g0.manual_seed(7)
            key.copy_(rand_residues((K - 1, 2, K, n), q_t, g0))
        broadcast_key(key, src=0)
        # SEAL-layout host copy of the key for the oracle check (taken before the in-place prepare)
        self.key_host = key.cpu().numpy().view(np.uint64) if keep_host else None
        self.prepared = key_format == "prepared"
        if self.prepared:  # one-time conversion to the engine's key format, outside the timed region
            eng.key_prepare(key)
            torch.cuda.synchronize(dev)
        self.a = rand_residues((batch, 2, L, n), q_t[:L], gen)
        self.b = rand_residues((batch, 2, L, n), q_t[:L], gen)
        self.out = torch.empty((batch, 2, L - 1, n), dtype=torch.int64, device=dev)
        self.stream = torch.cuda.current_stream(dev)
        self.streams = [self.stream] + [torch.cuda.Stream(dev) for _ in range(streams - 1)]
        self.sps = [mhe.ctypes.c_void_p(s_.cuda_stream) for s_ in self.streams]
        for s_ in self.sps:
            mhe.lib().mhe_ctx_reserve(eng._h, K - 1, s_)
        ptr = lambda t: mhe.ctypes.c_void_p(t.data_ptr())  # noqa: E731
        a_p = [ptr(self.a[i]) for i in range(batch)]
        b_p = [ptr(self.b[i]) for i in range(batch)]
        o_p = [ptr(self.out[i]) for i in range(batch)]
        self.k_p = ptr(key)
        self.G = G = max(1, group)
        # calls of G independent HMults each (mhe_hmult_batch: one batched key switch per call whose
        # entries share the relin key stream), dealt round robin over the streams
        arr = lambda ps: (mhe.ctypes.c_void_p * len(ps))(*ps)  # noqa: E731
        self.calls = [(i0, min(G, batch - i0), arr(a_p[i0:i0 + G]), arr(b_p[i0:i0 + G]), arr(o_p[i0:i0 + G]))
                      for i0 in range(0, batch, G)]

    def call_streams(self):
        """[(first entry, count, stream index)] of the calls one step issues."""
        return [(i0, cnt, ci % len(self.sps)) for ci, (i0, cnt, _, _, _) in enumerate(self.calls)]

    def run_calls(self, stream_list=None):
        stream_list = stream_list or self.sps
        for ci, (_, cnt, ca, cb, co) in enumerate(self.calls):
            st = stream_list[ci % len(stream_list)]
            if self.G == 1:
                rc = self.eng.hmult_raw(ca[0], cb[0], self.k_p, self.K, co[0], self.L, st)
            else:
                rc = self.eng.hmult_batch_raw(cnt, ca, cb, self.k_p, self.K, co, self.L, st)
            if rc:
                raise mhe.MheError(rc, mhe.lib().mhe_last_error().decode())

    def step(self):
        stream, streams = self.stream, self.streams
        if len(streams) > 1:  # the extra streams start after the main stream's prior work
            ev = torch.cuda.Event()
            ev.record(stream)
            for s_ in streams[1:]:
                s_.wait_event(ev)
        self.run_calls()
        if len(streams) > 1:  # join back so the timing events on the main stream cover all
            for s_ in streams[1:]:
                ev = torch.cuda.Event()
                ev.record(s_)
                stream.wait_event(ev)

    def host(self, t):
        return t.cpu().numpy().view(np.uint64)


def check_timed_outputs(w, entries, threads):
    """Recompute `entries` of the timed HMults with the oracle (test infrastructure, used here only as
    the checker) on the same inputs and the SEAL-layout key, and require identical words."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    oc = O.Context(LOG_N, w.moduli)
    idx = list(entries)
    a = np.ascontiguousarray(w.host(w.a[idx]))
    b = np.ascontiguousarray(w.host(w.b[idx]))
    got = w.host(w.out[idx])
    t0 = time.perf_counter()
    want, _ = oc.hmult_batch(a, b, w.key_host, threads=min(threads, len(idx)))
    dt = time.perf_counter() - t0
    bad = [i for j, i in enumerate(idx) if not np.array_equal(got[j], want[j])]
    if bad:
        raise AssertionError(f"timed HMult outputs {bad} differ from the oracle")
    return {"entries": idx, "calls_streams": [c for c in w.call_streams() if any(c[0] <= i < c[0] + c[1] for i in idx)],
            "vs": "oracle/mhe_oracle.c hmult (SEAL evaluator restatement), SEAL-layout key", "oracle_s": round(dt, 2)}


def launch_ranks(args):
    """`--gpus N` without a launcher: start N worker processes of this script (one per GPU, RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* set) and exit with the first failing child's code.  This
    process touches no GPU (import torch does not; no device is counted or opened here), so the
    workers own the devices."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        p.wait()
        if p.returncode and not rc:
            rc = p.returncode
    if rc:  # a failed rank can leave the others waiting in a collective
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc


def stub_worker(args, world, rank):
    """--stub: the launcher's rank plumbing without a GPU (gloo): every rank checks WORLD_SIZE
    against --gpus and joins one all-reduce; rank 0 prints the ranks seen (tests/test_dist.py)."""
    dist.init_process_group("gloo")
    assert dist.get_world_size() == world == args.gpus, (dist.get_world_size(), world, args.gpus)
    t = torch.tensor([1.0 + rank])
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"n_gpus": world, "backend": dist.get_backend(), "ranks_seen": dist.get_world_size(),
                          "rank_sum": float(t.item())}), flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=32, help="independent HMults per GPU per step")
    ap.add_argument("--limbs", type=int, default=44)
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="host cores for the CPU baseline (16 = one GPU's share of the box's CPUs)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--resnet-images", type=int, default=24,
                    help="ResNet-20 CIFAR-10 images per GPU for the sec/image leg (0 = skip)")
    ap.add_argument("--resnet-layers", type=int, default=20, choices=(20, 110),
                    help="20: config C3 (ResNet-20); 110: config C4's network (ResNet-110, one image per GPU "
                         "with --resnet-images 1 --resnet-streams 1)")
    # 3 x 8 measured best on one MI355X (profiles/r05g_resnet_batch_shapes.txt: 1.43 images/s vs 1.30 at
    # 2 x 4, 1.36 at 2 x 8, 1.18 at 4 x 8): 8 fibers fill a batched launch (MHE_MAXB), a third stream
    # overlaps the small passes of the other two
    ap.add_argument("--resnet-streams", type=int, default=3, help="host threads for the ResNet batch (one stream each)")
    ap.add_argument("--resnet-fibers", type=int, default=8,
                    help="images per host thread at a time as one seal::FiberBatch (1 = one image per thread)")
    ap.add_argument("--resnet-seed", type=int, default=0,
                    help="ResNet runner's reproducible seed sequence (0: fresh keys from OS entropy)")
    ap.add_argument("--resnet-key-draws", type=int, default=2,
                    help="extra fresh key sets (2 images each) for the logit error's spread over keys (N=1)")
    ap.add_argument("--c4", choices=("auto", "on", "off"), default="auto",
                    help="config C4 leg (ResNet-110, one image per GPU on the shared key set); auto = when N > 1")
    ap.add_argument("--key-format", choices=("prepared", "seal"), default="prepared",
                    help="relin key as the engine's prepared format (mhe_key_prepare, the residues of primes "
                         "< 2^51 as doubles; bit-identical results) or SEAL's u64 layout")
    ap.add_argument("--hmult-group", type=int, default=8,
                    help="HMults per mhe_hmult_batch call (one batched key switch sharing the relin key "
                         "stream; 1 = one mhe_hmult call each)")
    ap.add_argument("--streams", type=int, default=4,
                    help="HIP streams the batch is spread over (round robin; 4 = the hardware queues per process)")
    ap.add_argument("--stub", action="store_true", help="rank plumbing only, on gloo without a GPU (tests)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    if args.stub:
        return stub_worker(args, world, rank)
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
        assert dist.get_world_size() == args.gpus
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    L = args.limbs
    check = rank == 0 and not args.no_cpu  # keep the SEAL-layout key on the host for the output check
    w = HMultWorkload(dev, rank, L, args.batch, args.hmult_group, args.streams, args.key_format, keep_host=check)
    eng, n, moduli, B, G = w.eng, w.n, w.moduli, w.B, w.G
    stream, sps = w.stream, w.sps
    lib = mhe.lib()
    lib.mhe_ctx_set_timing(eng._h, 1)
    for _ in range(args.warmup):
        w.step()
    torch.cuda.synchronize(dev)
    km_ms, km_n = mhe.ctypes.c_double(), mhe.ctypes.c_int()
    mc_ms, mc_n = mhe.ctypes.c_double(), mhe.ctypes.c_int()  # k_modup_col, the second key-switch kernel
    lib.mhe_kernel_time(eng._h, 0, mhe.ctypes.byref(km_ms), mhe.ctypes.byref(km_n))  # drop the warmup launches
    lib.mhe_kernel_time(eng._h, 1, mhe.ctypes.byref(mc_ms), mhe.ctypes.byref(mc_n))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        w.step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    gpu_s = ev0.elapsed_time(ev1) / 1e3
    elapsed = max_over_ranks(max(wall, gpu_s), dev)
    # the timed calls' outputs, checked against the oracle on rank 0 (one entry per call, so every
    # stream and batch position class is covered), before the single-stream pass below rewrites them
    timed_check = None
    if check:
        entries = sorted({i0 + (ci * 3) % cnt for ci, (i0, cnt, _) in enumerate(w.call_streams())})
        timed_check = check_timed_outputs(w, entries, args.cpu_threads)
    # HIP-event time of the dominant kernel, recorded by the engine on the stream each launch
    # ran on (mhe_ctx_set_timing / mhe_kernel_time).  With several streams the launches of
    # different HMults overlap, so the kernel's own duration is taken from a short
    # single-stream pass after the timed region (the rocprofv3 summary under profiles/ is of
    # the same single-stream command: bench.py --streams 1).
    lib.mhe_kernel_time(eng._h, 0, mhe.ctypes.byref(km_ms), mhe.ctypes.byref(km_n))
    lib.mhe_kernel_time(eng._h, 1, mhe.ctypes.byref(mc_ms), mhe.ctypes.byref(mc_n))
    if len(sps) > 1:
        for _ in range(min(args.steps, 4)):
            w.run_calls(sps[:1])
        torch.cuda.synchronize(dev)
        lib.mhe_kernel_time(eng._h, 0, mhe.ctypes.byref(km_ms), mhe.ctypes.byref(km_n))
        lib.mhe_kernel_time(eng._h, 1, mhe.ctypes.byref(mc_ms), mhe.ctypes.byref(mc_n))
    km_avg_us = km_ms.value * 1e3 / max(km_n.value, 1)
    mc_avg_us = mc_ms.value * 1e3 / max(mc_n.value, 1)

    # HBM traffic per HMult from the committed PMC passes of the same workload (rocprofv3
    # FETCH_SIZE/WRITE_SIZE, gfx950-corrected; scripts/gpu_round.sh + scripts/traffic.py)
    traffic, traffic_src, km_traffic = None, None, None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic.json"))):
        try:
            t = json.load(open(f))
            if t.get("limbs", L) == L:
                traffic, traffic_src = t["hbm_bytes_per_hmult"], os.path.relpath(f, ROOT)
                pk = {k.split("<")[0]: v for k, v in t.get("per_kernel_GB_per_hmult", {}).items()}
                km_traffic = pk.get("k_ks_row_mac")
                km_traffic = None if km_traffic is None else km_traffic * 1e9 * min(G, B)  # G HMults per launch
        except (OSError, ValueError, KeyError):
            pass

    # SQ counters of the same workload (rocprofv3 --pmc SQ_INSTS_VALU ..., scripts/gpu_pmc.sh)
    sq_valu, sq_src = None, None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_sq_counters.json"))):
        try:
            t = json.load(open(f))
            if t.get("limbs", L) == L and "k_ks_row_mac" in t.get("SQ_INSTS_VALU", {}):
                sq_valu, sq_src = t["SQ_INSTS_VALU"]["k_ks_row_mac"], os.path.relpath(f, ROOT)
        except (OSError, ValueError, KeyError):
            pass

    hmults_per_gpu = B * args.steps
    value = world * hmults_per_gpu / elapsed
    per_hmult_s = gpu_s / hmults_per_gpu  # HIP-event time per HMult (batch over its streams)
    # algorithmic bytes as SURVEY.md §8(d) defines them (SEAL's u64 key layout); a prepared key
    # streams fewer (streamed_key_bytes_per_launch), which is what the format buys
    # one launch covers G HMults (mhe_hmult_batch): the key slice once, and every entry's target
    # limbs read ([L][n]) and key inner products written ([2][L+1][n])
    G_launch = min(G, B)
    io_bytes = G_launch * (L + 2 * (L + 1)) * n * 8
    km_bytes = ks_row_mac_key_bytes(L, n) + io_bytes
    km_streamed = ks_row_mac_key_bytes(L, n, moduli, w.prepared) + io_bytes
    hm_bytes = hmult_bytes(L)
    achieved = hm_bytes / per_hmult_s / 1e9
    km_achieved = km_bytes / (km_avg_us * 1e-6) / 1e9 if km_avg_us > 0 else 0.0
    result = {
        "metric": "homomorphic ciphertext mults/sec (N=2^16, L limbs)",
        "value": round(value, 3),
        "unit": "HMult/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64 residues, exact fp64-FMA modular arithmetic",
        "data": "synthetic: uniform RNS residues (mt-style seeded) + random relin key, NTT form",
        "config": {
            "workload": "C2: N=2^16 45-prime chain (44 data limbs + special), HMult = multiply+relinearize+rescale",
            "log_n": LOG_N,
            "limbs": L,
            "batch_per_gpu": B,
            "hmults_per_call": G,
            "call": "mhe_hmult_batch" if G > 1 else "mhe_hmult",
            "streams": args.streams,
            "parallelism": f"replicas{world} (independent ciphertexts per GPU, key broadcast over RCCL)",
            "ranks": (dist.get_world_size() if world > 1 else 1),
            "backend": (dist.get_backend() if world > 1 else None),
        },
        # rank 0 recomputed entries of the timed calls (the last step's outputs, one entry per
        # mhe_hmult_batch call / stream) with the oracle on the same inputs: identical words
        "timed_output_checked": timed_check is not None,
        "timed_output_check": timed_check,
        "roofline": {
            "bound": "hbm",
            "kernel": (f"k_ks_row_mac (fused ModUp row pass + key inner products; one launch per {G_launch} HMults "
                       "sharing the relin key stream)"),
            "hmults_per_launch": G_launch,
            "bytes_model": "relin key slice once per launch + per HMult: target limbs read, key products written",
            "achieved": round(km_achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(km_achieved / HBM_PEAK_GBS, 4),
            "traffic": km_traffic,
            "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE, gfx950-corrected)",
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_launch": km_bytes,
            "key_format": args.key_format,
            "streamed_key_bytes_per_launch": km_streamed,
            "avg_launch_us": round(km_avg_us, 2),
            "modup_col_avg_launch_us": round(mc_avg_us, 2),
            "launches_timed": km_n.value,
            "timing": "HIP events around each launch on its stream; single-stream pass when --streams > 1",
            # with one key stream shared by G_launch HMults the kernel moves few bytes per HMult and is
            # bound by FP64 VALU issue instead: valu_roofline (model lane-ops; SQ_INSTS_VALU when
            # committed) is the binding fraction, this HBM fraction only the bytes it moves
            "binding_resource": "valu" if G_launch > 1 else "hbm",
        },
        # the same kernel against the FP64 VALU issue rate ("also report the int-VALU
        # bound"; the engine's modular arithmetic runs on the FP64 pipe, csrc/fparith.h)
        "valu_roofline": (lambda v: {
            "bound": "valu",
            "kernel": "k_ks_row_mac",
            "model": "L^2*8*n/2 butterflies x 8 (q<2^47) or 11 FP64 lane-ops + 2L(L+1)n MACs x 7",
            **v,
            "peak_lane_ops_per_s": FP64_LANE_OPS_PEAK,
            "peak_source": "v_fma_f64 microbenchmark, profiles/r01_ubench_valu.txt (spec 39.3e12)",
            "floor_us": round(G_launch * v["fp64_lane_ops"] / FP64_LANE_OPS_PEAK * 1e6, 2),
            "frac": (round(G_launch * v["fp64_lane_ops"] / FP64_LANE_OPS_PEAK / (km_avg_us * 1e-6), 4)
                     if km_avg_us > 0 else None),
            "hmults_per_launch": G_launch,
            "sq_insts_valu_per_launch": sq_valu,
            "issued_lane_ops_frac": (round(sq_valu * 64 / FP64_LANE_OPS_PEAK / (km_avg_us * 1e-6), 4)
                                     if sq_valu and km_avg_us > 0 else None),
            "sq_source": sq_src,
        })(ks_row_mac_valu(L, n, moduli)),
        "hmult_roofline": {
            "bound": "hbm",
            "unit_of_work": "one HMult (tensor + key switch + rescale kernel sequence)",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_unit": "HBM bytes per HMult (PMC)",
            "algorithmic_bytes_per_hmult": hm_bytes,
            "us_per_hmult": round(per_hmult_s * 1e6, 2),
        },
    }
    # the HMult leg's engine (its per-stream workspaces: 8 entries at 44 limbs each) and buffers are
    # not needed by the ResNet legs: destroyed here, not left to the garbage collector
    torch.cuda.synchronize(dev)
    w.eng.close()
    del w
    torch.cuda.empty_cache()
    legs = []
    if args.resnet_images > 0:
        legs.append((args.resnet_layers, args.resnet_images, args.resnet_streams, args.resnet_fibers))
    if args.c4 == "on" or (args.c4 == "auto" and world > 1):
        legs.append((110, 1, 1, 1))  # config C4: ResNet-110, one image per GPU, shared key set
    for layers, images, streams, fibers in legs:
        r = resnet_leg(local, images, streams, layers, fibers, seed=args.resnet_seed,
                       key_draws=args.resnet_key_draws if layers == 20 and world == 1 else 0)
        t = torch.tensor([r["batch_wall_s"], r["sec_per_image_1stream"]], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        r["batch_wall_s"], r["sec_per_image_1stream"] = float(t[0]), float(t[1])
        r["images_per_s"] = round(world * images / r["batch_wall_s"], 4)
        r["n_gpus"] = world
        if layers == 20:
            r["vs_reference_cpu"] = round(RESNET20_CPU_S / r["sec_per_image_1stream"], 1)
        result[f"resnet{layers}"] = r
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(moduli, L, args.cpu_threads)
        for layers in (20, 110):
            r = result.get(f"resnet{layers}")
            if r and r.get("ops_per_image"):
                est = resnet_cpu_estimate(r["ops_per_image"], result["cpu_baseline"]["cores"])
                est["vs_gpu_1stream"] = round(est["estimated_cpu_s_per_image"] / r["sec_per_image_1stream"], 1)
                r["cpu_estimate"] = est
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
