"""ctypes binding of the encrypted ResNet runner (include/mhe_resnet_capi.h, libmhe_seal.so) and the
key sharing of SURVEY.md §8(e): one key set, made once, used by every GPU.

The reference keeps one key set in one process and fans images out over OpenMP threads
(cnn/infer_seal.cpp:404-577).  Here one process drives one GPU: rank `src` generates the keys
(secret, public, relinearization and the level-truncated Galois set), every key buffer is copied
into a torch tensor on its GPU and broadcast with torch.distributed (RCCL over xGMI on the box,
gloo on CPU), and each other rank imports the buffers into its own runner.  No collective runs on
the data path; results are gathered once at the end.
"""
import ctypes
import os

import numpy as np

from . import lib as _mhe_lib  # loads libmhe.so (and the HIP runtime order it needs) first

_HERE = os.path.dirname(os.path.abspath(__file__))
_seal = None

KIND_NAMES = {0: "secret", 1: "public", 2: "relin", 3: "galois"}


def seal_lib():
    global _seal
    if _seal is None:
        _mhe_lib()
        L = ctypes.CDLL(os.environ.get("MHE_SEAL_LIB_PATH") or os.path.join(os.path.dirname(_HERE), "libmhe_seal.so"))
        vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
        dp, ip, u64p = ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i32), ctypes.POINTER(u64)
        sig = {
            "mhe_resnet_create": (i32, [ctypes.POINTER(vp), i32, ctypes.c_char_p, ctypes.c_char_p, i32]),
            "mhe_resnet_create_seeded": (i32, [ctypes.POINTER(vp), i32, ctypes.c_char_p, ctypes.c_char_p, i32,
                                               ctypes.c_uint64]),
            "mhe_resnet_destroy": (i32, [vp]),
            "mhe_resnet_last_error": (ctypes.c_char_p, []),
            "mhe_resnet_key_count": (i32, [vp, ip]),
            "mhe_resnet_key_info": (i32, [vp, i32, ip, u64p, u64p, u64p]),
            "mhe_resnet_key_export": (i32, [vp, i32, vp]),
            "mhe_resnet_key_import": (i32, [vp, i32, u64, u64, u64, vp]),
            "mhe_resnet_finish_import": (i32, [vp]),
            "mhe_resnet_infer_batch": (i32, [vp, dp, i32, i32, dp, ip, dp, dp, dp, dp]),
            "mhe_resnet_infer_batch_fibers": (i32, [vp, dp, i32, i32, i32, dp, ip, dp, dp, dp, dp]),
            "mhe_resnet_info": (i32, [vp, dp, dp, ip]),
            "mhe_resnet_key_traffic": (i32, [vp, dp, i32]),
            "mhe_resnet_op_counts": (i32, [vp, i32, u64p, i32]),
            "mhe_resnet_key_format": (i32, [vp, ip]),
            "mhe_resnet_set_hoist": (i32, [vp, i32, i32]),
            "mhe_resnet_hoist_stats": (i32, [vp, ctypes.POINTER(ctypes.c_uint64), i32]),
            "mhe_resnet_scratch_bytes": (i32, [vp, ctypes.POINTER(ctypes.c_double)]),
            "mhe_resnet_plain_logits": (i32, [vp, dp, dp]),
            "mhe_resnet_plain_logits_approx": (i32, [vp, dp, dp]),
            "mhe_resnet_fallback_stats": (i32, [ctypes.POINTER(ctypes.c_uint64), i32]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _seal = L
    return _seal


def _check(rc):
    if rc != 0:
        raise RuntimeError(seal_lib().mhe_resnet_last_error().decode())


class Runner:
    """One ResNet runner on the calling process's GPU (MHE_DEVICE selects it)."""

    def __init__(self, layers, params_bin, comp_dir, generate_keys=True, seed=0):
        """seed != 0: the runner's PRNG (keys, encryption) is seeded, so runs repeat (0: random)."""
        h = ctypes.c_void_p()
        _check(seal_lib().mhe_resnet_create_seeded(ctypes.byref(h), layers, params_bin.encode(), comp_dir.encode(),
                                                   1 if generate_keys else 0, int(seed)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            seal_lib().mhe_resnet_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ keys
    def key_blobs(self):
        """[(kind, index, limbs, words)] of the exported key buffers."""
        n = ctypes.c_int()
        _check(seal_lib().mhe_resnet_key_count(self._h, ctypes.byref(n)))
        out = []
        for i in range(n.value):
            k, idx, limbs, words = ctypes.c_int(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
            _check(seal_lib().mhe_resnet_key_info(self._h, i, ctypes.byref(k), ctypes.byref(idx), ctypes.byref(limbs),
                                                  ctypes.byref(words)))
            out.append((k.value, idx.value, limbs.value, words.value))
        return out

    def export_key(self, i, dst_ptr):
        _check(seal_lib().mhe_resnet_key_export(self._h, i, ctypes.c_void_p(dst_ptr)))

    def import_key(self, kind, index, limbs, words, src_ptr):
        _check(seal_lib().mhe_resnet_key_import(self._h, kind, index, limbs, words, ctypes.c_void_p(src_ptr)))

    def finish_import(self):
        _check(seal_lib().mhe_resnet_finish_import(self._h))

    # ------------------------------------------------------------------ inference
    def infer_batch(self, images, threads, fibers=0):
        """images: [B][3072] doubles -> dict(logits [B][10], labels [B], seconds, boot, relu, wall).
        fibers > 1: that many images per host thread at a time as one seal::FiberBatch."""
        imgs = np.ascontiguousarray(images, dtype=np.float64)
        B = imgs.shape[0]
        logits = np.zeros((B, 10))
        labels = np.zeros(B, np.int32)
        sec, boot, relu = np.zeros(B), np.zeros(B), np.zeros(B)
        wall = ctypes.c_double()
        dp = ctypes.POINTER(ctypes.c_double)
        _check(seal_lib().mhe_resnet_infer_batch_fibers(
            self._h, imgs.ctypes.data_as(dp), B, threads, fibers, logits.ctypes.data_as(dp),
            labels.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), sec.ctypes.data_as(dp), boot.ctypes.data_as(dp),
            relu.ctypes.data_as(dp), ctypes.byref(wall)))
        return {"logits": logits, "labels": labels, "seconds": sec, "boot": boot, "relu": relu, "wall": wall.value}

    def key_traffic(self, reset=False):
        """Key-switching key bytes streamed since the last reset."""
        b = ctypes.c_double()
        _check(seal_lib().mhe_resnet_key_traffic(self._h, ctypes.byref(b), 1 if reset else 0))
        return b.value

    OP_KINDS = ("keyswitch", "rescale", "tensor", "mulplain", "addsub", "scalar", "ntt", "galois")  # MHE_OPK_*

    def op_counts(self, reset=False):
        """{kind: [count per level 0..63]} of the operations run since the last reset (mhe_op_counts:
        key switches per entry, the elementwise kinds per polynomial)."""
        out = {}
        for k, name in enumerate(self.OP_KINDS):
            c = (ctypes.c_uint64 * 64)()
            _check(seal_lib().mhe_resnet_op_counts(self._h, k, c, 1 if reset else 0))
            out[name] = [int(x) for x in c]
        return out

    def set_hoist(self, on, check=False):
        _check(seal_lib().mhe_resnet_set_hoist(self._h, 1 if on else 0, 1 if check else 0))

    def hoist_stats(self, reset=False):
        """(hoisted rotations, hoisted key-MAC launches, words differing under check) since reset."""
        v = (ctypes.c_uint64 * 3)()
        _check(seal_lib().mhe_resnet_hoist_stats(self._h, v, 1 if reset else 0))
        return tuple(int(x) for x in v)

    def scratch_bytes(self):
        b = ctypes.c_double()
        _check(seal_lib().mhe_resnet_scratch_bytes(self._h, ctypes.byref(b)))
        return b.value

    def keys_prepared(self):
        """True when the evaluation keys are in the engine's prepared format (mhe_key_prepare)."""
        p = ctypes.c_int()
        _check(seal_lib().mhe_resnet_key_format(self._h, ctypes.byref(p)))
        return bool(p.value)

    def plain_logits(self, image):
        """The network in plain doubles (exact ReLU) on one 3072-value image -> 10 logits."""
        img = np.ascontiguousarray(image, dtype=np.float64).reshape(3072)
        out = np.zeros(10)
        dp = ctypes.POINTER(ctypes.c_double)
        _check(seal_lib().mhe_resnet_plain_logits(self._h, img.ctypes.data_as(dp), out.ctypes.data_as(dp)))
        return out

    def plain_logits_approx(self, image):
        """The network in plain doubles with the encrypted network's minimax-composite ReLU."""
        img = np.ascontiguousarray(image, dtype=np.float64).reshape(3072)
        out = np.zeros(10)
        dp = ctypes.POINTER(ctypes.c_double)
        _check(seal_lib().mhe_resnet_plain_logits_approx(self._h, img.ctypes.data_as(dp), out.ctypes.data_as(dp)))
        return out

    @staticmethod
    def fallback_stats(reset=False):
        """(merged calls re-run member by member, allocations retried after a cache release, failed
        allocations), process-wide since the last reset: all 0 in a healthy run."""
        v = (ctypes.c_uint64 * 3)()
        _check(seal_lib().mhe_resnet_fallback_stats(v, 1 if reset else 0))
        return tuple(int(x) for x in v)

    def check_logits(self, images, logits, tol=0.05):
        """Decrypted logits vs the plain network: max |error| per image must stay below
        tol * max(1, max |plain logit|) (tests/cpp/resnet_test.cpp's band for ResNet-20; 0.08 is
        used for the deeper networks).  Returns (max relative error, [per-image errors]); raises on a miss."""
        errs = []
        for img, got in zip(images, logits):
            want = self.plain_logits(img)
            err = float(np.max(np.abs(np.asarray(got) - want)))
            bound = tol * max(1.0, float(np.max(np.abs(want))))
            errs.append(round(err, 5))
            if not err < bound:
                raise RuntimeError(f"encrypted ResNet logits off the plain network: max |error| {err:.4g} >= {bound:.4g}")
        return errs

    def info(self):
        s, gb, nk = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        _check(seal_lib().mhe_resnet_info(self._h, ctypes.byref(s), ctypes.byref(gb), ctypes.byref(nk)))
        return {"setup_s": s.value, "galois_key_gb": gb.value, "galois_keys": nk.value}


def share_keys(dist, source, device, src=0, export=None, import_=None, finish=None):
    """Broadcast one key set from rank `src` to every rank, one buffer at a time (so the extra HBM is
    one key, <= 1 GB).  `source` on rank src is a Runner (or any object with key_blobs/export_key);
    on the other ranks it is the Runner that receives (import_key/finish_import).  `export`,
    `import_`, `finish` override the runner methods (the CPU test drives host buffers with them).
    Returns (buffers, bytes) moved."""
    import torch

    rank = dist.get_rank()
    meta = [source.key_blobs() if rank == src else None]
    dist.broadcast_object_list(meta, src=src)
    blobs = meta[0]
    export = export or (lambda i, t: source.export_key(i, t.data_ptr()))
    import_ = import_ or (lambda b, t: source.import_key(b[0], b[1], b[2], b[3], t.data_ptr()))
    total = 0
    for i, b in enumerate(blobs):
        t = torch.empty(b[3], dtype=torch.int64, device=device)
        if rank == src:
            export(i, t)
        dist.broadcast(t, src=src)
        if rank != src:
            if t.is_cuda:
                torch.cuda.synchronize(t.device)  # the runner copies on its own stream
            import_(b, t)
        total += b[3] * 8
    if rank != src:
        (finish or source.finish_import)()
    return len(blobs), total
