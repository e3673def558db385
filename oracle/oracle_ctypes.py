"""ctypes view of the CPU oracle (TEST INFRASTRUCTURE — never imported by the product path).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
It wraps oracle/liboracle_{f32,f64}.so, the C restatement of /root/reference/train_vit.rs
(see oracle/oracle.h for the provenance and the defect fixes applied).
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

PARAM_NAMES = ["patch_w", "patch_b", "cls", "wpe",
               "ln1w", "ln1b", "qkvw", "qkvb", "attprojw", "attprojb",
               "ln2w", "ln2b", "fcw", "fcb", "fcprojw", "fcprojb",
               "lnfw", "lnfb", "head_w", "head_b"]


class VitConfig(ctypes.Structure):
    _fields_ = [("img", ctypes.c_int), ("patch", ctypes.c_int), ("in_ch", ctypes.c_int),
                ("channels", ctypes.c_int), ("num_layers", ctypes.c_int),
                ("num_heads", ctypes.c_int), ("num_classes", ctypes.c_int)]


def build(quiet=True):
    """Compile the oracle (gcc) in place."""
    import subprocess
    subprocess.run(["make", "-s", "-C", HERE], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)


class Oracle:
    """Thin numpy wrapper over one precision build of the oracle."""

    def __init__(self, precision="f32"):
        path = os.path.join(HERE, f"liboracle_{precision}.so")
        if not os.path.exists(path):
            build()
        self.lib = ctypes.CDLL(path)
        self.dtype = np.float32 if precision == "f32" else np.float64
        self.ctype = ctypes.c_float if precision == "f32" else ctypes.c_double
        L = self.lib
        P = ctypes.c_void_p
        i = ctypes.c_int
        L.ref_vit_create.restype = P
        L.ref_vit_create.argtypes = [ctypes.POINTER(VitConfig), i]
        L.ref_vit_destroy.argtypes = [P]
        L.ref_vit_forward.restype = self.ctype
        L.ref_vit_forward.argtypes = [P, P, P, P, i]
        L.ref_vit_backward.argtypes = [P, P, P]
        for n in ("ref_vit_logits", "ref_vit_losses", "ref_vit_probs", "ref_vit_encoded"):
            getattr(L, n).restype = P
            getattr(L, n).argtypes = [P]
        L.ref_vit_param_sizes.restype = ctypes.c_longlong
        L.ref_vit_param_sizes.argtypes = [ctypes.POINTER(VitConfig), P]
        L.ref_sgd_step.argtypes = [P, P, ctypes.c_longlong, self.ctype]
        L.ref_adamw_step.argtypes = [P, P, P, P, ctypes.c_longlong] + [self.ctype] * 5 + [ctypes.c_int]
        L.ref_set_num_threads.argtypes = [i]
        L.ref_get_num_threads.restype = i

    def set_num_threads(self, n):
        """OpenMP team size of the oracle's parallel loops (1 = the single-thread reference timing)."""
        self.lib.ref_set_num_threads(int(n))
        return int(self.lib.ref_get_num_threads())

    # -- helpers --------------------------------------------------------------------------
    def _p(self, a):
        if a is None:
            return None
        assert a.flags.c_contiguous, "oracle arrays must be C-contiguous"
        return a.ctypes.data_as(ctypes.c_void_p)

    def arr(self, a):
        return np.ascontiguousarray(a, dtype=self.dtype)

    def call(self, name, *args):
        """Call ref_<name> with numpy arrays / python ints / floats."""
        cargs = []
        for a in args:
            if isinstance(a, np.ndarray):
                cargs.append(self._p(a))
            elif a is None:
                cargs.append(None)
            elif isinstance(a, float):
                cargs.append(self.ctype(a))
            else:
                cargs.append(ctypes.c_int(int(a)))
        getattr(self.lib, "ref_" + name)(*cargs)

    def param_sizes(self, cfg):
        sizes = (ctypes.c_longlong * 20)()
        tot = self.lib.ref_vit_param_sizes(ctypes.byref(cfg), ctypes.cast(sizes, ctypes.c_void_p))
        return [int(s) for s in sizes], int(tot)

    def sgd_step(self, params, grads, lr):
        self.lib.ref_sgd_step(self._p(params), self._p(grads), params.size, self.ctype(lr))

    def adamw_step(self, params, grads, m, v, lr, beta1, beta2, eps, wd, t):
        self.lib.ref_adamw_step(self._p(params), self._p(grads), self._p(m), self._p(v), params.size,
                                *(self.ctype(x) for x in (lr, beta1, beta2, eps, wd)), int(t))


class RefViT:
    """Model-level oracle: ViT::forward / ViT::backward of train_vit.rs:188-373."""

    def __init__(self, oracle, cfg, B):
        self.o = oracle
        self.cfg = cfg
        self.B = B
        self.NP = (cfg.img // cfg.patch) ** 2
        self.T = self.NP + 1
        self.h = oracle.lib.ref_vit_create(ctypes.byref(cfg), B)
        self._keep = []

    def __del__(self):
        try:
            self.o.lib.ref_vit_destroy(self.h)
        except Exception:
            pass

    def forward(self, params, pixels, targets, B_global=None):
        pixels = self.o.arr(pixels)
        targets = None if targets is None else np.ascontiguousarray(targets, dtype=np.int32)
        self._keep = [pixels, targets]  # backward reads pixels/targets again
        return float(self.o.lib.ref_vit_forward(self.h, self.o._p(params), self.o._p(pixels),
                                                self.o._p(targets), B_global or self.B))

    def backward(self, params, grads):
        self.o.lib.ref_vit_backward(self.h, self.o._p(params), self.o._p(grads))

    def _view(self, fn, n):
        ptr = getattr(self.o.lib, fn)(self.h)
        return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(self.o.ctype)), shape=(n,)).copy()

    def logits(self):
        return self._view("ref_vit_logits", self.B * self.cfg.num_classes).reshape(self.B, -1)

    def losses(self):
        return self._view("ref_vit_losses", self.B)

    def probs(self):
        return self._view("ref_vit_probs", self.B * self.cfg.num_classes).reshape(self.B, -1)

    def encoded(self):
        return self._view("ref_vit_encoded", self.B * self.T * self.cfg.channels)


def split_params(oracle, cfg, flat):
    """flat canonical arena -> dict name -> view"""
    sizes, _ = oracle.param_sizes(cfg)
    out, off = {}, 0
    for n, s in zip(PARAM_NAMES, sizes):
        out[n] = flat[off:off + s]
        off += s
    return out
