"""vit.rs_amd — MI355X-native ViT training step: host-side mirror of the reference interface.

The product is libvit_hip.so (csrc/: gfx950 HIP kernels, the C ABI of include/vit_ops.h and the
native trainer of include/vit_trainer.h).  This module is the thin Python host over that C ABI
(ctypes, no torch types), mirroring the reference's model interface (/root/reference/
train_vit.rs: `ViT::build_from_checkpoint`, `forward`, `backward`, `optimizer_step`,
`mean_loss`) so tests and the benchmark read like the reference's own code.

There is no CPU fallback: if libvit_hip.so is missing or cannot be loaded, every entry point
raises.  If torch is used in the same process, import it BEFORE this package so that the
HIP runtime torch ships is the single runtime in the process.
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VIT_LIB") or os.path.join(HERE, "libvit_hip.so")  # VIT_LIB: A/B builds

from . import data  # noqa: E402  (configs, canonical layout, seeded synthetic inputs)

VIT_FP32, VIT_BF16, VIT_FP8 = 0, 1, 2
_lib = None


class VitError(RuntimeError):
    pass


class VitConfigC(ctypes.Structure):
    _fields_ = [("img", ctypes.c_int), ("patch", ctypes.c_int), ("in_ch", ctypes.c_int),
                ("channels", ctypes.c_int), ("num_layers", ctypes.c_int),
                ("num_heads", ctypes.c_int), ("num_classes", ctypes.c_int)]


class AdamWC(ctypes.Structure):
    _fields_ = [("beta1", ctypes.c_float), ("beta2", ctypes.c_float), ("eps", ctypes.c_float),
                ("weight_decay", ctypes.c_float)]


class CheckpointInfoC(ctypes.Structure):
    _fields_ = [("cfg", VitConfigC), ("num_params", ctypes.c_longlong), ("has_opt", ctypes.c_int),
                ("step", ctypes.c_int), ("adamw", AdamWC)]


def _cfg_c(cfg):
    return VitConfigC(cfg.img, cfg.patch, cfg.in_ch, cfg.channels, cfg.num_layers, cfg.num_heads,
                      cfg.num_classes)


def build(quiet=True):
    """Compile libvit_hip.so in place (hipcc, gfx950)."""
    import subprocess
    jobs = str(min(8, os.cpu_count() or 1))
    subprocess.run(["make", "-s", "-j", jobs, "-C", HERE], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)


_VOID = [("vit_clear_error", []), ("vit_set_stream", [ctypes.c_void_p]),
         ("vit_free", [ctypes.c_void_p]), ("vit_event_destroy", [ctypes.c_void_p]),
         ("vit_trainer_destroy", [ctypes.c_void_p]), ("vit_trainer_timing_reset", [ctypes.c_void_p]),
         ("vit_loader_close", [ctypes.c_void_p]), ("vit_jpeg_loader_close", [ctypes.c_void_p]), ("vit_kernel_hits_reset", [])]

# name -> (restype, argtypes)
P, I, LL, F, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_float, ctypes.c_size_t
_SIGS = {
    "vit_init": (I, [I]), "vit_get_stream": (P, []), "vit_sync": (I, []),
    "vit_last_error": (I, [ctypes.POINTER(ctypes.c_char_p)]),
    "vit_malloc": (P, [S]), "vit_memcpy_h2d": (I, [P, P, S]), "vit_memcpy_d2h": (I, [P, P, S]),
    "vit_memcpy_d2d": (I, [P, P, S]), "vit_memset": (I, [P, I, S]),
    "vit_event_create": (P, []), "vit_event_record": (I, [P]), "vit_event_elapsed_ms": (F, [P, P]),
    # reference ops (fp32)
    "residual_forward": (None, [P, P, P, I]),
    "matmul_forward": (None, [P, P, P, P, I, I, I, I]),
    "attention_forward": (None, [P, P, P, P, I, I, I, I]),
    "layernorm_forward": (None, [P, P, P, P, P, P, I, I, I]),
    "gelu_forward": (None, [P, P, I]),
    "softmax_forward": (None, [P, P, I, I, I]),
    "crossentropy_forward": (None, [P, P, P, I, I, I]),
    "residual_backward": (None, [P, P, P, I]),
    "matmul_backward": (None, [P, P, P, P, P, P, I, I, I, I]),
    "attention_backward": (None, [P, P, P, P, P, P, I, I, I, I]),
    "layernorm_backward": (None, [P, P, P, P, P, P, P, P, I, I, I]),
    "gelu_backward": (None, [P, P, P, I]),
    "crossentropy_softmax_backward": (None, [P, P, P, P, I, I, I]),
    "patch_embed_forward": (None, [P, P, P, P, P, P, I, I, I, I]),
    "patch_embed_backward": (None, [P, P, P, P, P, P, I, I, I, I]),
    "sgd_step": (None, [P, P, LL, F]),
    # bf16 extensions
    "matmul_forward_bf16": (None, [P, P, P, P, I, I, I, I]),
    "matmul_backward_bf16": (None, [P, P, P, P, P, P, I, I, I, I]),
    "attention_forward_fused_bf16": (None, [P, P, P, I, I, I, I]),
    "vit_attention_kernel_kind": (I, [I, I, I]),
    "attention_backward_fused_bf16": (None, [P, P, P, P, P, I, I, I, I]),
    "attention_backward_fused_bf16_ex": (None, [P, P, P, P, P, I, I, I, I, P]),
    "layernorm_forward_bf16": (None, [P, P, P, P, P, P, I, I, I]),
    "layernorm_backward_bf16": (None, [P, P, P, P, P, P, P, P, I, I, I]),
    "gelu_forward_bf16": (None, [P, P, I]),
    "gelu_backward_bf16": (None, [P, P, P, I]),
    "gemm_bf16_ex": (None, [P, LL, P, LL, I, P, LL, I, P, P, I, I, I, I, I]),
    "gemm_bf16_fused": (None, [P, P, LL, P, LL, P, LL, I, P, LL, I, P, P, I, I, I, I]),
    "mx_scale_size": (LL, [LL, I]),
    "quantize_mx_bf16_ex": (None, [P, P, P, LL, I, LL, LL]),
    "quantize_mx_f32_ex": (None, [P, P, P, LL, I, LL, LL]),
    "mx_cols_padded": (LL, [LL]),
    "quantize_mx_cols_bf16_ex": (None, [P, P, P, LL, I, LL]),
    "quantize_mx_rowcol_bf16_ex": (None, [P, P, P, P, P, LL, I, LL, LL, LL, LL]),
    "layernorm_forward_mx": (None, [P, P, P, P, P, P, P, P, P, LL, I, LL, LL, LL]),
    "layernorm_backward_stream": (None, [P, P, P, P, P, P, P, P, P, P, P, P, LL, I]),
    "layernorm_backward_stream_mx": (None, [P, P, P, P, P, P, P, P, P, P, P, P, LL, I, P, P, P, P, LL, LL, LL]),
    "gemm_fp8_fused": (None, [P, P, LL, P, LL, P, P, LL, P, P, LL, P, P, I, I, I, I]),
    "gemm_fp8_fused_mx": (None, [P, P, LL, P, LL, P, P, LL, P, P, LL, P, P, I, I, I, I, P, P]),
    "gemm_fp8_fused_mxc": (None, [P, P, LL, P, LL, P, P, LL, P, P, LL, P, P, I, I, I, I, P, P, P, P, LL, LL]),
    "gemm_bf16_set_variant": (None, [I]), "gemm_bf16_set_debug": (None, [I]),
    "gemm_bf16_set_trace": (None, [P]),
    "vit_kernel_hits": (I, [P, I]),
    "convert_f32_to_bf16": (None, [P, P, LL]),
    "convert_bf16_to_f32": (None, [P, P, LL]),
    # trainer
    "vit_trainer_create": (P, [ctypes.POINTER(VitConfigC), I, I, I]),
    "vit_trainer_num_params": (LL, [P]), "vit_trainer_device_bytes": (LL, [P]),
    "vit_trainer_set_params": (I, [P, P]), "vit_trainer_get_params": (I, [P, P]),
    "vit_trainer_get_grads": (I, [P, P]), "vit_trainer_set_batch": (I, [P, P, P]),
    "vit_trainer_set_batch_device": (I, [P, P, P]),
    "vit_trainer_forward": (I, [P, I]), "vit_trainer_zero_grad": (I, [P]),
    "vit_trainer_backward": (I, [P]), "vit_trainer_step": (I, [P, F]),
    "vit_trainer_train_step": (I, [P, F, I]), "vit_trainer_mean_loss": (F, [P]),
    "vit_trainer_get_logits": (I, [P, P]), "vit_trainer_sync": (I, [P]),
    "vit_trainer_stream": (P, [P]),
    "vit_layout_query": (I, [ctypes.POINTER(VitConfigC), P, P, ctypes.POINTER(LL)]),
    "vit_dp_unique_id_size": (I, []), "vit_dp_get_unique_id": (I, [ctypes.c_char_p]),
    "vit_trainer_dp_init": (I, [P, I, I, ctypes.c_char_p, I]),
    "vit_trainer_dp_ranks": (I, [P]),
    "vit_trainer_get_dp_snapshot": (I, [P, P]),
    "vit_trainer_set_timing": (I, [P, I]), "vit_trainer_set_concurrency": (I, [P, I]),
    "vit_trainer_set_option": (I, [P, ctypes.c_char_p, I]),
    "vit_trainer_timing": (I, [P, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_double),
                               ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_double), I]),
    "vit_trainer_step_adamw": (I, [P, F, F, F, F, F]),
    "vit_trainer_get_adamw_state": (I, [P, P, P, ctypes.POINTER(I)]),
    "vit_trainer_eval": (I, [P, P, ctypes.POINTER(I)]),
    # checkpoints (include/vit_checkpoint.h; host-only)
    "vit_config_num_params": (LL, [ctypes.POINTER(VitConfigC)]),
    "vit_checkpoint_read_info": (I, [ctypes.c_char_p, P]),
    "vit_checkpoint_write": (I, [ctypes.c_char_p, ctypes.POINTER(VitConfigC), P, P, P, I, P]),
    "vit_checkpoint_read": (I, [ctypes.c_char_p, ctypes.POINTER(VitConfigC), P, P, P]),
    # input pipeline (include/vit_data.h)
    "vit_loader_open": (P, [ctypes.c_char_p, ctypes.c_char_p, I, I, ctypes.c_ulonglong, I, I, I, I, I]),
    "vit_loader_num_records": (LL, [P]), "vit_loader_steps_per_epoch": (I, [P]),
    "vit_loader_next": (I, [P, ctypes.POINTER(P), ctypes.POINTER(P), ctypes.POINTER(LL), ctypes.POINTER(I)]),
    "vit_trainer_set_batch_u8": (I, [P, P, P, P, P]),
    # JPEG input pipeline (include/vit_jpeg.h)
    "vit_jpeg_probe": (I, [P, LL, ctypes.POINTER(I), ctypes.POINTER(I), ctypes.POINTER(I)]),
    "vit_jpeg_coefficients": (I, [P, LL, P, LL, P]),
    "vit_jpeg_loader_open": (P, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, I, ctypes.c_ulonglong, I, I,
                                 I, I, I, I]),
    "vit_jpeg_loader_num_records": (LL, [P]), "vit_jpeg_loader_steps_per_epoch": (I, [P]),
    "vit_jpeg_loader_next": (I, [P, ctypes.POINTER(P), ctypes.POINTER(LL), ctypes.POINTER(I)]),
    "vit_jpeg_loader_boxes": (I, [P, P]),
    "vit_jpeg_loader_decode_u8": (I, [P, P, I]),
    "vit_trainer_set_batch_jpeg": (I, [P, P, P, P]),
    "vit_trainer_save_checkpoint": (I, [P, ctypes.c_char_p]),
    "vit_trainer_load_checkpoint": (I, [P, ctypes.c_char_p]),
}


def exported_symbols():
    """Every symbol include/*.h declares (used by the ABI test)."""
    return sorted(set(_SIGS) | {n for n, _ in _VOID})


def lib():
    """Load libvit_hip.so (raises if absent — there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise VitError(f"{LIB_PATH} not built; run __graft_entry__.build() or make -C vit.rs_amd")
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        if os.environ.get("VIT_LIB") and not hasattr(L, name):
            continue  # an older A/B build may lack newer entry points
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    for name, args in _VOID:
        f = getattr(L, name)
        f.restype = None
        f.argtypes = args
    _lib = L
    return L


# launch-counter families (include/vit_ops.h VIT_HIT_*); GEMM families are base + epilogue
HIT_GEMM_128, HIT_GEMM_256x256, HIT_GEMM_256x128, HIT_GEMM_FP8, HIT_GEMM_F32 = 0, 16, 32, 48, 64
HIT_SPLITK_REDUCE, HIT_ATTN_FWD_MFMA, HIT_ATTN_BWD_PERSISTENT = 80, 81, 82
HIT_ATTN_BWD_ONEPASS, HIT_ATTN_BWD_PAIR, HIT_ATTN_GENERIC = 83, 84, 85
HIT_ATTN_BWD_XKEY, HIT_QUANT_ROWCOL = 86, 87
HIT_GEMM_PP = 88
HIT_LN_MX = 89
HIT_LNB_MX = 90


def kernel_hits():
    """Launch counts since the last kernel_hits_reset(), indexed by the HIT_* constants."""
    n = lib().vit_kernel_hits(None, 0)
    out = (ctypes.c_longlong * n)()
    lib().vit_kernel_hits(ctypes.cast(out, ctypes.c_void_p), n)
    return np.array(out[:], dtype=np.int64)


def kernel_hits_reset():
    lib().vit_kernel_hits_reset()


def check(what=""):
    """Raise the sticky library error, if any."""
    msg = ctypes.c_char_p()
    if lib().vit_last_error(ctypes.byref(msg)):
        text = msg.value.decode() if msg.value else "unknown"
        lib().vit_clear_error()
        raise VitError(f"{what}: {text}" if what else text)


# --------------------------------------------------------------------------- device buffers
class DeviceArray:
    """Owned device allocation with numpy up/download (vit_malloc / vit_memcpy)."""

    def __init__(self, shape, dtype):
        self.shape = tuple(shape) if isinstance(shape, (tuple, list)) else (int(shape),)
        self.dtype = np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape)) * self.dtype.itemsize
        self.ptr = lib().vit_malloc(max(self.nbytes, 16))
        if not self.ptr:
            check("vit_malloc")
            raise VitError("vit_malloc returned NULL")

    @classmethod
    def from_numpy(cls, a, dtype=None):
        a = np.ascontiguousarray(a if dtype is None else a.astype(dtype))
        d = cls(a.shape, a.dtype)
        d.upload(a)
        return d

    @classmethod
    def zeros(cls, shape, dtype):
        d = cls(shape, dtype)
        lib().vit_memset(d.ptr, 0, d.nbytes)
        check("vit_memset")
        return d

    def upload(self, a):
        a = np.ascontiguousarray(a, dtype=self.dtype)
        assert a.nbytes == self.nbytes
        lib().vit_memcpy_h2d(self.ptr, a.ctypes.data_as(ctypes.c_void_p), self.nbytes)
        check("h2d")

    def numpy(self):
        out = np.empty(self.shape, dtype=self.dtype)
        lib().vit_sync()
        lib().vit_memcpy_d2h(out.ctypes.data_as(ctypes.c_void_p), self.ptr, self.nbytes)
        check("d2h")
        return out

    def free(self):
        if self.ptr:
            lib().vit_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def bf16_bits(a):
    """fp32 numpy -> bf16 bits (uint16), round to nearest even."""
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    return r


def bf16_to_f32(b):
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


def call(name, *args):
    """Call a C-ABI op with DeviceArray / int / float arguments and raise on error."""
    L = lib()
    cargs = []
    for a in args:
        if isinstance(a, DeviceArray):
            cargs.append(a.ptr)
        elif a is None:
            cargs.append(None)
        else:
            cargs.append(a)
    getattr(L, name)(*cargs)
    L.vit_sync()
    check(name)


# --------------------------------------------------------------------------- checkpoints
def checkpoint_info(path):
    """Header of a checkpoint file (include/vit_checkpoint.h) as a dict; host-only."""
    info = CheckpointInfoC()
    if lib().vit_checkpoint_read_info(os.fsencode(path), ctypes.byref(info)):
        check("checkpoint_info")
    c = info.cfg
    cfg = data.VitCfg("checkpoint", c.img, c.patch, c.channels, c.num_layers, c.num_heads,
                      c.num_classes, c.in_ch)
    return {"cfg": cfg, "num_params": int(info.num_params), "has_opt": bool(info.has_opt),
            "step": int(info.step),
            "adamw": (info.adamw.beta1, info.adamw.beta2, info.adamw.eps, info.adamw.weight_decay)}


def write_checkpoint(path, cfg, params, m=None, v=None, step=0, adamw=None):
    """Write canonical fp32 params (+ AdamW m, v) in the checkpoint format; host-only."""
    params = np.ascontiguousarray(params, dtype=np.float32)
    assert params.size == cfg.num_params()
    ptrs = [params.ctypes.data_as(P)]
    keep = []
    for a in (m, v):
        if a is None:
            ptrs.append(None)
        else:
            a = np.ascontiguousarray(a, dtype=np.float32)
            assert a.size == params.size
            keep.append(a)
            ptrs.append(a.ctypes.data_as(P))
    hp = AdamWC(*adamw) if adamw is not None else None
    if lib().vit_checkpoint_write(os.fsencode(path), ctypes.byref(_cfg_c(cfg)), *ptrs, int(step),
                                  ctypes.byref(hp) if hp is not None else None):
        check("write_checkpoint")


def read_checkpoint(path, cfg):
    """(params, m, v) of a checkpoint written for cfg; m, v None without optimizer state."""
    info = checkpoint_info(path)
    n = cfg.num_params()
    p = np.empty(n, np.float32)
    m = np.empty(n, np.float32) if info["has_opt"] else None
    v = np.empty(n, np.float32) if info["has_opt"] else None
    if lib().vit_checkpoint_read(os.fsencode(path), ctypes.byref(_cfg_c(cfg)), p.ctypes.data_as(P),
                                 m.ctypes.data_as(P) if m is not None else None,
                                 v.ctypes.data_as(P) if v is not None else None):
        check("read_checkpoint")
    return p, m, v


# --------------------------------------------------------------------------- input pipeline
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


class Loader:
    """Native record loader (include/vit_data.h): uint8 [N, img, img, 3] + int32 [N] files,
    seeded per-epoch shuffle, the batch of DP rank `rank` of `world`, background assembly."""

    def __init__(self, images_path, labels_path, img, batch, seed=1337, rank=0, world=1,
                 shuffle=True, pinned=True, depth=3):
        self.img, self.B = img, batch
        self.h = lib().vit_loader_open(os.fsencode(images_path), os.fsencode(labels_path), img, batch,
                                       seed, rank, world, int(shuffle), int(pinned), depth)
        if not self.h:
            check("vit_loader_open")
            raise VitError("vit_loader_open failed")
        self.num_records = int(lib().vit_loader_num_records(self.h))
        self.steps_per_epoch = int(lib().vit_loader_steps_per_epoch(self.h))

    def next_raw(self):
        """(images_ptr, labels_ptr, epoch, step): host pointers valid until the next call."""
        ip, lp, ep, st = P(), P(), LL(), I()
        if lib().vit_loader_next(self.h, ctypes.byref(ip), ctypes.byref(lp), ctypes.byref(ep),
                                 ctypes.byref(st)):
            check("vit_loader_next")
        return ip.value, lp.value, ep.value, st.value

    def next(self):
        """(images uint8 [B, img, img, 3], labels int32 [B], epoch, step) — copies."""
        ip, lp, ep, st = self.next_raw()
        n = self.B * self.img * self.img * 3
        img = np.ctypeslib.as_array((ctypes.c_ubyte * n).from_address(ip)).copy()
        lab = np.ctypeslib.as_array((ctypes.c_int * self.B).from_address(lp)).copy()
        return img.reshape(self.B, self.img, self.img, 3), lab, ep, st

    def close(self):
        if getattr(self, "h", None):
            lib().vit_loader_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# --------------------------------------------------------------------------- model
def jpeg_probe(data):
    """(width, height, kind) of a JPEG byte string (kind 0 gray, 1 4:4:4, 2 4:2:2, 3 4:2:0); host-only."""
    buf = np.frombuffer(data, np.uint8)
    w, h, k = I(), I(), I()
    if lib().vit_jpeg_probe(buf.ctypes.data_as(P), buf.size, ctypes.byref(w), ctypes.byref(h), ctypes.byref(k)):
        check("jpeg_probe")
    return w.value, h.value, k.value


def jpeg_coefficients(data):
    """(coef int16 [blocks][64] natural order, info int32 [208]) of a JPEG byte string; host-only
    (the entropy-decoder half of the pipeline, for tests)."""
    buf = np.frombuffer(data, np.uint8)
    info = np.zeros(208, np.int32)
    if lib().vit_jpeg_coefficients(buf.ctypes.data_as(P), buf.size, None, 0, info.ctypes.data_as(P)):
        check("jpeg_coefficients")
    nc = int(info[3])
    nblk = sum(int(info[4 + 4 * c]) * int(info[5 + 4 * c]) for c in range(nc))
    coef = np.zeros((nblk, 64), np.int16)
    if lib().vit_jpeg_coefficients(buf.ctypes.data_as(P), buf.size, coef.ctypes.data_as(P), nblk, None):
        check("jpeg_coefficients")
    return coef, info


def write_jpeg_records(prefix, jpegs, labels):
    """Pack JPEG byte strings into the loader's record files: prefix.jpg (concatenated),
    prefix.idx (N+1 int64 offsets), prefix.lab (N int32).  Returns the three paths."""
    offs = np.zeros(len(jpegs) + 1, np.int64)
    offs[1:] = np.cumsum([len(j) for j in jpegs])
    with open(prefix + ".jpg", "wb") as f:
        for j in jpegs:
            f.write(j)
    offs.tofile(prefix + ".idx")
    np.asarray(labels, np.int32).tofile(prefix + ".lab")
    return prefix + ".jpg", prefix + ".idx", prefix + ".lab"


class JpegLoader:
    """Packed-JPEG record loader (include/vit_jpeg.h): host threads entropy-decode batches ahead;
    the GPU half (IDCT, chroma, colour, crop/flip/resize) runs in decode_u8() or feeds a trainer
    through ViT.set_batch_jpeg()."""

    def __init__(self, jpeg_path, index_path, labels_path, batch, seed=1337, rank=0, world=1,
                 shuffle=True, augment=False, depth=3, threads=4):
        self.B = batch
        self.h = lib().vit_jpeg_loader_open(os.fsencode(jpeg_path), os.fsencode(index_path),
                                            os.fsencode(labels_path), batch, seed, rank, world, int(shuffle),
                                            int(augment), depth, threads)
        if not self.h:
            check("vit_jpeg_loader_open")
            raise VitError("vit_jpeg_loader_open failed")
        self.num_records = int(lib().vit_jpeg_loader_num_records(self.h))
        self.steps_per_epoch = int(lib().vit_jpeg_loader_steps_per_epoch(self.h))

    def next(self):
        """Advance to the next batch: (labels int32 [B] copy, epoch, step)."""
        lp, ep, st = P(), LL(), I()
        if lib().vit_jpeg_loader_next(self.h, ctypes.byref(lp), ctypes.byref(ep), ctypes.byref(st)):
            check("vit_jpeg_loader_next")
        lab = np.ctypeslib.as_array((ctypes.c_int * self.B).from_address(lp.value)).copy()
        return lab, ep.value, st.value

    def boxes(self):
        """The current batch's crop boxes [B][5] = x0, y0, w, h, flip."""
        out = np.zeros((self.B, 5), np.int32)
        if lib().vit_jpeg_loader_boxes(self.h, out.ctypes.data_as(P)):
            check("vit_jpeg_loader_boxes")
        return out

    def decode_u8(self, img, out=None):
        """GPU half of the current batch -> DeviceArray uint8 [B, img, img, 3]."""
        if out is None:
            out = DeviceArray((self.B, img, img, 3), np.uint8)
        if lib().vit_jpeg_loader_decode_u8(self.h, out.ptr, img):
            check("vit_jpeg_loader_decode_u8")
        return out

    def close(self):
        if getattr(self, "h", None):
            lib().vit_jpeg_loader_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ViT:
    """Mirror of the reference's `struct ViT` (train_vit.rs:65-86) over the native trainer.

    build(cfg, batch, precision)      ~ ViT::build_from_checkpoint (:89) with canonical params
    forward(pixels, targets, b_glob)  ~ ViT::forward (:188); sets .mean_loss (:263)
    zero_grad(); backward()           ~ gradient zeroing (:272) + ViT::backward (:271)
    optimizer_step(lr)                ~ optimizer_step (:737)
    """

    def __init__(self, cfg, batch, precision=VIT_BF16, device=0):
        L = lib()
        self.cfg = cfg
        self.B = batch
        self.precision = precision
        c = VitConfigC(cfg.img, cfg.patch, cfg.in_ch, cfg.channels, cfg.num_layers,
                       cfg.num_heads, cfg.num_classes)
        self.h = L.vit_trainer_create(ctypes.byref(c), batch, precision, device)
        if not self.h:
            check("vit_trainer_create")
            raise VitError("vit_trainer_create failed")
        self.num_parameters = int(L.vit_trainer_num_params(self.h))
        assert self.num_parameters == cfg.num_params()
        self.mean_loss = -1.0

    @classmethod
    def build(cls, cfg, batch, precision=VIT_BF16, params=None, device=0):
        m = cls(cfg, batch, precision, device)
        if params is not None:
            m.set_params(params)
        return m

    def close(self):
        if getattr(self, "h", None):
            lib().vit_trainer_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _ok(self, rc, what):
        if rc:
            check(what)
            raise VitError(what)

    def set_params(self, flat):
        flat = np.ascontiguousarray(flat, dtype=np.float32)
        assert flat.size == self.num_parameters
        self._ok(lib().vit_trainer_set_params(self.h, flat.ctypes.data_as(P)), "set_params")

    def params(self):
        out = np.empty(self.num_parameters, dtype=np.float32)
        self._ok(lib().vit_trainer_get_params(self.h, out.ctypes.data_as(P)), "get_params")
        return out

    def grads(self):
        out = np.empty(self.num_parameters, dtype=np.float32)
        self._ok(lib().vit_trainer_get_grads(self.h, out.ctypes.data_as(P)), "get_grads")
        return out

    def set_batch(self, pixels, labels):
        """labels None = a forward-only batch (train_vit.rs:254-266: mean_loss = -1)."""
        px = np.ascontiguousarray(pixels, dtype=np.float32)
        assert px.shape == (self.B, 3, self.cfg.img, self.cfg.img)
        lb = None
        if labels is not None:
            lb = np.ascontiguousarray(labels, dtype=np.int32)
            assert lb.shape == (self.B,)
        self._ok(lib().vit_trainer_set_batch(self.h, px.ctypes.data_as(P),
                                             lb.ctypes.data_as(P) if lb is not None else None),
                 "set_batch")

    def set_batch_jpeg(self, loader, mean=IMAGENET_MEAN, std=IMAGENET_STD):
        """The JpegLoader's current batch -> normalised device pixels + labels
        (vit_trainer_set_batch_jpeg)."""
        m = np.asarray(mean, np.float32)
        sd = np.asarray(std, np.float32)
        self._ok(lib().vit_trainer_set_batch_jpeg(self.h, loader.h, m.ctypes.data_as(P), sd.ctypes.data_as(P)),
                 "set_batch_jpeg")

    def set_batch_u8(self, images, labels=None, mean=IMAGENET_MEAN, std=IMAGENET_STD):
        """uint8 [B, img, img, 3] (numpy array, or a host pointer from Loader.next_raw) ->
        normalised device pixels (vit_trainer_set_batch_u8)."""
        if isinstance(images, np.ndarray):
            images = np.ascontiguousarray(images, dtype=np.uint8)
            assert images.shape == (self.B, self.cfg.img, self.cfg.img, 3)
            iptr = images.ctypes.data_as(P)
        else:
            iptr = P(images)
        lptr = None
        if isinstance(labels, np.ndarray):
            labels = np.ascontiguousarray(labels, dtype=np.int32)
            assert labels.shape == (self.B,)
            lptr = labels.ctypes.data_as(P)
        elif labels is not None:
            lptr = P(labels)
        m = np.ascontiguousarray(mean, np.float32)
        sd = np.ascontiguousarray(std, np.float32)
        self._ok(lib().vit_trainer_set_batch_u8(self.h, iptr, lptr, m.ctypes.data_as(P),
                                                sd.ctypes.data_as(P)), "set_batch_u8")

    def forward(self, pixels=None, targets=None, b_global=None):
        if pixels is not None:
            self.set_batch(pixels, targets)
        self._ok(lib().vit_trainer_forward(self.h, int(b_global or self.B)), "forward")
        self.mean_loss = float(lib().vit_trainer_mean_loss(self.h))
        check("mean_loss")
        return self.mean_loss

    def forward_async(self, b_global=None):
        self._ok(lib().vit_trainer_forward(self.h, int(b_global or self.B)), "forward")

    def zero_grad(self):
        self._ok(lib().vit_trainer_zero_grad(self.h), "zero_grad")

    def backward(self):
        self._ok(lib().vit_trainer_backward(self.h), "backward")

    def optimizer_step(self, lr):
        self._ok(lib().vit_trainer_step(self.h, float(lr)), "optimizer_step")

    def optimizer_step_adamw(self, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0):
        """AdamW (vit_trainer_step_adamw)."""
        self._ok(lib().vit_trainer_step_adamw(self.h, float(lr), float(beta1), float(beta2),
                                              float(eps), float(weight_decay)), "step_adamw")

    def adamw_state(self):
        """(m, v, t) in canonical order."""
        m = np.empty(self.num_parameters, np.float32)
        v = np.empty(self.num_parameters, np.float32)
        t = ctypes.c_int()
        self._ok(lib().vit_trainer_get_adamw_state(self.h, m.ctypes.data_as(P), v.ctypes.data_as(P),
                                                   ctypes.byref(t)), "get_adamw_state")
        return m, v, t.value

    def evaluate(self, pixels=None, labels=None):
        """Forward + device top-1: (predictions [B], number correct or -1 without labels)."""
        if pixels is not None:
            self.set_batch(pixels, labels)
        pred = np.empty(self.B, np.int32)
        correct = ctypes.c_int()
        self._ok(lib().vit_trainer_eval(self.h, pred.ctypes.data_as(P), ctypes.byref(correct)), "eval")
        return pred, correct.value

    def save_checkpoint(self, path):
        self._ok(lib().vit_trainer_save_checkpoint(self.h, os.fsencode(path)), "save_checkpoint")

    def load_checkpoint(self, path):
        self._ok(lib().vit_trainer_load_checkpoint(self.h, os.fsencode(path)), "load_checkpoint")

    def train_step(self, lr, b_global=None):
        self._ok(lib().vit_trainer_train_step(self.h, float(lr), int(b_global or self.B)),
                 "train_step")

    def logits(self):
        out = np.empty((self.B, self.cfg.num_classes), dtype=np.float32)
        self._ok(lib().vit_trainer_get_logits(self.h, out.ctypes.data_as(P)), "get_logits")
        return out

    def sync(self):
        self._ok(lib().vit_trainer_sync(self.h), "sync")

    def device_bytes(self):
        return int(lib().vit_trainer_device_bytes(self.h))

    # ---- data parallel (RCCL over xGMI), one process per GPU
    @staticmethod
    def dp_unique_id():
        n = lib().vit_dp_unique_id_size()
        buf = ctypes.create_string_buffer(n)
        if lib().vit_dp_get_unique_id(buf):
            check("ncclGetUniqueId")
        return buf.raw

    def dp_init(self, rank, world, unique_id, overlap=True):
        self._ok(lib().vit_trainer_dp_init(self.h, rank, world, unique_id, int(overlap)), "dp_init")

    def dp_snapshot(self):
        """the dp_probe snapshot arena (canonical order): each chunk as it stood when reduced."""
        out = np.empty(self.num_parameters, dtype=np.float32)
        self._ok(lib().vit_trainer_get_dp_snapshot(self.h, out.ctypes.data_as(P)), "dp_snapshot")
        return out

    def dp_ranks(self):
        """ranks RCCL reports for the trainer's communicator (0 without DP)."""
        n = lib().vit_trainer_dp_ranks(self.h)
        if n < 0:
            check("dp_ranks")
        return n

    # ---- stream concurrency (micro-batch streams + weight-gradient stream), on by default
    def set_concurrency(self, on=True):
        self._ok(lib().vit_trainer_set_concurrency(self.h, int(on)), "set_concurrency")

    def set_option(self, name, value):
        self._ok(lib().vit_trainer_set_option(self.h, name.encode(), int(value)), f"set_option {name}")

    # ---- per-kernel-class timing (HIP events on the stream each kernel runs on)
    def set_timing(self, on=True):
        lib().vit_trainer_set_timing(self.h, int(on))

    def timing(self):
        n = 64
        names = (ctypes.c_char_p * n)()
        ms = (ctypes.c_double * n)()
        calls = (ctypes.c_longlong * n)()
        flops = (ctypes.c_double * n)()
        k = lib().vit_trainer_timing(self.h, names, ms, calls, flops, n)
        check("timing")
        return {names[i].decode(): {"ms": ms[i], "calls": calls[i], "flops": flops[i]}
                for i in range(k)}

    def timing_reset(self):
        lib().vit_trainer_timing_reset(self.h)
