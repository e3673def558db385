"""LayerNorm forward into MX (fp8 trainer ln1 / ln2) vs the unfused pair it replaces (HIP events):
ln_forward_bf16 + quantize_mx_rowcol_bf16, at ViT-H/14 shapes (C = 1280; 16448 tokens = one
micro-batch of 64 images, 32896 = B 128).
    python tools/bench_lnmx.py [--iters 20]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitpkg import vit  # noqa: E402


def timed(L, fn, iters):
    fn()
    L.vit_sync()
    e0, e1 = L.vit_event_create(), L.vit_event_create()
    L.vit_event_record(e0)
    for _ in range(iters):
        fn()
    L.vit_event_record(e1)
    L.vit_sync()
    return L.vit_event_elapsed_ms(e0, e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--C", type=int, default=1280)
    ap.add_argument("--rows", default="16448,32896", help="token counts (comma list)")
    a = ap.parse_args()
    L = vit.lib()
    assert L.vit_init(0) == 0
    C = a.C
    rng = np.random.default_rng(1)
    w = vit.DeviceArray.from_numpy(rng.normal(size=C).astype(np.float32))
    b = vit.DeviceArray.from_numpy(rng.normal(size=C).astype(np.float32))
    for R in [int(r) for r in a.rows.split(",")]:
        x = vit.DeviceArray.from_numpy(rng.normal(size=R * C).astype(np.float32))
        kp = int(L.mx_cols_padded(R))
        y = vit.DeviceArray.zeros(R * C, np.uint16)
        mu, rs = vit.DeviceArray.zeros(R, np.float32), vit.DeviceArray.zeros(R, np.float32)
        qc = vit.DeviceArray.zeros(C * kp, np.uint8)
        sc = vit.DeviceArray.zeros(int(L.mx_scale_size(C, kp)), np.uint8)
        qr = vit.DeviceArray.zeros(R * C, np.uint8)
        sr = vit.DeviceArray.zeros(int(L.mx_scale_size(R, C)), np.uint8)
        ln = lambda: L.layernorm_forward_bf16(y.ptr, mu.ptr, rs.ptr, x.ptr, w.ptr, b.ptr, 1, R, C)
        rc = lambda: L.quantize_mx_rowcol_bf16_ex(qr.ptr, sr.ptr, qc.ptr, sc.ptr, y.ptr, R, C, C, kp, 0, kp)
        mx = lambda: L.layernorm_forward_mx(qr.ptr, sr.ptr, qc.ptr, sc.ptr, mu.ptr, rs.ptr, x.ptr, w.ptr, b.ptr,
                                            R, C, kp, 0, kp)
        t_ln, t_rc, t_mx = timed(L, ln, a.iters), timed(L, rc, a.iters), timed(L, mx, a.iters)
        vit.check("lnmx")
        e = R * C
        print(f"[{R} x {C}] VIT_LNMX_XMAP={os.environ.get('VIT_LNMX_XMAP', '1')}: ln_bf16 {t_ln:7.1f} us "
              f"({6 * e / t_ln / 1e6:5.2f} TB/s)  rowcol {t_rc:7.1f} us ({4 * e / t_rc / 1e6:5.2f} TB/s)  "
              f"pair {t_ln + t_rc:7.1f} us  ln_mx {t_mx:7.1f} us ({6 * e / t_mx / 1e6:5.2f} TB/s)", flush=True)


if __name__ == "__main__":
    main()
