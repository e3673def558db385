"""MX quantizer throughput (HIP events): row form, column form and both from one read (rowcol),
ViT-H/14 micro-batch shapes ([16448 tokens] x C / 3C / 4C bf16).
    python tools/bench_quant.py [--iters 20]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitpkg import vit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--R", type=int, default=16448)  # one ViT-H/14 micro-batch (64 images)
    a = ap.parse_args()
    L = vit.lib()
    assert L.vit_init(0) == 0
    R = a.R
    for C in (1280, 3840, 5120):
        x = vit.DeviceArray.from_numpy(vit.bf16_bits(np.random.default_rng(C).normal(size=R * C).astype(np.float32)),
                                       np.uint16)
        kp = int(L.mx_cols_padded(R))
        q = vit.DeviceArray.zeros(max(C * kp, R * C), np.uint8)
        sl = vit.DeviceArray.zeros(max(int(L.mx_scale_size(C, kp)), int(L.mx_scale_size(R, C))), np.uint8)
        q2 = vit.DeviceArray.zeros(R * C, np.uint8)
        sl2 = vit.DeviceArray.zeros(int(L.mx_scale_size(R, C)), np.uint8)
        for name, fn in (("cols", lambda: L.quantize_mx_cols_bf16_ex(q.ptr, sl.ptr, x.ptr, R, C, C)),
                         ("rows", lambda: L.quantize_mx_bf16_ex(q.ptr, sl.ptr, x.ptr, R, C, C, C)),
                         ("rowcol", lambda: L.quantize_mx_rowcol_bf16_ex(q2.ptr, sl2.ptr, q.ptr, sl.ptr, x.ptr, R, C, C,
                                                                         kp, 0, kp))):
            fn()
            L.vit_sync()
            e0, e1 = L.vit_event_create(), L.vit_event_create()
            L.vit_event_record(e0)
            for _ in range(a.iters):
                fn()
            L.vit_event_record(e1)
            L.vit_sync()
            us = L.vit_event_elapsed_ms(e0, e1) * 1e3 / a.iters
            byts = R * C * 2 + R * C + R * C // 32 + (R * C + R * C // 32 if name == "rowcol" else 0)
            print(f"{name} VIT_ROWCOL_COLS={os.environ.get('VIT_ROWCOL_COLS', 'auto')} [{R} x {C}]: {us:8.1f} us  "
                  f"{byts / us / 1e6:6.2f} TB/s", flush=True)
            vit.check("quant")


if __name__ == "__main__":
    main()
