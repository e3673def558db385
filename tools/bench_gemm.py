"""Microbenchmark of the bf16 GEMM engine at the ViT-B/16 B=256 training shapes (HIP events).

    python tools/bench_gemm.py [--iters 20] [--batch 256]
Prints one line per GEMM (layout, M, N, K, ms, TFLOP/s).  VIT_GEMM=1 selects the 128x128 kernel.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitpkg import vit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--C", type=int, default=768)
    ap.add_argument("--only", default=None, help="comma-separated shape names")
    args = ap.parse_args()
    L = vit.lib()
    assert L.vit_init(0) == 0
    C, BT = args.C, args.batch * 197
    rng = np.random.default_rng(0)
    maxe = BT * 4 * C
    buf_a = vit.DeviceArray.from_numpy(vit.bf16_bits(rng.uniform(-1, 1, size=maxe).astype(np.float32)), np.uint16)
    buf_b = vit.DeviceArray.from_numpy(vit.bf16_bits(rng.uniform(-1, 1, size=16 * C * C).astype(np.float32)), np.uint16)
    buf_b2 = vit.DeviceArray.from_numpy(vit.bf16_bits(rng.uniform(-1, 1, size=maxe).astype(np.float32)), np.uint16)
    out = vit.DeviceArray.zeros(maxe * 2, np.float32)
    bias = vit.DeviceArray.zeros(4 * C, np.float32)
    e0, e1 = L.vit_event_create(), L.vit_event_create()
    # (name, M, N, K, ak, bk, epi)
    shapes = []
    for nm, oc, ic in (("qkv", 3 * C, C), ("proj", C, C), ("fc", 4 * C, C), ("fcproj", C, 4 * C)):
        shapes.append((f"fwd_{nm}", BT, oc, ic, 1, 1, 3))
        shapes.append((f"dgrad_{nm}", BT, ic, oc, 1, 0, 0))
        shapes.append((f"wgrad_{nm}", oc, ic, BT, 0, 0, 2))
    tot_ms, tot_fl = 0.0, 0.0
    if args.only:
        keep = set(args.only.split(","))
        shapes = [sh for sh in shapes if sh[0] in keep]
    for name, M, N, K, ak, bk, epi in shapes:
        lda = K if ak else M
        ldb = K if bk else N
        B_ = buf_b if (ak and name.startswith(("fwd", "dgrad"))) else buf_b2
        def run():
            L.gemm_bf16_ex(out.ptr, N, buf_a.ptr, lda, ak, B_.ptr, ldb, bk,
                           bias.ptr if epi != 2 else None, None, M, N, K, epi, 0)
        for _ in range(3):
            run()
        L.vit_sync()
        vit.check(name)
        L.vit_event_record(e0)
        for _ in range(args.iters):
            run()
        L.vit_event_record(e1)
        ms = L.vit_event_elapsed_ms(e0, e1) / args.iters
        vit.check(name)
        fl = 2.0 * M * N * K
        tot_ms += ms
        tot_fl += fl
        print(f"{name:14s} M={M:6d} N={N:5d} K={K:6d}  {ms:8.3f} ms  {fl / ms / 1e9:8.1f} TFLOP/s", flush=True)
    print(f"{'all':14s} {tot_ms:8.3f} ms per layer-set  {tot_fl / tot_ms / 1e9:8.1f} TFLOP/s")


if __name__ == "__main__":
    main()
