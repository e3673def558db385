"""Microbenchmark of the fused bf16 attention kernels (HIP events); default ViT-B/16 B=256.
    python tools/bench_attn.py [--iters 10] [--batch 256] [--T 197] [--NH 12] [--hs 64] [--generic]
    ViT-H/14 B=128: --batch 128 --T 257 --NH 16 --hs 80"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitpkg import vit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--T", type=int, default=197)
    ap.add_argument("--NH", type=int, default=12)
    ap.add_argument("--hs", type=int, default=64)
    ap.add_argument("--generic", action="store_true", help="force the generic VALU kernels")
    ap.add_argument("--colsum", action="store_true", help="backward with the fused qkv-bias gradient (trainer form)")
    ap.add_argument("--env-ab", default=None,
                    help="A/B of backward environments in one process, interleaved round by round, e.g. "
                         "'VIT_ATTN_BWD_NOPAD=0|VIT_ATTN_BWD_NOPAD=1' (median of --rounds)")
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    if args.generic:
        os.environ["VIT_ATTN_GENERIC"] = "1"
    L = vit.lib()
    assert L.vit_init(0) == 0
    B, T, NH = args.batch, args.T, args.NH
    C = args.hs * NH
    kind = {1: "mfma", 2: "generic"}.get(L.vit_attention_kernel_kind(T, C, NH), "unsupported")
    rng = np.random.default_rng(0)
    qkv = vit.DeviceArray.from_numpy(vit.bf16_bits(rng.normal(size=B * T * 3 * C).astype(np.float32)), np.uint16)
    dout = vit.DeviceArray.from_numpy(vit.bf16_bits(rng.normal(size=B * T * C).astype(np.float32)), np.uint16)
    out = vit.DeviceArray.zeros(B * T * C, np.uint16)
    lse = vit.DeviceArray.zeros(B * NH * T, np.float32)
    dqkv = vit.DeviceArray.zeros(B * T * 3 * C, np.uint16)
    dbias = vit.DeviceArray.zeros(3 * C, np.float32)
    bwd = ((lambda: L.attention_backward_fused_bf16_ex(dqkv.ptr, dout.ptr, qkv.ptr, out.ptr, lse.ptr, B, T, C, NH, dbias.ptr))
           if args.colsum else
           (lambda: L.attention_backward_fused_bf16(dqkv.ptr, dout.ptr, qkv.ptr, out.ptr, lse.ptr, B, T, C, NH)))
    e0, e1 = L.vit_event_create(), L.vit_event_create()
    fl_f = 4.0 * B * T * T * C
    if args.env_ab:
        confs = args.env_ab.split("|")
        fwd = lambda: L.attention_forward_fused_bf16(out.ptr, lse.ptr, qkv.ptr, B, T, C, NH)  # noqa: E731
        res = {(c, d): [] for c in confs for d in ("fwd", "bwd")}
        for _ in range(args.rounds):
            for c in confs:
                for kv in filter(None, c.split(",")):
                    k, val = kv.split("=")
                    os.environ[k] = val
                for d, fn in (("fwd", fwd), ("bwd", bwd)):
                    for _ in range(2):
                        fn()
                    L.vit_sync()
                    L.vit_event_record(e0)
                    for _ in range(args.iters):
                        fn()
                    L.vit_event_record(e1)
                    res[(c, d)].append(L.vit_event_elapsed_ms(e0, e1) / args.iters)
                    vit.check(c)
        for (c, d), v in res.items():
            ms = float(np.median(v))
            fl = fl_f if d == "fwd" else 2 * fl_f
            print(f"attention {d} [{c}] B={B} T={T} NH={NH} hs={args.hs}: median {ms * 1e3:8.1f} us "
                  f"min {min(v) * 1e3:8.1f} us  {fl / ms / 1e9:7.1f} TFLOP/s", flush=True)
        return
    for name, fn, fl in (
            ("fwd", lambda: L.attention_forward_fused_bf16(out.ptr, lse.ptr, qkv.ptr, B, T, C, NH), fl_f),
            ("bwd" + ("+colsum" if args.colsum else ""), bwd, 2 * fl_f)):
        for _ in range(2):
            fn()
        L.vit_sync()
        vit.check(name)
        L.vit_event_record(e0)
        for _ in range(args.iters):
            fn()
        L.vit_event_record(e1)
        ms = L.vit_event_elapsed_ms(e0, e1) / args.iters
        vit.check(name)
        print(f"attention {name} [{kind} B={B} T={T} NH={NH} hs={args.hs}]: {ms * 1e3:8.1f} us  {fl / ms / 1e9:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
