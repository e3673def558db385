"""A/B of full training steps in ONE process (cdna_hip_programming.md §5.4 rule 24): configs are
applied between steps and interleaved round by round; the median ms/step per config is printed.
    python tools/ab_step.py "gemm_debug=0|gemm_debug=4" [--rounds 4 --steps 3]
A config is `key=value` pairs joined by `,`: trainer options (microbatch, dgrad_transposed),
concurrency (0/1), gemm_variant, gemm_debug.  --dtype fp8 for the MXFP8 step (option fp8_ln_mx)."""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitpkg import vit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--model", default="vit_b16")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"])
    args = ap.parse_args()
    L = vit.lib()
    assert L.vit_init(0) == 0
    cfg = vit.data.CONFIGS[args.model]
    m = vit.ViT(cfg, args.batch, vit.VIT_FP8 if args.dtype == "fp8" else vit.VIT_BF16)
    m.set_params(vit.data.init_params(cfg, "ref", seed=1337))
    px, lab = vit.data.synthetic_batch(cfg, args.batch, seed=1337)
    m.set_batch(px, lab)
    confs = [c for c in args.configs.split("|")]

    def apply(c):
        for kv in filter(None, c.split(",")):
            k, v = kv.split("=")
            v = int(v)
            if k == "concurrency":
                m.set_concurrency(bool(v))
            elif k == "gemm_variant":
                L.gemm_bf16_set_variant(v)
            elif k == "gemm_debug":
                L.gemm_bf16_set_debug(v)
            else:
                m.set_option(k, v)

    res = {c: [] for c in confs}
    for c in confs:  # warm every configuration once
        apply(c)
        m.train_step(1e-4)
        m.sync()
    for _ in range(args.rounds):
        for c in confs:
            apply(c)
            m.train_step(1e-4)
            m.sync()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                m.train_step(1e-4)
            m.sync()
            res[c].append((time.perf_counter() - t0) / args.steps * 1e3)
    for c in confs:
        v = np.array(res[c])
        print(f"{c:50s} median {np.median(v):8.3f} ms/step  min {v.min():8.3f}  "
              f"({args.batch / np.median(v) * 1e3:8.1f} img/s)", flush=True)


if __name__ == "__main__":
    main()
