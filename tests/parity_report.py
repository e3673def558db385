"""Per-tensor parity of the native trainer against the fp32 CPU oracle (the reference loops,
oracle/oracle.c), for every precision mode, written as JSON (profiles/<tag>_parity.json).

    python tests/parity_report.py [--out profiles/r02_parity.json]

For each (config, batch, mode): relative error of the loss, and for the logits and each of the 20
parameter-gradient tensors (canonical order, train_vit.rs:10-27 + ViT tensors):
  max    = max |gpu - ref| / max |ref|                   (the tests' gate metric)
  median = median over elements with |ref| > 1e-3 max |ref| of |gpu - ref| / |ref|
  frac_1e-4 = share of elements with |gpu - ref| <= 1e-4 |ref| + 1e-6 (SURVEY.md §8d, fp32 mode)
Inputs: seeded synthetic batches, "parity" init (every gradient path non-degenerate).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # tests/ -> repo root
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from vitpkg import vit  # noqa: E402
import oracle_ctypes as oc  # noqa: E402

MODES = {"fp32": vit.VIT_FP32, "bf16": vit.VIT_BF16, "fp8": vit.VIT_FP8}


def stats(a, r):
    a = np.asarray(a, np.float64).ravel()
    r = np.asarray(r, np.float64).ravel()
    d = np.abs(a - r)
    mx = max(np.abs(r).max(), 1e-30)
    sel = np.abs(r) > 1e-3 * mx
    med = float(np.median(d[sel] / np.abs(r[sel]))) if sel.any() else 0.0
    ok = d <= 1e-4 * np.abs(r) + 1e-6
    return {"max": float(d.max() / mx), "median": med, "frac_1e-4": float(ok.mean())}


def run(cfg, B, modes, seed=3):
    params = vit.data.init_params(cfg, "parity", seed=seed)
    px, lab = vit.data.synthetic_batch(cfg, B, seed=seed + 2)
    o = oc.Oracle("f32")
    m = oc.RefViT(o, oc.VitConfig(cfg.img, cfg.patch, cfg.in_ch, cfg.channels, cfg.num_layers,
                                  cfg.num_heads, cfg.num_classes), B)
    p = o.arr(params)
    t0 = time.time()
    loss_r = m.forward(p, px, lab)
    g_r = np.zeros_like(p)
    m.backward(p, g_r)
    logits_r = m.logits()
    t_oracle = time.time() - t0
    out = {"config": cfg.name, "batch": B, "T": cfg.T, "C": cfg.channels, "layers": cfg.num_layers,
           "head_size": cfg.head_size, "oracle_s": round(t_oracle, 2), "modes": {}}
    for mode in modes:
        t = vit.ViT.build(cfg, B, MODES[mode], params=params)
        t.zero_grad()
        loss = t.forward(px, lab)
        t.backward()
        g = t.grads()
        rec = {"loss": {"gpu": loss, "oracle": loss_r, "rel": abs(loss - loss_r) / abs(loss_r)},
               "logits": stats(t.logits(), logits_r),
               "grads": {n: stats(a, b) for n, a, b in zip(cfg.split(g).keys(), cfg.split(g).values(),
                                                           cfg.split(g_r).values())}}
        rec["max_grad_tensor"] = max(v["max"] for v in rec["grads"].values())
        out["modes"][mode] = rec
        t.close()
        print(f"{cfg.name} B={B} {mode}: loss {rec['loss']['rel']:.2e} logits {rec['logits']['max']:.2e} "
              f"max grad {rec['max_grad_tensor']:.2e}", flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02_parity.json"))
    ap.add_argument("--quick", action="store_true", help="small configs only")
    args = ap.parse_args()
    assert vit.lib().vit_init(0) == 0
    C = vit.data.CONFIGS
    h14_l1 = vit.data.VitCfg("vit_h14_l1", img=224, patch=14, channels=1280, num_layers=1, num_heads=16,
                             num_classes=1000)
    runs = [(C["test_h64"], 4, ["fp32", "bf16", "fp8"]), (C["vit_tiny16"], 8, ["fp32", "bf16"]),
            (h14_l1, 1, ["fp32", "bf16", "fp8"])]
    if not args.quick:
        runs.append((C["vit_b16"], 1, ["fp32", "bf16", "fp8"]))
    res = {"what": __doc__.strip().splitlines()[0], "oracle": "oracle/oracle.c (fp32, -ffp-contract=off)",
           "runs": [run(cfg, B, modes) for cfg, B, modes in runs]}
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
