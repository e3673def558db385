"""Per-tensor parity of the native trainer against the fp32 CPU oracle (the reference loops,
oracle/oracle.c), for every precision mode, written as JSON (profiles/<tag>_parity.json).

    python tests/parity_report.py [--out profiles/r02_parity.json]

For each (config, batch, mode): relative error of the loss, and for the logits and each of the 20
parameter-gradient tensors (canonical order, train_vit.rs:10-27 + ViT tensors):
  max    = max |gpu - ref| / max |ref|                   (gate part (1), tests/parity.py)
  frac   = share of elements with |gpu - ref| <= tol |ref| + floor_rel max|ref| (part (2'); fp32 rule
           for fp32 mode, bf16 rule for bf16 / fp8)
  frac_abs1e-6 = the same with SURVEY.md §8d's absolute floor 1e-6 (reported, not gated)
  rms    = rms |gpu - ref| / rms |ref|
  median = median over elements with |ref| > 1e-3 max |ref| of |gpu - ref| / |ref|
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
sys.path.insert(0, os.path.join(ROOT, "tests"))
import parity  # noqa: E402

MODES = {"fp32": vit.VIT_FP32, "bf16": vit.VIT_BF16, "fp8": vit.VIT_FP8}


RULES = {"fp32": parity.FP32, "bf16": parity.BF16, "fp8": parity.BF16}


def stats(a, r, mode):
    m = parity.metrics(a, r, RULES[mode]["tol"], RULES[mode]["floor_rel"])
    a = np.asarray(a, np.float64).ravel()
    r = np.asarray(r, np.float64).ravel()
    sel = np.abs(r) > 1e-3 * np.abs(r).max()
    m["median"] = float(np.median(np.abs(a - r)[sel] / np.abs(r[sel]))) if sel.any() else 0.0
    return m


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
               "logits": stats(t.logits(), logits_r, mode),
               "grads": {n: stats(a, b, mode) for n, a, b in zip(cfg.split(g).keys(), cfg.split(g).values(),
                                                                 cfg.split(g_r).values())}}
        rec["max_grad_tensor"] = max(v["max"] for v in rec["grads"].values())
        rec["min_frac"] = min([rec["logits"]["frac"]] + [v["frac"] for v in rec["grads"].values()])
        rec["min_frac_abs1e-6"] = min([rec["logits"]["frac_abs1e-6"]] +
                                      [v["frac_abs1e-6"] for v in rec["grads"].values()])
        out["modes"][mode] = rec
        t.close()
        print(f"{cfg.name} B={B} {mode}: loss {rec['loss']['rel']:.2e} logits {rec['logits']['max']:.2e} "
              f"max grad {rec['max_grad_tensor']:.2e} min frac {rec['min_frac']:.5f} "
              f"(abs-1e-6 floor {rec['min_frac_abs1e-6']:.5f})", flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03_parity.json"))
    ap.add_argument("--quick", action="store_true", help="small configs only")
    ap.add_argument("--prod", action="store_true", help="add the production-engine config (B=128)")
    args = ap.parse_args()
    assert vit.lib().vit_init(0) == 0
    C = vit.data.CONFIGS
    h14_l1 = vit.data.VitCfg("vit_h14_l1", img=224, patch=14, channels=1280, num_layers=1, num_heads=16,
                             num_classes=1000)
    runs = [(C["test_h64"], 4, ["fp32", "bf16", "fp8"]), (C["vit_tiny16"], 8, ["fp32", "bf16"]),
            (h14_l1, 1, ["fp32", "bf16", "fp8"])]
    if not args.quick:
        runs.append((C["vit_b16"], 1, ["fp32", "bf16", "fp8"]))
    if args.prod:
        prod = vit.data.VitCfg("prod_l2", img=224, patch=16, channels=256, num_layers=2, num_heads=4,
                               num_classes=1000)
        runs.append((prod, 128, ["fp32", "bf16", "fp8"]))
    res = {"what": __doc__.strip().splitlines()[0], "oracle": "oracle/oracle.c (fp32, -ffp-contract=off)",
           "runs": [run(cfg, B, modes) for cfg, B, modes in runs]}
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
