"""Per-tensor parity of one config / mode against the fp32 oracle, for A/B of library builds
(VIT_LIB=<path> selects the build).  python tools/ab_parity.py [--config vit_b16] [--batch 1] [--mode bf16]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
from vitpkg import vit  # noqa: E402
import oracle_ctypes as oc  # noqa: E402
import parity  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="vit_b16")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--mode", default="bf16")
    a = ap.parse_args()
    assert vit.lib().vit_init(0) == 0
    cfg = vit.data.CONFIGS[a.config]
    params = vit.data.init_params(cfg, "parity", seed=3)
    px, lab = vit.data.synthetic_batch(cfg, a.batch, seed=5)
    o = oc.Oracle("f32")
    ref = oc.RefViT(o, oc.VitConfig(cfg.img, cfg.patch, cfg.in_ch, cfg.channels, cfg.num_layers, cfg.num_heads,
                                    cfg.num_classes), a.batch)
    p = o.arr(params)
    loss_r = ref.forward(p, px, lab)
    g_r = np.zeros_like(p)
    ref.backward(p, g_r)
    m = vit.ViT.build(cfg, a.batch, {"bf16": vit.VIT_BF16, "fp8": vit.VIT_FP8, "fp32": vit.VIT_FP32}[a.mode],
                      params=params)
    m.zero_grad()
    loss = m.forward(px, lab)
    m.backward()
    pairs = parity.tensors(cfg, m.logits(), m.grads(), ref.logits(), g_r)
    rep = {n: parity.metrics(x, r, 2e-2, 1e-2) for n, (x, r) in pairs.items()}
    print(os.environ.get("VIT_LIB", "default"), f"loss rel {abs(loss - loss_r) / abs(loss_r):.2e}")
    for n, r in rep.items():
        print(f"  {n:10s} max {r['max']:.5f} rms {r['rms']:.5f} frac {r['frac']:.5f}")


if __name__ == "__main__":
    main()
