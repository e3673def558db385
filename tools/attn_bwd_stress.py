"""Repeat an attention backward variant (VIT_ATTN_BWD; default: the persistent one-pass kernel) on one
input: compares it with the one-workgroup-per-item kernel (VIT_ATTN_BWD=one) and reports runs that
differ from the first (nondeterminism) and where.
    python tools/attn_bwd_stress.py [--B 2 --T 197 --NH 3 --runs 30]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitpkg import vit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--T", type=int, default=197)
    ap.add_argument("--NH", type=int, default=3)
    ap.add_argument("--runs", type=int, default=30)
    ap.add_argument("--variant", default="persistent", help="VIT_ATTN_BWD value under test")
    a = ap.parse_args()
    assert vit.lib().vit_init(0) == 0
    B, T, NH, HS = a.B, a.T, a.NH, 64
    C = NH * HS
    rng = np.random.default_rng(T * 7 + NH)
    qb = vit.bf16_bits(rng.normal(size=B * T * 3 * C).astype(np.float32))
    gq = vit.DeviceArray.from_numpy(qb)
    gout = vit.DeviceArray.zeros(B * T * C, np.uint16)
    glse = vit.DeviceArray.zeros(B * NH * T, np.float32)
    vit.call("attention_forward_fused_bf16", gout, glse, gq, B, T, C, NH)
    gdy = vit.DeviceArray.from_numpy(vit.bf16_bits(rng.normal(size=B * T * C).astype(np.float32)))

    def run(variant):
        os.environ["VIT_ATTN_BWD"] = variant
        gd = vit.DeviceArray.zeros(B * T * 3 * C, np.uint16)
        vit.call("attention_backward_fused_bf16", gd, gdy, gq, gout, glse, B, T, C, NH)
        return gd.numpy().reshape(B, T, 3, NH, HS)

    ref = run("one")
    first = run(a.variant)
    f, r = vit.bf16_to_f32(first).astype(np.float64), vit.bf16_to_f32(ref).astype(np.float64)
    print(f"{a.variant} vs one: {(first != ref).sum()} differing values, max |diff| / max |one| = "
          f"{np.abs(f - r).max() / np.abs(r).max():.2e}", flush=True)
    bad = 0
    for k in range(a.runs):
        x = run(a.variant)
        d = x != first
        if d.any():
            bad += 1
            idx = np.argwhere(d)
            print(f"run {k}: {d.sum()} values differ from run 0", flush=True)
            for part in range(3):
                sel = idx[idx[:, 2] == part]
                if len(sel):
                    print(f"   {'qkv'[part]}: b {np.unique(sel[:, 0])} t {np.unique(sel[:, 1])[:40]} "
                          f"h {np.unique(sel[:, 3])} d {np.unique(sel[:, 4])[:16]} n={len(sel)}", flush=True)
    print(f"{bad}/{a.runs} runs differ from the first (nondeterminism)", flush=True)



if __name__ == "__main__":
    main()
