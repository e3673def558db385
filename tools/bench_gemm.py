"""Microbenchmark of the bf16 GEMM engines at the trainer's ViT-B/16 B=256 GEMMs (HIP events).

    python tools/bench_gemm.py [--iters 10] [--variants 2,4] [--no-epi]

Every GEMM of one transformer layer (forward, dgrad, wgrad) with the epilogue the trainer uses
(bias, GELU pair, fp32 residual, GELU' with the fused fc-bias column sum, split-K slabs).  Engines
are A/B'd in ONE process, interleaved round by round (cdna_hip_programming.md §5.4 rule 24); the
median over rounds is printed.  --no-epi adds main-loop-only rows (gemm_bf16_set_debug(2)).
Operands are uniform [-1, 1) bf16 (random data: zero-filled operands read ~20 % fast).
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitpkg import vit  # noqa: E402


FP8 = 108  # pseudo-variant column: the MXFP8 engine


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--C", type=int, default=768)
    ap.add_argument("--variants", default="2,4")
    ap.add_argument("--no-epi", action="store_true")
    ap.add_argument("--modes", default=None,  # 256*n: first-round stagger of n s_sleep(127)
                    help="comma-separated gemm_bf16_set_debug flag sets to A/B (2 = no epilogue, "
                         "4 = g2 prefetch depth 3); default 0 (and 2 with --no-epi)")
    ap.add_argument("--only", default=None, help="comma-separated GEMM names")
    ap.add_argument("--fp8", action="store_true",
                    help="also time the MXFP8 engine (column v108) on the forward / dgrad GEMMs")
    args = ap.parse_args()
    L = vit.lib()
    assert L.vit_init(0) == 0
    C, BT = args.C, args.batch * 197
    rng = np.random.default_rng(0)
    big = BT * 4 * C

    def dev_bf16(n):
        return vit.DeviceArray.from_numpy(vit.bf16_bits(rng.uniform(-1, 1, size=n).astype(np.float32)), np.uint16)

    act = dev_bf16(big)       # A operands (activations / output gradients)
    act2 = dev_bf16(big)      # B operand of wgrad
    wts = dev_bf16(4 * C * C)  # weights
    aux16 = dev_bf16(big)     # GELU' input
    aux32 = vit.DeviceArray.from_numpy(rng.uniform(-1, 1, size=BT * C).astype(np.float32))
    out = vit.DeviceArray.zeros(big, np.float32)
    out2 = vit.DeviceArray.zeros(big, np.uint16)
    bias = vit.DeviceArray.from_numpy(rng.uniform(-1, 1, size=4 * C).astype(np.float32))
    csum = vit.DeviceArray.zeros(4 * C, np.float32)
    e0, e1 = L.vit_event_create(), L.vit_event_create()
    if args.fp8:  # MXFP8 copies of the A and weight operands (quantized once)
        q_act = vit.DeviceArray.zeros(big, np.uint8)
        s_act = vit.DeviceArray.zeros(int(L.mx_scale_size(BT, 4 * C)) * 4, np.uint8)
        q_w = vit.DeviceArray.zeros(4 * C * C, np.uint8)
        s_w = vit.DeviceArray.zeros(int(L.mx_scale_size(4 * C, 4 * C)) * 4, np.uint8)

    # name, M, N, K, a_kcontig, lda, b_kcontig, ldb, epi
    g = [
        ("fwd_qkv", BT, 3 * C, C, 1, C, 1, C, 3),
        ("fwd_proj", BT, C, C, 1, C, 1, C, 5),
        ("fwd_fc", BT, 4 * C, C, 1, C, 1, C, 8),  # the trainer's gelu' / gelu pair (epi 4: pre / gelu)
        ("fwd_fcproj", BT, C, 4 * C, 1, 4 * C, 1, 4 * C, 5),
        # dgrads read the transposed weight copy (K-contiguous), as the trainer does
        ("dgrad_fcproj", BT, 4 * C, C, 1, C, 1, C, 9),  # x stored gelu' + colsum (epi 6: gelu' here)
        ("dgrad_fc", BT, C, 4 * C, 1, 4 * C, 1, 4 * C, 3),
        ("dgrad_proj", BT, C, C, 1, C, 1, C, 3),
        ("dgrad_qkv", BT, C, 3 * C, 1, 3 * C, 1, 3 * C, 3),
        ("wgrad_fcproj", C, 4 * C, BT, 0, C, 0, 4 * C, 2),
        ("wgrad_fc", 4 * C, C, BT, 0, 4 * C, 0, C, 2),
        ("wgrad_proj", C, C, BT, 0, C, 0, C, 2),
        ("wgrad_qkv", 3 * C, C, BT, 0, 3 * C, 0, C, 2),
    ]
    if args.only:
        keep = set(args.only.split(","))
        g = [x for x in g if x[0] in keep]
    variants = [int(v) for v in args.variants.split(",")] + ([FP8] if args.fp8 else [])
    modes = [int(x) for x in args.modes.split(",")] if args.modes else ([0, 2] if args.no_epi else [0])

    def run(name, M, N, K, ak, lda, bk, ldb, epi, var=2):
        if var == FP8:
            if epi == 2:
                return
            aux = aux16.ptr if epi in (6, 9) else (aux32.ptr if epi == 5 else None)
            L.gemm_fp8_fused(out.ptr if epi in (0, 5) else out2.ptr, out.ptr if epi in (4, 8) else None, N, aux, N,
                             q_act.ptr, s_act.ptr, K, q_w.ptr, s_w.ptr, K, bias.ptr if epi not in (6, 9) else None,
                             csum.ptr if epi in (6, 9) else None, M, N, K, epi)
            return
        if epi == 2:
            L.gemm_bf16_ex(out.ptr, N, act.ptr, lda, ak, act2.ptr, ldb, bk, None, None, M, N, K, 2, 0)
        else:
            aux = aux16.ptr if epi in (6, 9) else (aux32.ptr if epi == 5 else None)
            L.gemm_bf16_fused(out.ptr if epi in (0, 5) else out2.ptr, out.ptr if epi in (4, 8) else None, N,
                              aux, N, act.ptr, lda, ak, wts.ptr, ldb, bk,
                              bias.ptr if epi not in (6, 9) else None, csum.ptr if epi in (6, 9) else None,
                              M, N, K, epi)

    res = {}
    for rd in range(args.rounds):
        for sh in g:
            for var in variants:
                for mode in modes:
                    if var == FP8 and sh[8] == 2:
                        continue
                    if var == FP8:  # operands of this shape quantized (untimed)
                        L.quantize_mx_bf16_ex(q_act.ptr, s_act.ptr, act.ptr, sh[1], sh[3], sh[3], sh[3])
                        L.quantize_mx_bf16_ex(q_w.ptr, s_w.ptr, wts.ptr, sh[2], sh[3], sh[3], sh[3])
                    L.gemm_bf16_set_variant(var if var != FP8 else 0)
                    L.gemm_bf16_set_debug(mode)
                    for _ in range(2):
                        run(*sh, var=var)
                    L.vit_sync()
                    vit.check(sh[0])
                    L.vit_event_record(e0)
                    for _ in range(args.iters):
                        run(*sh, var=var)
                    L.vit_event_record(e1)
                    L.vit_sync()
                    ms = L.vit_event_elapsed_ms(e0, e1) / args.iters
                    vit.check(sh[0])
                    res.setdefault((sh[0], var, mode), []).append(ms)
    L.gemm_bf16_set_debug(0)
    tot = {}
    print(f"{'gemm':14s} {'M':>6s} {'N':>5s} {'K':>6s} epi " +
          " ".join(f"{'v%d/f%d' % (v, m):>16s}" for v in variants for m in modes))
    for sh in g:
        name, M, N, K = sh[:4]
        fl = 2.0 * M * N * K
        cells = []
        for v in variants:
            for m in modes:
                if (name, v, m) not in res:
                    cells.append("-")
                    continue
                ms = float(np.median(res[(name, v, m)]))
                tot[(v, m)] = tot.get((v, m), 0.0) + ms
                cells.append(f"{ms * 1e3:7.1f}us {fl / ms / 1e9:6.0f}TF")
        print(f"{name:14s} {M:6d} {N:5d} {K:6d} {sh[8]:3d} " + " ".join(f"{c:>16s}" for c in cells), flush=True)
    fl_all = sum(2.0 * x[1] * x[2] * x[3] for x in g)
    print("total per layer: " + "  ".join(
        f"v{v}/f{m} {tot[(v, m)]:.3f} ms ({fl_all / tot[(v, m)] / 1e9:.0f} TF/s)"
        for v in variants for m in modes if v != FP8))


if __name__ == "__main__":
    main()
