"""Barrier timeline of the ping-pong GEMM engine (variant 11, gemm_pp.hip) from a diagnostic build:
    bash tools/build_variant.sh pptrace csrc/gemm_pp.hip -DVIT_PP_TRACE=1
    VIT_LIB=vit.rs_amd/build_pptrace/libvit_hip.so python tools/pp_trace.py [--only fwd_fc] [--batch 128]
Lane 0 of every wave of workgroups 0..7 stamps s_memtime (shader cycles) when it reaches each barrier
and when it leaves it.  Per tile (nk barriers) this prints, averaged over those workgroups: the main
group's work per K-step interval (leave -> reach), the epilogue group's work per interval, and how long
each group waited at the barrier for the other."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitpkg import vit  # noqa: E402

SHAPES = {
    "fwd_qkv": (2304, 768, 3), "fwd_proj": (768, 768, 5), "fwd_fc": (3072, 768, 8),
    "fwd_fcproj": (768, 3072, 5), "dgrad_fcproj": (3072, 768, 9), "dgrad_fc": (768, 3072, 3),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="fwd_fc,dgrad_fcproj,fwd_proj,dgrad_fc")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--debug", type=int, default=0, help="gemm_bf16_set_debug flags (2: no epilogue)")
    args = ap.parse_args()
    L = vit.lib()
    assert L.vit_init(0) == 0
    M = args.batch * 197
    rng = np.random.default_rng(0)
    mk = lambda n: vit.DeviceArray.from_numpy(vit.bf16_bits(rng.uniform(-1, 1, size=n).astype(np.float32)), np.uint16)
    for name in args.only.split(","):
        N, K, epi = SHAPES[name]
        A, W, aux = mk(M * K), mk(N * K), mk(M * N)
        res = vit.DeviceArray.from_numpy(rng.uniform(-1, 1, size=M * N).astype(np.float32))
        bias = vit.DeviceArray.from_numpy(rng.uniform(-1, 1, size=N).astype(np.float32))
        C = vit.DeviceArray.zeros(M * N, np.float32)
        C2 = vit.DeviceArray.zeros(M * N, np.uint16)
        cs = vit.DeviceArray.zeros(N, np.float32)
        tr = vit.DeviceArray.zeros(8 * 8 * 512, np.uint64)
        L.gemm_bf16_set_variant(11)
        L.gemm_bf16_set_debug(args.debug)

        def run():
            vit.call("gemm_bf16_fused", C, C2 if epi == 8 else None, N, res if epi == 5 else (aux if epi == 9 else None),
                     N, A, K, 1, W, K, 1, bias if epi != 9 else None, cs if epi == 9 else None, M, N, K, epi)
        run()
        L.gemm_bf16_set_trace(tr.ptr)
        run()
        L.vit_sync()
        L.gemm_bf16_set_trace(None)
        L.gemm_bf16_set_debug(0)
        t = tr.numpy().reshape(8, 8, 512).astype(np.int64)
        nk = K // 32
        tiles = (M + 191) // 192 * (N // 256)
        nb = 256
        print(f"\n{name}: M={M} N={N} K={K} epi={epi}, {tiles} tiles, nk={nk}")
        for blk in range(8):
            my = (tiles - blk + nb - 1) // nb
            nbar = 1 + my * nk
            a = t[blk, :, 0:2 * nbar:2]   # reach
            r = t[blk, :, 1:2 * nbar:2]   # leave
            if (a == 0).any():
                print(f"  block {blk}: incomplete record"); continue
            rel = r.max(0)                # release of barrier k
            rows = []
            for j in range(my):
                ks = range(1 + j * nk, 1 + (j + 1) * nk)
                g = j & 1
                mw = [w for w in range(8) if (w >> 2) == g]
                ew = [w for w in range(8) if (w >> 2) != g]
                work_m = np.mean([a[w, k] - rel[k - 1] for w in mw for k in ks])
                work_e = np.mean([a[w, k] - rel[k - 1] for w in ew for k in ks])
                wait_m = np.mean([rel[k] - a[w, k] for w in mw for k in ks])
                wait_e = np.mean([rel[k] - a[w, k] for w in ew for k in ks])
                span = rel[ks[-1]] - rel[ks[0] - 1]
                rows.append((span, work_m, wait_m, work_e, wait_e))
            if blk < 2:
                for j, (sp, wm, wtm, we, wte) in enumerate(rows):
                    print(f"  blk {blk} tile {j}: {sp:7d} cyc = {sp / nk:6.0f}/step | main work {wm:6.0f} wait {wtm:5.0f}"
                          f" | epi work {we:6.0f} wait {wte:5.0f}")
            last = t[blk, :, 2 * nbar - 1].max()
            end = t[blk][t[blk] > 0].max()
            if blk < 2:
                print(f"  blk {blk}: launch span {end - t[blk, :, 0].min()} cyc, after the last barrier {end - last}")


if __name__ == "__main__":
    main()
