"""Where the MXFP8 streaming engine (f8::gemm_kernel_s) waits, from a diagnostic build:
    bash tools/build_variant.sh f8trace csrc/gemm_fp8.hip -DVIT_F8_TRACE=1
    VIT_LIB=vit.rs_amd/build_f8trace/libvit_hip.so python tools/f8_trace.py [--only fwd_qkv,dgrad_fc]
Lane 0 of every wave of workgroups 0..7 sums shader cycles (s_memtime) spent in the main loops, in
the epilogues, and inside the main loop: waiting for its LDS reads before a barrier (lgkmcnt(0)), in
the barrier itself, and in the counted vmcnt waits for the LDS-DMA ring.  Printed per K-step (64
fp8 elements: 8 scaled 32x32x64 MFMAs per wave, 1024 matrix-pipe cycles for the two waves of a SIMD: 64 per MFMA)
and per tile, averaged over waves 0-3 (leading) and 4-7 (one barrier behind), ViT-H/14 shapes."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitpkg import vit  # noqa: E402

C = 1280
SHAPES = {  # name: N, K, epi
    "fwd_qkv": (3 * C, C, 3), "fwd_proj": (C, C, 5), "fwd_fc": (4 * C, C, 8), "fwd_fcproj": (C, 4 * C, 5),
    "dgrad_fcproj": (4 * C, C, 9), "dgrad_fc": (C, 4 * C, 3), "dgrad_qkv": (C, 3 * C, 3),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="fwd_qkv,dgrad_fc,fwd_fc,dgrad_fcproj")
    ap.add_argument("--M", type=int, default=64 * 257)  # one ViT-H/14 micro-batch
    args = ap.parse_args()
    L = vit.lib()
    assert L.vit_init(0) == 0
    M = args.M
    rng = np.random.default_rng(0)

    def quant(R, K):
        x = vit.DeviceArray.from_numpy(vit.bf16_bits(rng.normal(size=R * K).astype(np.float32)), np.uint16)
        q = vit.DeviceArray.zeros(R * K, np.uint8)
        sc = vit.DeviceArray.zeros(int(L.mx_scale_size(R, K)), np.uint8)
        vit.call("quantize_mx_bf16_ex", q, sc, x, R, K, K, K)
        return q, sc

    for name in args.only.split(","):
        N, K, epi = SHAPES[name]
        qa, sa = quant(M, K)
        qw, sw = quant(N, K)
        out = vit.DeviceArray.zeros(M * N, np.float32)
        out2 = vit.DeviceArray.zeros(M * N, np.uint16)
        aux16 = vit.DeviceArray.from_numpy(vit.bf16_bits(rng.normal(size=M * N).astype(np.float32)), np.uint16)
        aux32 = vit.DeviceArray.from_numpy(rng.normal(size=M * N).astype(np.float32))
        bias = vit.DeviceArray.from_numpy(rng.normal(size=N).astype(np.float32))
        cs = vit.DeviceArray.zeros(N, np.float32)
        tr = vit.DeviceArray.zeros(8 * 8 * 16, np.uint64)

        def run():
            aux = aux16 if epi in (6, 9) else (aux32 if epi == 5 else None)
            vit.call("gemm_fp8_fused", out if epi in (0, 5) else out2, out if epi in (4, 8) else None, N, aux, N,
                     qa, sa, K, qw, sw, K, bias if epi not in (6, 9) else None, cs if epi in (6, 9) else None,
                     M, N, K, epi)
        run()
        L.gemm_bf16_set_trace(tr.ptr)
        e0, e1 = L.vit_event_create(), L.vit_event_create()
        L.vit_event_record(e0)
        run()
        L.vit_event_record(e1)
        L.vit_sync()
        L.gemm_bf16_set_trace(None)
        us = L.vit_event_elapsed_ms(e0, e1) * 1e3
        t = tr.numpy().reshape(8, 8, 16).astype(np.int64)
        tiles, nk = t[:, :, 5], t[:, :, 6]
        print(f"\n{name}: M={M} N={N} K={K} epi={epi}: {us:.1f} us ({2.0 * M * N * K / us / 1e6:.0f} TF/s), "
              f"{int(tiles[0, 0])} tiles x {int(nk[0, 0])} steps on workgroup 0")
        if tiles.max() == 0:
            print("  (no trace: not the diagnostic build, or not the streaming engine)")
            continue
        steps = (tiles * nk).astype(np.float64)
        ghz = np.median(t[:, :, 8] / np.maximum(t[:, :, 9], 1)) * 0.1
        print(f"  in-kernel shader clock {ghz:.2f} GHz (s_memtime / s_memrealtime x 100 MHz, median of 64 waves)")
        for grp, ws in (("waves 0-3", slice(0, 4)), ("waves 4-7", slice(4, 8))):
            s = steps[:, ws]
            main, lgk, bar, vm = (t[:, ws, i] / s for i in range(4))
            epi_c = t[:, ws, 4] / tiles[:, ws]
            work = main - lgk - bar - vm
            print(f"  {grp}: per step {main.mean():6.0f} cyc = work {work.mean():5.0f} + lds wait {lgk.mean():4.0f} "
                  f"+ barrier {bar.mean():5.0f} + dma wait {vm.mean():4.0f}  (MFMA pipe share of the step: "
                  f"{1024 / main.mean() * 100:.0f} %)  | epilogue {epi_c.mean():6.0f} cyc/tile "
                  f"({epi_c.mean() / (main.mean() * nk[0, 0]) * 100:.0f} % of the main loop)")


if __name__ == "__main__":
    main()
