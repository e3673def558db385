"""Per-workgroup timeline of one bf16 GEMM launch (gemm_bf16_set_trace): start, main-loop end and
end of every workgroup (s_memrealtime, 100 MHz) with its CU, for the trainer's ViT-B/16 B=256 shapes.

    python tools/gemm_trace.py [--variants 2,5] [--only fwd_fc,fwd_qkv] [--stagger 0]

Prints per GEMM and engine: launch span, mean main-loop and epilogue time per workgroup, workgroups
per CU, the share of epilogue time during which the CU's other resident workgroup was in its main
loop, and the time from one workgroup's end to the next start on the same CU slot."""
import argparse
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitpkg import vit  # noqa: E402

SHAPES = {  # name: M, N, K, epi (A, W K-contiguous: forward / input-gradient GEMMs)
    "fwd_qkv": (50432, 2304, 768, 3), "fwd_proj": (50432, 768, 768, 5), "fwd_fc": (50432, 3072, 768, 8),
    "fwd_fcproj": (50432, 768, 3072, 5), "dgrad_fcproj": (50432, 3072, 768, 9), "dgrad_fc": (50432, 768, 3072, 3),
}


def analyse(tr, nwaves):
    t0, t1, hw = tr[:, 0].astype(np.int64), tr[:, 1].astype(np.int64), tr[:, 3]
    t2 = tr[:, 4:4 + nwaves].astype(np.int64).max(1)       # last wave's end
    t2w0 = tr[:, 2].astype(np.int64)
    tp = tr[:, 12].astype(np.int64)
    base = t0.min()
    t0, t1, t2, t2w0, tp = t0 - base, t1 - base, t2 - base, t2w0 - base, tp - base
    cu = (hw >> 32) * 4096 + ((hw & 0xFFFFFFFF) >> 8 & 0xFF)
    by = collections.defaultdict(list)
    for i in range(len(t0)):
        by[int(cu[i])].append((t0[i], t1[i], t2[i]))
    over, epi_tot, gaps, conc = 0, 0, [], []
    for k, wgs in by.items():
        wgs.sort()
        for a in wgs:
            e0, e1 = a[1], a[2]
            epi_tot += e1 - e0
            for b in wgs:
                if b is a:
                    continue
                lo, hi = max(e0, b[0]), min(e1, b[1])  # b in its main loop during a's epilogue
                if hi > lo:
                    over += hi - lo
        # residency: max concurrent workgroups on this CU
        ev = sorted([(w[0], 1) for w in wgs] + [(w[2], -1) for w in wgs])
        c = m = 0
        for _, d in ev:
            c += d
            m = max(m, c)
        conc.append(m)
        ends = sorted(w[2] for w in wgs)
        starts = sorted(w[0] for w in wgs)[m:]
        gaps += [s - e for s, e in zip(starts, ends)]
    us = 0.01  # ticks -> us
    return {"span_us": (t2.max()) * us, "main_us": float(np.mean(t1 - t0)) * us,
            "prologue_us": float(np.mean(tp - t0)) * us, "wave_skew_us": float(np.mean(t2 - t2w0)) * us,
            "epi_us": float(np.mean(t2 - t1)) * us, "cus": len(by), "wg_per_cu": len(t0) / len(by),
            "max_resident": int(np.max(conc)), "epi_overlap": over / max(epi_tot, 1),
            "turnaround_us": float(np.median(gaps)) * us if gaps else 0.0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="2,5")
    ap.add_argument("--only", default="fwd_fc,fwd_qkv,fwd_proj")
    ap.add_argument("--stagger", type=int, default=0, help="first-round stagger, 0.5 us units (g4 engines)")
    ap.add_argument("--M", type=int, default=0, help="token rows (default 50432; 25216 = one micro-batch)")
    ap.add_argument("--per-round", action="store_true", help="persistent engine: tile times by round")
    ap.add_argument("--debug", default="0", help="comma-separated extra gemm_bf16_set_debug flags to compare "
                    "(16: the persistent engine drains its stores after each epilogue)")
    args = ap.parse_args()
    L = vit.lib()
    assert L.vit_init(0) == 0
    rng = np.random.default_rng(0)
    Mx, Nx, Kx = 50432, 3072, 3072

    def dev_bf16(n):
        return vit.DeviceArray.from_numpy(vit.bf16_bits(rng.uniform(-1, 1, size=n).astype(np.float32)), np.uint16)

    act, wts = dev_bf16(Mx * Kx), dev_bf16(Nx * Kx)
    aux16, aux32 = dev_bf16(Mx * Nx), vit.DeviceArray.from_numpy(rng.uniform(-1, 1, size=Mx * 768).astype(np.float32))
    out = vit.DeviceArray.zeros(Mx * Nx, np.float32)
    out2 = vit.DeviceArray.zeros(Mx * Nx, np.uint16)
    bias = vit.DeviceArray.from_numpy(rng.uniform(-1, 1, size=Nx).astype(np.float32))
    csum = vit.DeviceArray.zeros(Nx, np.float32)
    trace = vit.DeviceArray.zeros(16 * 8192, np.uint64)
    for name in args.only.split(","):
        M, N, K, epi = SHAPES[name]
        if args.M:
            M = args.M
        for var, dbg in [(int(v), int(d)) for v in args.variants.split(",") for d in args.debug.split(",")]:
            L.gemm_bf16_set_variant(var)
            L.gemm_bf16_set_debug(args.stagger * 256 + dbg)

            def run():
                aux = aux16.ptr if epi in (6, 9) else (aux32.ptr if epi == 5 else None)
                L.gemm_bf16_fused(out.ptr if epi in (0, 5) else out2.ptr, out.ptr if epi in (4, 8) else None, N,
                                  aux, N, act.ptr, K, 1, wts.ptr, K, 1, bias.ptr if epi not in (6, 9) else None,
                                  csum.ptr if epi in (6, 9) else None, M, N, K, epi)
            for _ in range(3):
                run()
            L.vit_sync()
            L.gemm_bf16_set_trace(trace.ptr)
            run()
            L.vit_sync()
            L.gemm_bf16_set_trace(None)
            vit.check(name)
            bm, bn = (256, 256) if var in (2, 7) else (256, 128)
            nwg = -(-M // bm) * -(-N // bn)
            tr = trace.numpy().reshape(-1, 16)[:nwg]
            r = analyse(tr, 8 if var in (2, 7) else 4)
            print(f"{name:13s} v{var} d{dbg} span {r['span_us']:7.1f} us  prologue {r['prologue_us']:5.2f}  main {r['main_us']:6.2f}  "
                  f"epi(last wave) {r['epi_us']:6.2f}  wave-end skew {r['wave_skew_us']:5.2f}  "
                  f"CUs {r['cus']}  wg/CU {r['wg_per_cu']:.1f}  resident {r['max_resident']}  "
                  f"epi beside other's main loop {r['epi_overlap']:.2f}  turnaround {r['turnaround_us']:.2f} us",
                  flush=True)
            if args.per_round:  # tiles of each CU in start order: round j = the CU's j-th tile
                t0, t1 = tr[:, 0].astype(np.int64), tr[:, 1].astype(np.int64)
                t2 = tr[:, 4:12].astype(np.int64).max(1)
                hw = tr[:, 3]
                cu = (hw >> 32) * 4096 + ((hw & 0xFFFFFFFF) >> 8 & 0xFF)
                rounds = collections.defaultdict(list)
                by = collections.defaultdict(list)
                for k in range(len(t0)):
                    by[int(cu[k])].append(k)
                for ks in by.values():
                    for j, k in enumerate(sorted(ks, key=lambda k: t0[k])):
                        rounds[j].append(k)
                base = t0.min()
                for j in sorted(rounds):
                    ks = np.array(rounds[j])
                    print(f"    round {j}: {len(ks):4d} tiles  start {np.mean(t0[ks] - base) * 0.01:7.1f} us  "
                          f"main {np.mean(t1[ks] - t0[ks]) * 0.01:6.2f}  epi {np.mean(t2[ks] - t1[ks]) * 0.01:6.2f} us", flush=True)
    L.gemm_bf16_set_debug(0)
    L.gemm_bf16_set_variant(0)


if __name__ == "__main__":
    main()
