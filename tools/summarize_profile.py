"""Summarise a tools/profile.sh run into profiles/ (tracked).

    python tools/summarize_profile.py r01 [--src gpurun_out/r01]

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied as is)
  profiles/<tag>_bench.json         the bench.py line of the same round
  profiles/<tag>_traffic.json       HBM bytes per dispatch per kernel from the two PMC passes:
                                    FETCH_SIZE x 2 (gfx950 tallies 128-B reads at 64 B,
                                    MI355X_MICROARCH.md "HBM / rocprofv3") + WRITE_SIZE, in bytes
                                    (rocprofv3 reports both counters in KiB)
  profiles/<tag>_summary.md         human-readable table: time share, avg duration, traffic
bench.py reads <tag>_traffic.json (the newest one) to fill roofline.traffic for its dominant
kernel; the kernel symbol of each bench timing class is in CLASS_KERNELS below.
"""
import argparse
import csv
import glob
import json
import os
import re
import shutil
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# bench timing class -> (kernel-name regex, grid x of the launch at ViT-B/16 B=256 or None).
# g2::gemm_kernel<a_kcontig, b_kcontig, epi, ...>; epi numbers from vit.rs_amd/csrc/gemm.h.
CLASS_KERNELS = {
    # epi 9 / 8 (stored gelu' x product, gelu' / gelu pair) since r02b; 6 / 4 before; the persistent
    # streaming engine g2::gemm_kernel_s<epi> since r04
    "gemm_fcproj_dgrad": (r"g2::gemm_kernel(<true, (true|false), |_s<)(6|9)\b", None),  # dgrad B = transposed weight copy since dd2b73c
    "gemm_fc_fwd": (r"g2::gemm_kernel(<true, true, |_s<)(4|8)\b", None),
    "gemm_qkv_fwd": (r"g2::gemm_kernel(<true, true, |_s<)3\b", None),
    "gemm_proj_dgrad": (r"g2::gemm_kernel<true, false, 3\b", None),
    "attention_bwd": (r"attn_bwd(p|1|_pair)_k", None),
    "attention_fwd": (r"attn_fwd_k", None),
}


# one kernel instance serving two classes, told apart per dispatch by traffic: the fp32-residual
# epilogue runs proj fwd (A 1 x C wide) and fcproj fwd (A 4 x C wide) alternately in every layer;
# the smaller half of its dispatches (by bytes) is proj fwd, the larger fcproj fwd
SPLIT_KERNELS = {
    r"g2::gemm_kernel(<true, true, |_s<)5\b": ("gemm_proj_fwd", "gemm_fcproj_fwd"),
}


def find(src, pattern):
    hits = glob.glob(os.path.join(src, "**", pattern), recursive=True)
    return sorted(hits)[0] if hits else None


def read_pmc(path, counter):
    """-> {kernel_name: [bytes per dispatch, ...]}"""
    out = defaultdict(list)
    if not path:
        return out
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            out[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--src", default=None)
    a = ap.parse_args()
    src = a.src or os.path.join(ROOT, "gpurun_out", a.tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)

    stats_csv = find(os.path.join(src, "ktrace"), "*kernel_stats.csv")
    assert stats_csv, f"no kernel_stats.csv under {src}/ktrace"
    shutil.copy(stats_csv, os.path.join(dst, f"{a.tag}_kernel_stats.csv"))
    with open(stats_csv) as f:
        stats = list(csv.DictReader(f))

    bench = None
    bj = os.path.join(src, "bench.json")
    if os.path.exists(bj) and os.path.getsize(bj):
        bench = json.loads(open(bj).read().strip().splitlines()[-1])
        with open(os.path.join(dst, f"{a.tag}_bench.json"), "w") as f:
            json.dump(bench, f, indent=1)

    fetch = read_pmc(find(os.path.join(src, "pmc_fetch"), "*counter_collection.csv"), "FETCH_SIZE")
    write = read_pmc(find(os.path.join(src, "pmc_write"), "*counter_collection.csv"), "WRITE_SIZE")
    traffic = {}
    for k in set(fetch) | set(write):
        fr, wr = fetch.get(k, []), write.get(k, [])
        rd = 2.0 * sum(fr) / len(fr) if fr else None
        wb = sum(wr) / len(wr) if wr else None
        traffic[k] = {"dispatches": max(len(fr), len(wr)), "read_bytes": rd, "write_bytes": wb,
                      "bytes_per_dispatch": (rd or 0.0) + (wb or 0.0)}
    classes = {}
    for cls, (rx, _) in CLASS_KERNELS.items():
        ks = [k for k in traffic if re.search(rx, k)]
        if ks:
            tot = sum(traffic[k]["bytes_per_dispatch"] * traffic[k]["dispatches"] for k in ks)
            n = sum(traffic[k]["dispatches"] for k in ks)
            classes[cls] = {"kernels": ks, "bytes_per_dispatch": tot / n}
    for rx, (lo_cls, hi_cls) in SPLIT_KERNELS.items():
        for k in set(fetch) & set(write):
            if not re.search(rx, k) or len(fetch[k]) != len(write[k]) or len(fetch[k]) < 2:
                continue
            per = sorted(2.0 * f_ + w_ for f_, w_ in zip(fetch[k], write[k]))
            h = len(per) // 2
            classes[lo_cls] = {"kernels": [k], "bytes_per_dispatch": sum(per[:h]) / h, "split": "smaller half"}
            classes[hi_cls] = {"kernels": [k], "bytes_per_dispatch": sum(per[h:]) / (len(per) - h),
                               "split": "larger half"}
    with open(os.path.join(dst, f"{a.tag}_traffic.json"), "w") as f:
        json.dump({"tag": a.tag, "correction": "FETCH_SIZE*2 + WRITE_SIZE, KiB->bytes",
                   "classes": classes, "kernels": traffic}, f, indent=1)

    tot_ns = sum(float(r["TotalDurationNs"]) for r in stats)
    lines = [f"# Profile {a.tag}", "",
             "rocprofv3 --kernel-trace --stats over `bench.py --steps 5 --warmup 2` (ViT-B/16, B=256, "
             "1x MI355X); traffic from separate FETCH_SIZE / WRITE_SIZE passes (1 step).", ""]
    if bench:
        lines += [f"bench: {bench['value']} {bench['unit']}, {bench['ms_per_step']} ms/step, "
                  f"roofline {json.dumps(bench.get('roofline'))}", ""]
    lines += ["| kernel | calls | total ms | avg us | % | HBM MB/dispatch |", "|---|---|---|---|---|---|"]
    for r in sorted(stats, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
        name = r["Name"]
        t = traffic.get(name)
        mb = f"{t['bytes_per_dispatch'] / 1e6:.1f}" if t else "-"
        lines.append(f"| `{name[:90]}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                     f"{float(r['AverageNs']) / 1e3:.1f} | {100 * float(r['TotalDurationNs']) / tot_ns:.1f} | {mb} |")
    with open(os.path.join(dst, f"{a.tag}_summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines[:40]))


if __name__ == "__main__":
    main()
