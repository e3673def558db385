"""MFMA utilisation per kernel from a rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE pass.
    python tools/mfma_util.py gpurun_out/r01e_mfma/run_counter_collection.csv > profiles/r01e_mfma_util.md
SQ_VALU_MFMA_BUSY_CYCLES counts matrix-core busy cycles summed over the chip's SIMDs (32 per
v_mfma_f32_32x32x16_bf16, 16 per 16x16x32, MI355X_MICROARCH.md); GRBM_GUI_ACTIVE is summed over the
8 XCDs, so the kernel's clock cycles are GRBM_GUI_ACTIVE / 8 and the effective clock is that over
the dispatch's wall time.  util = MFMA_BUSY / (cycles * 256 CUs * 4 SIMDs)."""
import csv
import sys
from collections import defaultdict

SIMDS = 256 * 4
rows = defaultdict(dict)
for r in csv.DictReader(open(sys.argv[1])):
    d = rows[int(r["Dispatch_Id"])]
    d["name"] = r["Kernel_Name"]
    d["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
agg = defaultdict(lambda: [0, 0.0, 0.0, 0.0])
for d in rows.values():
    if "SQ_VALU_MFMA_BUSY_CYCLES" not in d or "GRBM_GUI_ACTIVE" not in d:
        continue
    a = agg[d["name"]]
    a[0] += 1
    a[1] += d["dur"]
    a[2] += d["SQ_VALU_MFMA_BUSY_CYCLES"]
    a[3] += d["GRBM_GUI_ACTIVE"] / 8
tot = sum(a[1] for a in agg.values())
print("| kernel | calls | avg us | % time | MFMA busy (util) | eff. clock GHz |")
print("|---|---|---|---|---|---|")
busy_t = cyc_t = 0.0
for name, (n, dur, busy, cyc) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    if dur / tot < 0.002:
        continue
    util = busy / (cyc * SIMDS) if cyc else 0.0
    clk = cyc / dur / 1e9 if dur else 0.0
    busy_t += busy
    cyc_t += cyc
    print(f"| `{name[:90]}` | {n} | {dur / n * 1e6:.1f} | {100 * dur / tot:.1f} | {100 * util:.1f} % | {clk:.2f} |")
print(f"\nall listed kernels: MFMA busy {100 * busy_t / (cyc_t * SIMDS):.1f} % of SIMD-cycles "
      f"(kernels serialised, one step)")
