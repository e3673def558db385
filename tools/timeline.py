"""Concurrency analysis of a rocprofv3 kernel trace: for the last N steps (split at sgd_bf16_k),
the wall span, the union of busy intervals, and per-stream / per-kernel busy time.
    python tools/timeline.py gpurun_out/tl/run_results.db|run_kernel_trace.csv [steps]"""
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
if db.endswith(".csv"):  # rocprofv3 --output-format csv kernel trace
    import csv
    rows = sorted(((r["Kernel_Name"], int(r["Stream_Id"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                   for r in csv.DictReader(open(db))), key=lambda r: r[2])
else:
    c = sqlite3.connect(db)
    rows = c.execute("select name, stream_id, start, end from kernels order by start").fetchall()
sgd = [i for i, r in enumerate(rows) if "sgd_bf16_k" in r[0]]
lo, hi = sgd[-nsteps - 1] + 1, sgd[-1] + 1
seg = rows[lo:hi]
t0, t1 = seg[0][2], max(r[3] for r in seg)
span = t1 - t0
iv = sorted((r[2], r[3]) for r in seg)
busy, cs, ce = 0, iv[0][0], iv[0][1]
for s, e in iv[1:]:
    if s > ce:
        busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
tot = sum(r[3] - r[2] for r in seg)
print(f"steps {nsteps}: span {span / 1e6 / nsteps:.2f} ms/step, GPU busy (union) {busy / 1e6 / nsteps:.2f}, "
      f"sum of kernel durations {tot / 1e6 / nsteps:.2f} (overlap factor {tot / busy:.2f})")
per_stream = defaultdict(int)
for r in seg:
    per_stream[r[1]] += r[3] - r[2]
for k, v in sorted(per_stream.items()):
    print(f"  stream {k}: {v / 1e6 / nsteps:.2f} ms/step busy")
per_k = defaultdict(lambda: [0, 0])
for r in seg:
    per_k[r[0][:80]][0] += r[3] - r[2]
    per_k[r[0][:80]][1] += 1
for k, v in sorted(per_k.items(), key=lambda kv: -kv[1][0])[:12]:
    print(f"  {v[0] / 1e6 / nsteps:7.2f} ms/step  n={v[1] // nsteps:4d}  {k}")
