"""Per-kernel time summary from a rocprofv3 rocpd database (the `kernels` view).
    python tools/kstats.py gpurun_out/prof3/run_results.db [top]"""
import sqlite3
import sys

db = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
rows = c.execute(f"select {name_col}, count(*), sum(end-start), avg(end-start) from kernels group by {name_col} order by sum(end-start) desc").fetchall()
tot = sum(r[2] for r in rows)
print(f"{'kernel':90s} {'calls':>6s} {'total_ms':>9s} {'avg_us':>9s} {'%':>5s}")
for n, k, s, a in rows[:top]:
    print(f"{n[:90]:90s} {k:6d} {s / 1e6:9.3f} {a / 1e3:9.1f} {100 * s / tot:5.1f}")
print("total ms", tot / 1e6)
