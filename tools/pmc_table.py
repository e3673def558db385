"""Average PMC counter values per kernel from rocprofv3 rocpd databases.
    python tools/pmc_table.py <db> [<db> ...] [--filter substr]"""
import sqlite3
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
flt = None
for a in sys.argv[1:]:
    if a.startswith("--filter="):
        flt = a.split("=", 1)[1]
acc = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for db in args:
    c = sqlite3.connect(db)
    for name, disp, cnt, val, d in c.execute(
            "select kernel_name, dispatch_id, counter_name, sum(value), max(duration) from counters_collection group by dispatch_id, counter_name"):
        if flt and flt not in name:
            continue
        acc[name][cnt].append(val)
        dur[name].append(d)
for name, cs in acc.items():
    print(name[:100], " avg dur us %.1f" % (sum(dur[name]) / len(dur[name]) / 1e3))
    for k in sorted(cs):
        v = cs[k]
        print(f"    {k:28s} {sum(v) / len(v):16.0f}")
