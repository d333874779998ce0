"""Per-kernel table of the PMC passes written by scripts/pmc_passes.sh.
usage: python scripts/pmc_table.py gpurun_out/pmc_<tag> [kernel-substring ...]"""
import glob
import os
import sqlite3
import sys

d = sys.argv[1]
filt = sys.argv[2:]
rows = {}
for db in sorted(glob.glob(os.path.join(d, "p*", "*.db"))):
    con = sqlite3.connect(db)
    for name, ctr, v, c in con.execute("select name, counter_name, avg(counter_value), count(*) from pmc_events group by name, counter_name"):
        k = name.split("(")[0].replace("void ", "")
        rows.setdefault(k, {})[ctr] = v
tr = glob.glob(os.path.join(d, "trace", "*.db"))
avg = {}
if tr:
    con = sqlite3.connect(tr[0])
    for name, calls, a in con.execute("select name, total_calls, average from top_kernels"):
        avg[name.split("(")[0].replace("void ", "")] = (calls, a)
for k, c in sorted(rows.items()):
    if filt and not any(f in k for f in filt):
        continue
    print(k, "calls/avg_us=", avg.get(k))
    for ctr, v in sorted(c.items()):
        extra = ""
        if ctr == "FETCH_SIZE":
            extra = f"  (x2 bytes = {2 * v * 1024 / 1e9:.3f} GB)"
        if ctr == "WRITE_SIZE":
            extra = f"  (bytes = {v * 1024 / 1e9:.3f} GB)"
        print(f"   {ctr:28s} {v:16.1f}{extra}")
