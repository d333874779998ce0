"""Per-query GPU timeline from a rocprofv3 --kernel-trace --memory-copy-trace csv pair:
python scripts/tl_summary.py DIR/PREFIX FIRST_KERNEL_SUBSTRING [query index, default last]."""
import csv
import sys

pre, mark = sys.argv[1], sys.argv[2]
which = int(sys.argv[3]) if len(sys.argv) > 3 else -1
ev = [(int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Kernel_Name"][:70])
      for k in csv.DictReader(open(pre + "_kernel_trace.csv"))]
try:
    ev += [(int(c["Start_Timestamp"]), int(c["End_Timestamp"]), "COPY " + c["Direction"])
           for c in csv.DictReader(open(pre + "_memory_copy_trace.csv"))]
except FileNotFoundError:
    pass
ev.sort()
starts = [i for i, e in enumerate(ev) if mark in e[2]]
a = starts[which]
b = starts[which + 1] if which != -1 and which + 1 < len(starts) else len(ev)
t0 = prev = ev[a][0]
busy = 0
for s, e, n in ev[a:b]:
    print(f"{(s - t0) / 1e3:9.1f} us  gap {(s - prev) / 1e3:7.1f}  dur {(e - s) / 1e3:8.1f}  {n}")
    busy += e - s
    prev = max(prev, e)
print(f"span {(prev - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle {(prev - t0 - busy) / 1e3:.1f} us")
