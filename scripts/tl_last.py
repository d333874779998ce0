"""Timeline of the last N kernels (and copies) of a rocprofv3 csv run:
python scripts/tl_last.py DIR N  (finds *_kernel_trace.csv under DIR)."""
import csv
import glob
import sys

d, n = sys.argv[1], int(sys.argv[2])
kt = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
ev = [(int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Kernel_Name"][:90]) for k in csv.DictReader(open(kt))]
for c in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
    ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r["Direction"]) for r in csv.DictReader(open(c))]
ev.sort()
ev = ev[-n:]
t0 = prev = ev[0][0]
busy = 0
for s, e, name in ev:
    print(f"{(s - t0) / 1e3:9.1f} us  gap {(s - prev) / 1e3:7.1f}  dur {(e - s) / 1e3:8.1f}  {name}")
    busy += e - s
    prev = max(prev, e)
print(f"span {(prev - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")
