"""Print the key numbers of a bench.py JSON line (file argument)."""
import json
import sys

d = None
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
r = d["roofline"]
print("headline rows/s %.4g  ms/step %.3f  passA %.3f ms frac %.4f  per_kernel %s" % (
    d["value"], d["ms_per_step"], r["kernel_ms"], r["frac"], r["per_kernel_ms"]))
if "zero_d" in d:
    z = d["zero_d"]
    print("zero_d sum %.3f ms (kernel %.3f, %.3f frac)  mean %.3f ms  count %.3f ms" % (
        z["sum"]["ms"], z["sum"]["kernel_ms"], z["sum"]["kernel_frac"], z["mean"]["ms"], z["count"]["ms"]))
if "c2_sorted_y" in d:
    c = d["c2_sorted_y"]
    print("c2 sorted y %.3f ms  overflow/step %d  ok %s" % (c["ms_per_step"], c["overflow_rows_per_step"], c["count_equal"]))
for k in ("groupby", "groupby_sorted_keys"):
    if k in d:
        g = d[k]
        for m in ("auto", "fused", "hash"):
            print("%-20s %-6s %7.2f ms ok=%s overflow=%s kernels=%s" % (k, m, g[m]["seconds"] * 1e3, g[m]["check"]["ok"],
                                                                     g[m].get("overflow_rows"), g[m]["kernel_ms_last"]))
if "count_only" in d:
    c = d["count_only"]
    print("count_only %.3f ms  %s  frac %.4f pipeline %.4f" % (c["ms_per_step"], c["per_kernel_ms"], c["kernel_frac"],
                                                              c["pipeline_frac"]))
for k in ("c1", "c4", "host_columns", "cpu_baseline"):
    if d.get(k):
        print(k, json.dumps(d[k])[:400])
print("check", d["check"])
