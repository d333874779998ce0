"""One-screen digest of a bench.py JSON line: python scripts/bench_brief.py gpurun_out/bench.log"""
import json
import sys

line = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(line)
r = d["roofline"]
print("C2", round(d["value"] / 1e9, 2), "G rows/s", round(d["ms_per_step"], 3), "ms/step  frac", r["frac"], r["per_kernel_ms"],
      "traffic", r.get("traffic"))
c = d.get("count_only")
if c:
    print("count_only", round(c["ms_per_step"], 3), "ms", c["per_kernel_ms"], "frac", c["kernel_frac"])
c = d.get("filtered")
if c:
    print("filtered", {k: (round(v.get("ms_per_step", v.get("ms", 0)), 3), v["per_kernel_ms"], v["check"]["ok"]) for k, v in c.items()})
c = d.get("c2_float32")
if c:
    print("c2_float32", round(c["ms_per_step"], 3), "ms", c["per_kernel_ms"], "ok", c["check"]["ok"])
for lay in ("groupby", "groupby_sorted_keys"):
    if lay in d:
        print(lay, {k: (round(v["seconds"] * 1e3, 3), v["kernel_ms_last"]) for k, v in d[lay].items() if isinstance(v, dict)})
if "aggs" in d:
    print("aggs", {k: (v["ms"], v["ratio_to_c2"], v["per_kernel_ms"]) for k, v in d["aggs"].items()})
if "h2o" in d:
    print("h2o", {q: (d["h2o"][q]["ms"], d["h2o"][q]["check"]["ok"]) for q in d["h2o"] if q.startswith("q")})
if "ordered_set" in d:
    print("set", {k: d["ordered_set"][k]["ms"] for k in ("random", "sorted")})
if "c4" in d and "frac_of_pinned_h2d" in d["c4"]:
    print("c4", d["c4"]["frac_of_pinned_h2d"])
ck = d["check"]
print("check", ck["ok"], {k: v.get("ok") for k, v in ck.get("prefix_oracle", {}).items()})
