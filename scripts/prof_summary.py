"""Summarise a rocprofv3 run (rocpd SQLite output) into a text table for profiles/.

usage: python scripts/prof_summary.py gpurun_out/prof_<tag> [profiles/<tag>_pmc.json ROWS] > profiles/<tag>.txt
Per kernel: calls, average duration (us; rocpd top_kernels reports us), and the PMC counters collected in the separate
--pmc passes (FETCH_SIZE / WRITE_SIZE, kB per dispatch as rocprofv3 reports them).  Per
MI355X_MICROARCH.md §HBM, FETCH_SIZE on gfx950 reads half the bytes of a wide coalesced
streaming read: the 'fetch_GB_x2' column doubles it.  Units: rocprofv3 reports both counters
in KiB (bytes = value * 1024, cdna_hip_programming.md §7).  With a second argument the
per-kernel numbers are also written as JSON (bench.py reads the HBM traffic from it).
"""
import glob
import os
import sqlite3
import sys


def short(name):
    return name.split("(")[0].replace("void ", "")


def kernel_stats(db):
    con = sqlite3.connect(db)
    rows = con.execute("select name, total_calls, total_duration, average from top_kernels").fetchall()
    return {short(n): (c, tot, avg) for n, c, tot, avg in rows}


def pmc(db):
    con = sqlite3.connect(db)
    rows = con.execute("select name, counter_name, avg(counter_value), count(*) from pmc_events group by name, counter_name").fetchall()
    return {(short(n), c): v for n, c, v, _ in rows}


def main(d, json_path=None, rows=None):
    out = {}
    trace = glob.glob(os.path.join(d, "trace", "*.db"))[0]
    ks = kernel_stats(trace)
    counters = {}
    for sub in ("fetch", "write"):
        f = glob.glob(os.path.join(d, sub, "*.db"))
        if f:
            counters.update(pmc(f[0]))
    print(f"# rocprofv3 --kernel-trace --stats summary of {d}")
    print(f"{'kernel':60s} {'calls':>6s} {'avg_us':>11s} {'total_ms':>10s} {'FETCH_kB':>12s} {'fetch_GB_x2':>11s} {'WRITE_kB':>12s}")
    for k, (c, tot, avg) in sorted(ks.items(), key=lambda kv: -kv[1][1]):
        f = counters.get((k, "FETCH_SIZE"))
        w = counters.get((k, "WRITE_SIZE"))
        fs = f"{f:12.0f}" if f is not None else f"{'-':>12s}"
        f2 = f"{2 * f * 1024 / 1e9:11.3f}" if f is not None else f"{'-':>11s}"
        ws = f"{w:12.0f}" if w is not None else f"{'-':>12s}"
        print(f"{k[:60]:60s} {c:6d} {avg:11.2f} {tot / 1e3:10.3f} {fs} {f2} {ws}")
        out[k] = {"calls": c, "avg_us": avg, "fetch_bytes_x2": None if f is None else 2 * f * 1024,
                  "write_bytes": None if w is None else w * 1024}
    if json_path:
        import json
        with open(json_path, "w") as fh:
            json.dump({"source": d, "rows": rows, "bins": 1024, "kernels": out}, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None, int(float(sys.argv[3])) if len(sys.argv) > 3 else None)
