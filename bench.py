"""Benchmark of the binned-statistics hot path on MI355X (BASELINE.json configs[1] at N=1).

One step = one query pass over resident synthetic columns:
``count(binby=[x, y], limits=[[-4, 4], [-4, 4]], shape=1024)`` + ``sum(w)`` on the same
binners (one merged pass, as ExecutorLocal merges them), 1e9 float64 rows per GPU
(weak scaling), through the superagg surface -> libvaexhip C-ABI -> HIP kernels; with
N > 1 GPUs the rows are sharded by rank and the dense grids are all-reduced over RCCL.
Fresh aggregator grids are created in every step (as a query does), and every step reads
both grids back to host numpy arrays (get_result, cpu.py:592-605) inside the timed region.
The roofline's kernel durations come from HIP events in a second, instrumented run of the
same steps (no timers inside the timed region).

Prints ONE JSON line (rank 0) with the roofline of the binning pipeline (HIP events on the
library stream) and the CPU baseline (the oracle's C restatement with the reference
threading model, on a bounded sample, rank 0 at N=1 only).
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_METRIC = "rows/sec 2D count grid 1e9×f64 + groupby-sum 1e6 keys; HBM GB/s %peak"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
TILE_KERNELS = ["tile_sample", "tile_scatter", "tile_scatter_f64", "tile_scatter_ord", "tile_scatter_set", "tile_reduce"]


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--rows", type=float, default=1e9, help="rows per GPU")
    p.add_argument("--bins", type=int, default=1024)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline work")
    p.add_argument("--no-groupby", action="store_true")
    p.add_argument("--no-count-only", action="store_true")
    p.add_argument("--no-f32", action="store_true", help="skip the C2 leg on float32 copies of x, y, w")
    p.add_argument("--no-filtered", action="store_true", help="skip the selection / filtered-groupby legs")
    p.add_argument("--no-layouts", action="store_true", help="skip the sorted-layout legs")
    p.add_argument("--host-rows", type=float, default=2e8,
                   help="rows of the PCIe-inclusive measurement (host numpy columns); 0 = skip")
    p.add_argument("--groupby-rows", type=float, default=1e9)
    p.add_argument("--c4-rows", type=float, default=2e9,
                   help="rows of the C4 leg (2D mean streamed from a memory-mapped HDF5 file); 0 = skip")
    p.add_argument("--h2o-rows", type=float, default=1e9,
                   help="rows of the h2o G1 leg (benchmarks/groupbyh2o.py q1-q5, q7, q10); 0 = skip")
    p.add_argument("--dist-groupby-rows", type=float, default=1e9, help="C3 rows per rank of the multi-GPU groupby legs")
    p.add_argument("--dist-h2o-rows", type=float, default=2.5e8, help="h2o rows per rank of the multi-GPU leg; 0 = skip")
    p.add_argument("--check", action="store_true", help="verify size-independent properties")
    p.add_argument("--breakdown", action="store_true", help="print host-side timing of one step")
    p.add_argument("--no-aggs", action="store_true", help="skip the first / var legs on the C2 grid")
    p.add_argument("--no-set", action="store_true", help="skip the ordered_set.update leg")
    p.add_argument("--dry-launch", action="store_true",
                   help="(launcher test) every rank prints its rank environment and exits before any GPU call")
    p.add_argument("--dry-launch-fail-rank", type=int, default=-1,
                   help="(launcher test) with --dry-launch, this rank exits with status 3")
    return p.parse_args()


def launch_ranks(args, argv):
    """``--gpus N`` (N > 1) without a launcher: start N rank processes of this script, one per
    GPU, as torch.distributed.run would (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
    MASTER_PORT in each child's environment), wait for all of them and return a non-zero
    status when any fails (the others are then terminated: they would wait at the first
    collective forever).  The children inherit stdout, so rank 0's JSON line is this
    command's output.  Runs before anything imports vaex_amd or touches the GPU, and starts
    children (never exec), so this process stays GPU-free.  Replaces the reference's thread
    fan-out over chunks (execution.py:214-289) at process-per-GPU granularity."""
    import socket
    import subprocess
    n = args.gpus
    # two free ports: MASTER_PORT and the host channel's (vaex_amd.comm, VAEX_AMD_COMM_PORT)
    with socket.socket() as s1, socket.socket() as s2:
        s1.bind(("127.0.0.1", 0))
        s2.bind(("127.0.0.1", 0))
        port, comm_port = s1.getsockname()[1], s2.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), VAEX_AMD_COMM_PORT=str(comm_port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    alive = set(range(n))
    while alive:
        for r in sorted(alive):
            c = procs[r].poll()
            if c is None:
                continue
            alive.discard(r)
            if c != 0 and rc == 0:
                print(f"bench.py: rank {r} exited with status {c}; stopping the other ranks", file=sys.stderr, flush=True)
                rc = c if c > 0 else 1
                for q in alive:
                    procs[q].terminate()
        time.sleep(0.05)
    return rc


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_launch:
        print(json.dumps({"rank": rank, "local_rank": local_rank, "world": world, "gpus": args.gpus,
                          "master_addr": os.environ.get("MASTER_ADDR"), "master_port": os.environ.get("MASTER_PORT"),
                          "pid": os.getpid()}), flush=True)
        sys.exit(3 if rank == args.dry_launch_fail_rank else 0)
    dist = None
    import vaex_amd
    from vaex_amd import _lib, superagg
    from vaex_amd.device import DeviceArray
    from vaex_amd import distributed as vdist

    _lib.call("vh_set_device", local_rank)
    # BENCH_FORCE_DIST=1: the N>1 code path (RCCL communicator, grid all-reduce,
    # max-over-ranks timing) on a single rank, to exercise it on a one-GPU box
    if world > 1 or os.environ.get("BENCH_FORCE_DIST"):
        from vaex_amd import comm as vcomm
        dist = vcomm.init("rccl")
    # the world RCCL actually reduced over: an all-reduce of one per rank through the
    # communicator (None without one)
    rccl_ranks = int(dist.allreduce(np.ones(1, np.int64))[0]) if dist is not None else None
    n = int(args.rows)
    bins = args.bins
    # resident synthetic columns (each rank its own shard: seeds offset by rank)
    x = DeviceArray.random(n, "normal", seed=2 + 1000 * rank)
    y = DeviceArray.random(n, "normal", seed=3 + 1000 * rank)
    w = DeviceArray.random(n, "uniform", seed=4 + 1000 * rank)

    def step():
        bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, bins)
        by = superagg.BinnerScalar_float64("y", -4.0, 4.0, bins)
        bx.set_data(x)
        by.set_data(y)
        grid = superagg.Grid([bx, by])
        count = superagg.AggCount_int64(grid)
        total = superagg.AggSum_float64(grid)
        total.set_data(w, 0)
        grid.bin([count, total])
        if dist is not None:
            vdist.allreduce_aggs([count, total])
        # the grids read back to host numpy arrays, as get_result does (cpu.py:592-605)
        return np.asarray(count), np.asarray(total)

    def barrier():
        if dist is not None:
            vdist.barrier()
        _lib.synchronize()

    for _ in range(args.warmup):
        step()
    if args.breakdown and rank == 0:
        _lib.synchronize()
        t = [time.perf_counter()]
        bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, bins)
        by = superagg.BinnerScalar_float64("y", -4.0, 4.0, bins)
        bx.set_data(x)
        by.set_data(y)
        grid = superagg.Grid([bx, by])
        t.append(time.perf_counter())
        count = superagg.AggCount_int64(grid)
        total = superagg.AggSum_float64(grid)
        total.set_data(w, 0)
        t.append(time.perf_counter())
        grid.bin([count, total])
        t.append(time.perf_counter())
        np.asarray(count), np.asarray(total)
        t.append(time.perf_counter())
        del count, total, grid
        t.append(time.perf_counter())
        print("breakdown_ms", {k: round((b - a) * 1e3, 3) for k, a, b in
                               zip(["grid", "aggs", "bin", "read_back", "free"], t, t[1:])}, flush=True)
    # timed region: no HIP-event timers inside it
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if dist is not None:
        elapsed = vdist.allreduce_scalar(elapsed, "max")
    ms_per_step = elapsed / args.steps * 1e3
    total_rows = n * world * args.steps
    value = total_rows / elapsed

    # per-kernel HIP-event durations from a separate instrumented run of the same steps
    _lib.timing_reset()
    _lib.timing_enable(True)
    for _ in range(args.steps):
        step()
    _lib.synchronize()
    _lib.timing_enable(False)

    # roofline of the dominant kernel (pass A of the tiled path): algorithmic bytes = 24 B/row
    # (x, y, w read once) x rows per launch / its average HIP-event duration
    kernel_ms = {}
    for k in TILE_KERNELS + ["bin_fused_global", "bin_fused_lds"]:
        cnt, ms = _lib.timing_read(k)
        if cnt:
            kernel_ms[k] = (cnt, ms)
    algo_bytes = 24 * n
    dom = max(kernel_ms, key=lambda k: kernel_ms[k][1]) if kernel_ms else None
    dom_ms = kernel_ms[dom][1] / kernel_ms[dom][0] if dom else None
    achieved = algo_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms else None
    launches = max([c for c, _ in kernel_ms.values()] or [1])
    pipeline_ms = sum(ms for _, ms in kernel_ms.values()) / max(launches, 1)
    roofline = {
        "bound": "hbm",
        "kernel": dom,
        "achieved": round(achieved, 1) if achieved else None,
        "peak": HBM_PEAK_GBPS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBPS, 4) if achieved else None,
        "traffic": None,
        "algorithmic_bytes_per_launch": algo_bytes,
        "kernel_ms": round(dom_ms, 4) if dom_ms else None,
        "kernel_timing": "HIP events on the library stream, a second instrumented run of the same steps",
        "per_kernel_ms": {k: round(ms / c, 4) for k, (c, ms) in kernel_ms.items()},
        # whole binning pipeline (sample + pass A + pass B) against the same 24 B/row
        "pipeline_ms": round(pipeline_ms, 4),
        "pipeline_achieved": round(algo_bytes / (pipeline_ms * 1e-3) / 1e9, 1) if pipeline_ms else None,
    }
    traffic = pmc_traffic(dom, n, bins)
    if traffic:
        roofline["traffic"] = traffic["bytes"]
        roofline["traffic_source"] = traffic["source"]

    # full-size properties of the last timed step's result (every run): every row lands in
    # one cell (the synthetic columns hold no NaN, NaN rows would sit in cell 0), and the
    # grid's sum equals an independent reduction of w (a 0-d sum: the reduction kernel, not
    # the tile path) within 1e-6 relative
    count, total = res
    local_w = float(vaex_amd.from_arrays(w=w).sum("w"))
    ref_sum = vdist.allreduce_scalar(local_w, "sum") if dist is not None else local_w
    c_tot = int(np.asarray(count).sum())
    s_tot = float(np.asarray(total).sum())
    check = {"count_total": c_tot, "rows": n * world, "count_equal": c_tot == n * world,
             "sum_total": s_tot, "sum_reference": ref_sum,
             "sum_rel_err": abs(s_tot - ref_sum) / abs(ref_sum) if ref_sum else None}
    check["ok"] = bool(check["count_equal"] and check["sum_rel_err"] is not None and check["sum_rel_err"] < 1e-6)

    extra = {}
    if rank == 0 and world == 1:
        extra["zero_d"] = bench_zero_d(w, n, args)
    if rank == 0 and world == 1 and not args.no_layouts:
        extra["c2_sorted_y"] = bench_c2_layout(x, w, n, bins, args)
    if rank == 0 and world == 1 and not args.no_groupby:
        extra["groupby"] = bench_groupby(int(args.groupby_rows), args)
        if not args.no_layouts:
            extra["groupby_sorted_keys"] = bench_groupby(int(args.groupby_rows), args, layout="sorted")
    if rank == 0 and world == 1 and not args.no_count_only:
        extra["count_only"] = bench_count_only(x, y, n, bins, args)
    if rank == 0 and world == 1 and not args.no_f32:
        extra["c2_float32"] = bench_c2_float32(n, bins, args, check["sum_reference"])
    if rank == 0 and world == 1 and not args.no_filtered:
        extra["filtered"] = bench_filtered(x, y, w, n, bins, args)
    if rank == 0 and world == 1 and not args.no_aggs:
        extra["aggs"] = bench_other_aggs(x, y, w, n, bins, args, ms_per_step)
    if rank == 0 and world == 1 and not args.no_set:
        extra["ordered_set"] = bench_ordered_set(int(args.groupby_rows), args)
    if rank == 0 and world == 1 and args.host_rows > 0:
        extra["host_columns"] = bench_host_columns(x, y, w, int(min(args.host_rows, n)), bins)
    if rank == 0 and world == 1 and args.c4_rows > 0:
        extra["c4"] = bench_c4(int(args.c4_rows), bins)
    if rank == 0 and world == 1 and args.h2o_rows > 0:
        extra["h2o"] = bench_h2o(int(args.h2o_rows))
    if dist is not None:
        # the multi-GPU BASELINE configs through the RCCL path, every rank (C4: a streamed
        # 2-d mean + grid all-reduce; C3 / C5: hash-partition exchange, dense all-reduce, h2o)
        d = bench_dist(dist, rank, world, args)
        if rank == 0:
            extra["dist"] = d
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, oracle_grid = cpu_baseline(x, y, w, n, bins, args.cpu_seconds)
        # driver-box parity: the oracle's grid of the baseline sample against the GPU's grid
        # of the same rows, cell by cell (outside every timed region)
        check["prefix_oracle"] = {"c2": prefix_parity_c2(x, y, w, bins, *oracle_grid)}
        if not args.no_groupby:
            cpu["groupby"], check["prefix_oracle"]["c3"] = cpu_baseline_groupby()
        check["ok"] = bool(check["ok"] and all(v.get("ok") for v in check["prefix_oracle"].values()))
        extra["c1"] = bench_c1(args)

    if rank == 0:
        line = {
            "metric": BASELINE_METRIC,
            "value": value,
            "unit": "rows/s",
            "n_gpus": rccl_ranks if rccl_ranks is not None else world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: x,y ~ N(0,1), w ~ U[0,1) float64 generated in HBM (counter-based splitmix64)",
            "config": {
                "workload": "C2 (BASELINE configs[1]): count(binby=[x,y], limits=[[-4,4],[-4,4]], shape=1024)"
                            " + sum(w), one merged pass",
                "rows_per_gpu": n,
                "grid": [bins + 3, bins + 3],
                "parallelism": f"row-shard x{world}" + (" + RCCL grid all-reduce" if world > 1 else ""),
                "rccl_ranks": rccl_ranks,
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        line["check"] = check
        line.update(extra)
        print(json.dumps(line), flush=True)
    if dist is not None:
        vdist.shutdown()


PMC_FILE = os.path.join(ROOT, "profiles", "pmc_c2.json")
PMC_KERNEL = {"tile_scatter_f64": "k_tile_scatter_f64<2, 1, 3, double, false, double>", "tile_scatter": "k_tile_scatter<2, 1>",
              "tile_reduce": "k_tile_reduce<1>"}


def pmc_traffic(timer, n, bins):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC passes
    (profiles/pmc_c2.json, written by scripts/prof_summary.py from separate FETCH_SIZE and
    WRITE_SIZE passes of this same bench command): 2 x FETCH_SIZE (gfx950 reports half of
    a wide streaming read, MI355X_MICROARCH.md §HBM) + WRITE_SIZE, KiB -> bytes.  Only used
    when the profiled workload is the one being run."""
    try:
        with open(PMC_FILE) as f:
            pmc = json.load(f)
    except (OSError, ValueError):
        return None
    if pmc.get("rows") != n or pmc.get("bins") != bins or timer not in PMC_KERNEL:
        return None
    for name, k in pmc["kernels"].items():
        if PMC_KERNEL[timer] in name and k.get("fetch_bytes_x2") is not None and k.get("write_bytes") is not None:
            return {"bytes": int(k["fetch_bytes_x2"] + k["write_bytes"]),
                    "source": f"{os.path.relpath(PMC_FILE, ROOT)} ({pmc.get('source')}): 2*FETCH_SIZE + WRITE_SIZE"}
    return None


def bench_count_only(x, y, n, bins, args):
    """C2 count-only variant (SURVEY.md §8d target: >= 60 % of HBM peak at 16 B/row):
    count(binby=[x, y]) alone, same timing method as the headline line."""
    from vaex_amd import _lib, superagg

    def step():
        bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, bins)
        by = superagg.BinnerScalar_float64("y", -4.0, 4.0, bins)
        bx.set_data(x)
        by.set_data(y)
        grid = superagg.Grid([bx, by])
        count = superagg.AggCount_int64(grid)
        grid.bin([count])
        return count

    for _ in range(max(1, args.warmup)):
        step()
    _lib.synchronize()
    _lib.timing_reset()
    _lib.timing_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    _lib.synchronize()
    t = time.perf_counter() - t0
    _lib.timing_enable(False)
    per = {}
    for k in TILE_KERNELS + ["bin_fused_global", "bin_fused_lds"]:
        c, ms = _lib.timing_read(k)
        if c:
            per[k] = ms / c
    dom = max(per, key=per.get) if per else None
    pipe = sum(per.values())
    return {"rows": n, "ms_per_step": t / args.steps * 1e3, "rows_per_s": n * args.steps / t,
            "algorithmic_bytes_per_row": 16, "per_kernel_ms": {k: round(v, 4) for k, v in per.items()},
            "kernel": dom, "kernel_GBps": round(16 * n / (per[dom] * 1e-3) / 1e9, 1) if dom else None,
            "kernel_frac": round(16 * n / (per[dom] * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4) if dom else None,
            "pipeline_GBps": round(16 * n / (pipe * 1e-3) / 1e9, 1) if pipe else None,
            "pipeline_frac": round(16 * n / (pipe * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4) if pipe else None}


def bench_c2_float32(n, bins, args, sum_reference):
    """C2 on float32 copies of the x, y, w draws (vaex files often hold float32): count +
    sum(w) on the 1027^2 grid through the fast float32 pass A (k_tile_scatter_f64<2, 1, 3,
    float>), same timing method as the headline line; 12 B/row read.  Checks: every row
    counted, and the grid's sum within 1e-6 of the float64 column's sum (float32 rounding of
    U[0, 1) values is ~3e-8 relative)."""
    from vaex_amd import _lib, superagg
    from vaex_amd.device import DeviceArray
    # the same counter-based draws as x, y, w (seeds 2, 3, 4), each rounded to float32
    x4 = DeviceArray.random(n, "normal", seed=2, dtype="float32")
    y4 = DeviceArray.random(n, "normal", seed=3, dtype="float32")
    w4 = DeviceArray.random(n, "uniform", seed=4, dtype="float32")

    def step():
        bx = superagg.BinnerScalar_float32("x", -4.0, 4.0, bins)
        by = superagg.BinnerScalar_float32("y", -4.0, 4.0, bins)
        bx.set_data(x4)
        by.set_data(y4)
        grid = superagg.Grid([bx, by])
        count = superagg.AggCount_int64(grid)
        s = superagg.AggSum_float32(grid)
        s.set_data(w4, 0)
        grid.bin([count, s])
        return count, s

    for _ in range(max(1, args.warmup)):
        res = step()
    _lib.synchronize()
    _lib.timing_reset()
    _lib.timing_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    _lib.synchronize()
    t = time.perf_counter() - t0
    _lib.timing_enable(False)
    per = {}
    for k in TILE_KERNELS + ["tile_scatter_f32", "bin_fused_global", "bin_fused_lds"]:
        c, ms = _lib.timing_read(k)
        if c:
            per[k] = ms / c
    c_tot = int(np.asarray(res[0]).sum())
    s_tot = float(np.asarray(res[1]).sum())
    rel = abs(s_tot - sum_reference) / abs(sum_reference) if sum_reference else None
    dom = max(per, key=per.get) if per else None
    return {"rows": n, "ms_per_step": t / args.steps * 1e3, "rows_per_s": n * args.steps / t,
            "algorithmic_bytes_per_row": 12, "per_kernel_ms": {k: round(v, 4) for k, v in per.items()},
            "kernel": dom, "kernel_GBps": round(12 * n / (per[dom] * 1e-3) / 1e9, 1) if dom else None,
            "check": {"count_total": c_tot, "count_equal": c_tot == n, "sum_total": s_tot, "sum_rel_err_vs_f64": rel,
                      "ok": bool(c_tot == n and rel is not None and rel < 1e-6)}}


def bench_filtered(x, y, w, n, bins, args):
    """Selections and filters (one keep mask per chunk, shared by the aggregators; DESIGN
    §5.11).  c2_selection: C2's count + sum(w) with the selection w > 0.5 -- the mask
    evaluated by the expression kernel inside every step, then the row-masked fast pass A.
    groupby_filtered: C3's groupby(key).agg(sum) on df[df.v > 0] through the DataFrame API
    (dense route, row-masked ordinal pass A); the frame keeps its filter mask, as the
    reference keeps filter masks per block, so `first_ms` (a fresh filtered frame: the
    filter's evaluation included) is reported beside the steady-state `ms`.  Checks: the masked grid's
    count total equals the number of kept rows; the groups' count total equals the filtered
    frame's length."""
    import vaex_amd
    from vaex_amd import _lib, superagg
    from vaex_amd.device import DeviceArray
    out = {}
    dfc = vaex_amd.from_arrays(x=x, y=y, w=w)

    def c2_step():
        keep = dfc.evaluate("w > 0.5")
        bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, bins)
        by = superagg.BinnerScalar_float64("y", -4.0, 4.0, bins)
        bx.set_data(x)
        by.set_data(y)
        grid = superagg.Grid([bx, by])
        count = superagg.AggCount_int64(grid)
        s = superagg.AggSum_float64(grid)
        s.set_data(w, 0)
        count.set_data_mask(keep)
        s.set_data_mask(keep)
        grid.bin([count, s])
        return count, keep

    def timed(fn, names):
        for _ in range(max(1, args.warmup)):
            res = fn()
        _lib.synchronize()
        _lib.timing_reset()
        _lib.timing_enable(True)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            res = fn()
        _lib.synchronize()
        t = time.perf_counter() - t0
        _lib.timing_enable(False)
        per = {}
        for k in names:
            c, ms = _lib.timing_read(k)
            if c:
                per[k] = round(ms / c, 4)
        return res, t / args.steps, per

    (count, keep), t, per = timed(c2_step, ["expr", "tile_sample", "tile_scatter_f64", "tile_scatter", "tile_reduce"])
    kept = int(np.count_nonzero(keep.to_numpy()))
    c_tot = int(np.asarray(count).sum())
    out["c2_selection"] = {"rows": n, "selection": "w > 0.5", "ms_per_step": t * 1e3, "rows_per_s": n / t,
                           "per_kernel_ms": per, "check": {"count_total": c_tot, "kept_rows": kept, "ok": c_tot == kept}}
    del count, keep
    m = int(args.groupby_rows)
    keys = DeviceArray.random(m, "randint", seed=5, a=5, b=5 + 1_000_000, dtype="int32")
    v = DeviceArray.random(m, "normal", seed=6)
    base = vaex_amd.from_arrays(key=keys, v=v)
    _lib.synchronize()
    t0 = time.perf_counter()
    dff = base[base.v > 0]
    dff.groupby("key", agg={"v": ["sum", "count"]})
    _lib.synchronize()
    first_ms = (time.perf_counter() - t0) * 1e3
    res, t, per = timed(lambda: dff.groupby("key", agg={"v": ["sum", "count"]}),
                        ["expr", "tile_sample", "tile_scatter_ord", "tile_scatter", "tile_reduce"])
    g_tot = int(np.asarray(res["v"].to_numpy()).sum())
    flen = len(dff)
    out["groupby_filtered"] = {"rows": m, "filter": "v > 0", "ms": t * 1e3, "first_ms": first_ms, "rows_per_s": m / t,
                               "groups": len(res),
                               "per_kernel_ms": per, "check": {"count_total": g_tot, "filtered_rows": flen,
                                                                "ok": g_tot == flen and len(res) > 0}}
    return out


def bench_other_aggs(x, y, w, n, bins, args, c2_ms):
    """Other aggregators on the C2 grid (1027^2 cells, 1e9 rows resident), end to end with the
    grids read back, median of the steps:
      first -- first(w, order=o, binby=[x, y]) (AggFirst, superagg.cpp:436-511) with a fourth
               column o ~ U[0, 1): the tile-partitioned engine (first.hip); algorithmic bytes
               32 per row (x, y, w, o);
      var   -- var(w, binby=[x, y]) (agg.py:191-229: AggSumMoment(2) + sum + count of w in
               one tile pass); 24 B per row.
    ratio_to_c2 = ms / the headline count+sum step."""
    import vaex_amd
    from vaex_amd import _lib
    from vaex_amd.device import DeviceArray
    o = DeviceArray.random(n, "uniform", seed=9)
    df = vaex_amd.from_arrays(x=x, y=y, w=w, o=o)
    lim = [[-4.0, 4.0], [-4.0, 4.0]]
    out = {}
    legs = (("first", lambda: df.first("w", "o", binby=["x", "y"], limits=lim, shape=bins), 32,
             ["first_sample", "first_scatter", "first_reduce", "bin_indices", "bin_aggregate"]),
            ("var", lambda: df.var("w", binby=["x", "y"], limits=lim, shape=bins), 24,
             TILE_KERNELS + ["bin_indices", "bin_aggregate"]))
    for name, f, bpr, kernels in legs:
        r = f()
        _lib.synchronize()
        ts = []
        _lib.timing_reset()
        _lib.timing_enable(True)
        for _ in range(max(3, args.steps // 2)):
            t0 = time.perf_counter()
            r = f()
            ts.append(time.perf_counter() - t0)
        _lib.synchronize()
        _lib.timing_enable(False)
        per = {}
        for k in kernels:
            c, ms = _lib.timing_read(k)
            if c:
                per[k] = ms / c
        t = float(np.median(ts))
        dom = max(per, key=per.get) if per else None
        out[name] = {"ms": round(t * 1e3, 3), "rows_per_s": n / t, "ratio_to_c2": round(t * 1e3 / c2_ms, 3),
                     "algorithmic_bytes_per_row": bpr, "per_kernel_ms": {k: round(v, 4) for k, v in per.items()},
                     "kernel": dom,
                     "kernel_frac": round(bpr * n / (per[dom] * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4) if dom else None,
                     "finite_cells": int(np.isfinite(np.asarray(r)).sum())}
    c = df.count(binby=["x", "y"], limits=lim, shape=bins)
    out["var"]["cells_with_rows"] = int((np.asarray(c) > 0).sum())
    del df, o
    return out


def bench_ordered_set(n, args):
    """ordered_set_int32.update over the C3 keys (1e9 int32 rows, 1e6 distinct; random and
    sorted layouts): the standalone set build of df._set / Grouper (hash_primitives.hpp:96-281),
    median of 3, with the set kernels' HIP-event times; algorithmic bytes 4 per row."""
    from vaex_amd import _lib, superutils
    from vaex_amd.device import DeviceArray
    out = {"rows": n, "algorithmic_bytes_per_row": 4}
    names = ["set_sample", "set_insert", "set_reduce", "set_rank", "set_direct"]
    for layout in ("random", "sorted"):
        if layout == "sorted":
            keys = DeviceArray.random(n, "sorted_int", a=5, b=5 + 1_000_000, dtype="int32")
        else:
            keys = DeviceArray.random(n, "randint", seed=5, a=5, b=5 + 1_000_000, dtype="int32")
        s = superutils.ordered_set_int32()
        s.update(keys)
        _lib.synchronize()
        ts = []
        _lib.timing_reset()
        _lib.timing_enable(True)
        for _ in range(3):
            s = superutils.ordered_set_int32()
            t0 = time.perf_counter()
            s.update(keys)
            m = len(s)
            ts.append(time.perf_counter() - t0)
        _lib.timing_enable(False)
        per = {}
        for k in names:
            c, ms = _lib.timing_read(k)
            if c:
                per[k] = round(ms / 3, 4)
        t = float(np.median(ts))
        out[layout] = {"ms": round(t * 1e3, 3), "rows_per_s": n / t, "keys": m, "keys_ok": m == 1_000_000,
                       "per_kernel_ms": per}
        del keys, s
    return out


def bench_zero_d(w, n, args):
    """0-d aggregations (no binby; agg.hpp:76-105 with no binners): df.sum('w'),
    df.mean('w') (sum + non-NaN count of w in one pass) and df.count() on the resident w
    column, end to end (median of steps), with the reduction kernel's HIP-event time against
    8 B/row (count(*) reads nothing: the count is the row count)."""
    import vaex_amd
    from vaex_amd import _lib
    df = vaex_amd.from_arrays(w=w)
    out = {"rows": n, "algorithmic_bytes_per_row": 8}
    for name, f in (("sum", lambda: df.sum("w")), ("mean", lambda: df.mean("w")), ("count", lambda: df.count())):
        f()
        _lib.synchronize()
        ts = []
        _lib.timing_reset()
        _lib.timing_enable(True)
        for _ in range(max(3, args.steps)):
            t0 = time.perf_counter()
            r = f()
            ts.append(time.perf_counter() - t0)
        _lib.synchronize()
        _lib.timing_enable(False)
        c, ms = _lib.timing_read("bin_reduce0")
        k_ms = ms / c if c else None
        t = float(np.median(ts))
        out[name] = {"ms": round(t * 1e3, 4), "rows_per_s": n / t, "value": float(r),
                     "kernel_ms": round(k_ms, 4) if k_ms else None}
        if name != "count" and k_ms:
            out[name]["kernel_GBps"] = round(8 * n / (k_ms * 1e-3) / 1e9, 1)
            out[name]["kernel_frac"] = round(8 * n / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
    out["count_equal"] = int(out["count"]["value"]) == n
    return out


def bench_host_columns(x, y, w, m, bins):
    """PCIe-inclusive rate: the same count+sum query on host (numpy) columns, which the
    library streams through its double-buffered pinned H2D pipeline (16 Mi-row chunks)."""
    from vaex_amd import _lib, superagg
    hx, hy, hw = x[:m].to_numpy(), y[:m].to_numpy(), w[:m].to_numpy()

    def run():
        bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, bins)
        by = superagg.BinnerScalar_float64("y", -4.0, 4.0, bins)
        bx.set_data(hx)
        by.set_data(hy)
        grid = superagg.Grid([bx, by])
        count = superagg.AggCount_int64(grid)
        total = superagg.AggSum_float64(grid)
        total.set_data(hw, 0)
        grid.bin([count, total])
        return count

    run()
    _lib.synchronize()
    times = []
    for _ in range(2):
        t0 = time.perf_counter()
        c = run()
        _lib.synchronize()
        times.append(time.perf_counter() - t0)
    t = min(times)
    ok = int(np.asarray(c).sum()) == m
    return {"rows": m, "seconds": t, "rows_per_s": m / t, "host_GBps": 24 * m / t / 1e9, "count_equal": ok}


def h2d_peak(nbytes=1 << 30, reps=4):
    """Host -> HBM copy rate of this box, the C4 leg's roofline: hipHostMalloc'd sources
    copied to one HBM block as one 1 GiB copy, and as 4 back-to-back 256 MiB copies on 1, 2
    and 4 streams (best of `reps` each); `pinned_GBps` is the best of those.  Measured with
    the HIP runtime directly (ctypes), outside the library under test."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(vp), sz, ctypes.c_uint]
    hip.hipMalloc.argtypes = [ctypes.POINTER(vp), sz]
    hip.hipMemcpyAsync.argtypes = [vp, vp, sz, ctypes.c_int, vp]
    hip.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
    hip.hipStreamSynchronize.argtypes = [vp]
    hip.hipFree.argtypes = [vp]
    hip.hipHostFree.argtypes = [vp]
    hip.hipStreamDestroy.argtypes = [vp]
    src, dst = vp(), vp()
    if hip.hipHostMalloc(ctypes.byref(src), nbytes, 0) or hip.hipMalloc(ctypes.byref(dst), nbytes):
        return {"error": "allocation failed"}
    ctypes.memset(src, 1, nbytes)
    streams = [vp() for _ in range(4)]
    for st in streams:
        hip.hipStreamCreateWithFlags(ctypes.byref(st), 1)
    out = {}
    try:
        for name, pieces, ns in (("1x1GiB", 1, 1), ("4x256MiB_1stream", 4, 1), ("4x256MiB_2streams", 4, 2),
                                 ("4x256MiB_4streams", 4, 4)):
            part = nbytes // pieces
            best = float("inf")
            for _ in range(reps):
                t0 = time.perf_counter()
                for i in range(pieces):
                    hip.hipMemcpyAsync(vp(dst.value + i * part), vp(src.value + i * part), part, 1, streams[i % ns])
                for st in streams[:ns]:
                    hip.hipStreamSynchronize(st)
                best = min(best, time.perf_counter() - t0)
            out[name] = round(nbytes / best / 1e9, 2)
    finally:
        for st in streams:
            hip.hipStreamDestroy(st)
        hip.hipFree(dst)
        hip.hipHostFree(src)
    out["pinned_GBps"] = max(out.values())
    return out


def bench_c4(rows, bins, repeats=2):
    """C4's query on one GPU (BASELINE configs[3] per rank): mean(w, binby=[x, y], shape=1024)
    over x, y, w float64 columns of `rows` rows in a vaex HDF5 file written by export_hdf5 and
    opened with vaex_amd.open (memory-mapped; page cache warm), so every row crosses the host
    link through the library's double-buffered pipeline.  Roofline: the box's measured pinned
    host -> HBM rate.  Host-pipeline modes: 'bounce' (host threads copy each chunk into a
    pinned bounce buffer, DMA from there), 'register_per_chunk' (each chunk's pages are
    registered for its copy), 'pageable' (the runtime's pageable copy path) and
    'registered_mapping' (the default: the file mapping is registered once, on first use,
    and every chunk is DMA'd in place)."""
    import shutil
    import tempfile
    import vaex_amd
    from vaex_amd.device import DeviceArray
    nbytes = 24 * rows
    out = {"rows": rows, "bytes": nbytes, "algorithmic_bytes_per_row": 24}
    try:
        with open("/proc/meminfo") as f:
            avail = {l.split(":")[0]: int(l.split()[1]) * 1024 for l in f}.get("MemAvailable", 0)
    except OSError:
        avail = 0
    cands = [d for d in ("/dev/shm", tempfile.gettempdir()) if os.path.isdir(d)]
    where = next((d for d in cands if shutil.disk_usage(d).free > 1.15 * nbytes), None)
    if where is None or avail < 2.2 * nbytes:
        out["skipped"] = f"needs {2.2 * nbytes / 1e9:.0f} GB host memory and {1.15 * nbytes / 1e9:.0f} GB of file space"
        return out
    out["h2d"] = h2d_peak()
    path = os.path.join(where, f"vaex_amd_c4_{os.getpid()}.hdf5")
    try:
        t0 = time.perf_counter()
        cols = {"x": DeviceArray.random(rows, "normal", seed=12), "y": DeviceArray.random(rows, "normal", seed=13),
                "w": DeviceArray.random(rows, "uniform", seed=14)}
        vaex_amd.from_arrays(**cols).export_hdf5(path)
        del cols
        out["write_seconds"] = round(time.perf_counter() - t0, 2)
        out["file_dir"] = where
        df = vaex_amd.open(path)
        lim = [[-4.0, 4.0], [-4.0, 4.0]]
        modes = (("bounce", "0", "0"), ("register_per_chunk", "0", "1"), ("pageable", "0", "2"),
                 ("registered_mapping", "1", "0"))
        for mode, reg, pipe in modes:
            os.environ["VH_HOST_REGISTER"], os.environ["VH_HOST_PIPE"] = reg, pipe
            t0 = time.perf_counter()
            df.mean("w", binby=["x", "y"], limits=lim, shape=bins)  # warm (page cache, pinned buffers)
            first = time.perf_counter() - t0
            ts = []
            for _ in range(repeats):
                t0 = time.perf_counter()
                m = df.mean("w", binby=["x", "y"], limits=lim, shape=bins)
                ts.append(time.perf_counter() - t0)
            t = float(np.median(ts))
            gbps = nbytes / t / 1e9
            out[mode] = {"seconds": round(t, 4), "first_call_seconds": round(first, 4), "rows_per_s": rows / t,
                         "host_GBps": round(gbps, 2), "frac_of_pinned_h2d": round(gbps / out["h2d"]["pinned_GBps"], 3),
                         "finite_cells": int(np.isfinite(m).sum())}
        os.environ.pop("VH_HOST_REGISTER", None)
        os.environ.pop("VH_HOST_PIPE", None)
        c = df.count(binby=["x", "y"], limits=lim, shape=bins, edges=True)
        out["count_equal"] = int(np.asarray(c).sum()) == rows
        best = max((m[0] for m in modes), key=lambda k: out[k]["host_GBps"])
        out["best_mode"] = best
        out["frac_of_pinned_h2d"] = out[best]["frac_of_pinned_h2d"]
    finally:
        os.environ.pop("VH_HOST_REGISTER", None)
        os.environ.pop("VH_HOST_PIPE", None)
        df = None
        if os.path.exists(path):
            os.remove(path)
    return out


def bench_c2_layout(x, w, n, bins, args):
    """Row-order robustness: the headline C2 query (count + sum(w), 1027^2 grid) with y sorted
    (ascending normal quantiles, x random), timed like the headline step, and the tile path's
    overflow rows (pass-A rows that missed their region; global atomics)."""
    from vaex_amd import _lib, superagg
    from vaex_amd.device import DeviceArray
    ys = DeviceArray.random(n, "sorted_normal", a=0.0, b=1.0)

    def step():
        bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, bins)
        by = superagg.BinnerScalar_float64("y", -4.0, 4.0, bins)
        bx.set_data(x)
        by.set_data(ys)
        grid = superagg.Grid([bx, by])
        count = superagg.AggCount_int64(grid)
        total = superagg.AggSum_float64(grid)
        total.set_data(w, 0)
        grid.bin([count, total])
        return np.asarray(count), np.asarray(total)

    for _ in range(max(1, args.warmup)):
        step()
    _lib.synchronize()
    _lib.stat_read("tile_overflow_rows", reset=True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        c, _s = step()
    _lib.synchronize()
    t = (time.perf_counter() - t0) / args.steps
    over = _lib.stat_read("tile_overflow_rows", reset=True) / max(1, args.steps)
    del ys
    return {"layout": "y sorted (ascending normal quantiles), x random", "rows": n, "ms_per_step": t * 1e3,
            "rows_per_s": n / t, "overflow_rows_per_step": over, "count_equal": int(c.sum()) == n}


def bench_groupby(n, args, layout="random"):
    """C3: groupby(int32 key, 1e6 distinct).agg({v: [sum, count]}) on resident columns, end to
    end (every pass, result read-back into host numpy columns), best of 3:
      auto  -- what DataFrame.groupby picks for this dense key range: one min/max pass, then
               the BinnerOrdinal grid through the tile path (fast ordinal pass A);
      fused -- the one-pass hash-partitioned aggregation (hashagg.hip) the frame takes for
               sparse int keys, run on the same columns through its API;
      hash  -- assume_sparse=True: the ordered_set grouper's result (groups in the order their
               keys first appear): for this dense key range the grid route + vh_dense_first_order
               (a run-head prefix scan for each group's first row, a radix sort of the groups);
      hash_minmax -- the same with min + max + sum + count(*) of v (one carried value slot).
    Per-kernel milliseconds from HIP events on the library stream."""
    from vaex_amd import _lib
    from vaex_amd.device import DeviceArray
    from vaex_amd.hashagg import HashAgg
    import vaex_amd
    if layout == "sorted":  # every key's rows consecutive, keys ascending
        keys = DeviceArray.random(n, "sorted_int", a=5, b=5 + 1_000_000, dtype="int32")
    else:
        keys = DeviceArray.random(n, "randint", seed=5, a=5, b=5 + 1_000_000, dtype="int32")
    v = DeviceArray.random(n, "normal", seed=6)
    df = vaex_amd.from_arrays(key=keys, v=v)
    out = {"rows": n, "algorithmic_bytes_per_row": 12, "layout": layout}
    names = ["minmax", "tile_sample", "tile_scatter", "tile_scatter_ord", "tile_scatter_set", "tile_reduce", "ha_sample",
             "ha_scatter", "ha_scatter_f64", "ha_reduce", "ha_finish", "ha_first", "dense_first", "set_sample", "set_insert",
             "set_reduce", "set_rank", "bin_fused_global"]

    def run(mode):
        if mode == "fused":
            ha = HashAgg(keys.dtype, [v.dtype], [False])
            ha.update(keys, [v])
            k, c, s, _ = ha.finish()
            return k, c, s[0]
        if mode == "hash_minmax":  # assume_sparse=True with min + max + sum (+ count(*))
            dfg = df.groupby("key", agg={"v": ["sum", "count", "min", "max"]}, assume_sparse=True)
            return dfg["key"].to_numpy(), dfg["v"].to_numpy(), dfg["v_sum"].to_numpy()
        dfg = df.groupby("key", agg={"v": ["sum", "count"]}, assume_sparse="auto" if mode == "auto" else True)
        # {"v": ["sum", "count"]} names the count(*) column "v" (groupby.py:345-402)
        return dfg["key"].to_numpy(), dfg["v"].to_numpy(), dfg["v_sum"].to_numpy()

    v_total = float(vaex_amd.from_arrays(v=v).sum("v"))  # independent 0-d reduction
    ref_groups = None
    for mode in ("auto", "fused", "hash", "hash_minmax"):
        run(mode)  # warm-up
        _lib.trace_report()
        _lib.synchronize()
        times = []
        prof = None
        if os.environ.get("BENCH_PROFILE_GROUPBY"):
            import cProfile
            prof = cProfile.Profile()
        for name in ("tile_overflow_rows", "hashagg_overflow_rows", "set_overflow_rows"):
            _lib.stat_read(name, reset=True)
        for _ in range(max(1, min(3, args.steps))):
            _lib.timing_reset()
            _lib.timing_enable(True)
            if prof:
                prof.enable()
            t0 = time.perf_counter()
            res = run(mode)
            _lib.synchronize()
            times.append(time.perf_counter() - t0)
            if prof:
                prof.disable()
            _lib.timing_enable(False)
        if prof:
            import pstats
            print("groupby mode", mode, [round(x * 1e3, 2) for x in times], file=sys.stderr)
            print({k: (c, round(t * 1e3, 2)) for k, (c, t) in _lib.trace_report().items()}, file=sys.stderr)
            pstats.Stats(prof, stream=sys.stderr).sort_stats("tottime").print_stats(12)
        t = min(times)
        per = {}
        for k in names:
            c, ms = _lib.timing_read(k)
            if c:
                per[k] = round(ms, 3)
        # outside the timed region: full-size properties of the last result -- every row
        # counted once, the sum total against an independent reduction, routes agree
        gk, gc, gs = (np.asarray(a) for a in res)
        order = np.argsort(gk, kind="stable")
        check = {"count_total": int(gc.sum()), "count_equal": int(gc.sum()) == n,
                 "sum_rel_err": abs(float(gs.sum(dtype=np.float64)) - v_total) / abs(v_total)}
        if ref_groups is None:
            ref_groups = (gk[order], gc[order])
        else:
            check["same_groups_as_auto"] = bool(np.array_equal(gk[order], ref_groups[0])
                                                and np.array_equal(gc[order], ref_groups[1]))
        check["ok"] = check["count_equal"] and check["sum_rel_err"] < 1e-6 and check.get("same_groups_as_auto", True)
        groups = len(gk)
        over = {name: _lib.stat_read(name, reset=True) for name in ("tile_overflow_rows", "hashagg_overflow_rows",
                                                                     "set_overflow_rows")}
        out[mode] = {"groups": groups, "check": check, "seconds": t, "rows_per_s": n / t, "algorithmic_GBps": 12 * n / t / 1e9,
                     "kernel_ms_last": per, "overflow_rows": {k: v for k, v in over.items() if v}}
    del keys, v, df
    return out


H2O_BYTES = {"q1": 2, "q2": 2, "q3": 9, "q4": 6, "q5": 9, "q7": 5, "q10": 10}


def h2o_frame(n, seed0=0, executor=None):
    """benchmarks/fixtures.py:38-70's columns for G1_1e9_1e2 (i1_100 int8 in [5, 105), i4_1M
    int32 in [5, 1e6 + 5), i1_10 int8 in [5, 15), x4 float32 normal), generated in HBM
    (counter-based; seeds offset per rank), with benchmarks/groupbyh2o.py:26-36's aliases
    (id1 / id2 / id4 / id5 = i1_100, id3 / id6 = i4_1M, v1 / v2 = i1_10, v3 = x4)."""
    from vaex_amd.dataframe import DataFrame
    from vaex_amd.device import DeviceArray
    cols = {"i1_100": DeviceArray.random(n, "randint", seed=seed0 + 21, a=5, b=105, dtype="int8"),
            "i4_1M": DeviceArray.random(n, "randint", seed=seed0 + 22, a=5, b=1_000_005, dtype="int32"),
            "i1_10": DeviceArray.random(n, "randint", seed=seed0 + 23, a=5, b=15, dtype="int8"),
            "x4": DeviceArray.random(n, "normal", seed=seed0 + 24, dtype="float32")}
    df = DataFrame(cols, executor=executor)
    for a, b in [("id1", "i1_100"), ("id2", "i1_100"), ("id3", "i4_1M"), ("id4", "i1_100"), ("id5", "i1_100"),
                 ("id6", "i4_1M"), ("v1", "i1_10"), ("v2", "i1_10"), ("v3", "x4")]:
        df.columns[a] = df.columns[b]
    return df


def h2o_queries(df):
    """benchmarks/groupbyh2o.py:39-93 exactly as written there."""
    return {
        "q1": lambda: df.groupby(["id1"]).agg({"v1": "sum"}),
        "q2": lambda: df.groupby(["id1", "id2"]).agg({"v1": "sum"}),
        "q3": lambda: df.groupby(["id3"]).agg({"v1": "sum", "v3": "mean"}),
        "q4": lambda: df.groupby(["id4"]).agg({"v1": "mean", "v2": "mean", "v3": "mean"}),
        "q5": lambda: df.groupby(["id6"]).agg({"v1": "sum", "v2": "sum", "v3": "sum"}),
        "q7": lambda: df.groupby(["id3"]).agg({"v1": "max", "v2": "min"}),
        "q10": lambda: df.groupby(["id1", "id2", "id3", "id4", "id5", "id6"]).agg({"v3": "sum", "v1": "count"}),
    }


def h2o_check(q, r, n, sums):
    """Size-independent properties of one h2o result: the group count the columns imply
    (id1 = id2 = id4 = id5 and id3 = id6 alias one column each), a count total equal to the
    rows (q10), the v1 sum total equal to an independent 0-d sum of i1_10 (q1, q3, q5)."""
    groups = len(r)
    exp = {"q1": 100, "q2": 100, "q4": 100}.get(q)
    out = {"groups": groups}
    ok = True
    if exp is not None:
        out["groups_expected"] = exp
        ok = groups == exp
    else:
        ok = groups > 0
    if q == "q10":
        c = int(np.asarray(r["v1"].to_numpy()).sum())
        out["count_total"] = c
        ok = ok and c == n
    if q in ("q1", "q3", "q5"):
        s = int(np.asarray(r["v1"].to_numpy()).astype(np.int64).sum())
        out["v1_sum_total"] = s
        ok = ok and s == sums["v1"]
    out["ok"] = bool(ok)
    return out


def bench_h2o(n, reps=3):
    """C5's queries on one GPU (BASELINE configs[4] per rank): h2o groupby G1 at n rows,
    q1-q5, q7, q10 of benchmarks/groupbyh2o.py on HBM columns, end to end (result DataFrame
    on the host), best of `reps` after a warm-up (q10: best of two); algorithmic bytes per
    row = the distinct columns a query reads."""
    from vaex_amd import _lib
    # the leg starts from empty block caches, as a fresh process would: the earlier legs'
    # cached page-locked blocks (C4's bounce buffers, grids) would otherwise hold the cache's
    # cap and q10's multi-GB result columns would be hipHostMalloc'd for every query
    _lib.synchronize()
    _lib.trim_caches()
    df = h2o_frame(n)
    sums = {"v1": int(df.sum("i1_10"))}
    out = {"rows": n, "data": "fixtures.py schema generated in HBM (int8 / int32 / float32)"}
    for q, f in h2o_queries(df).items():
        f()
        _lib.synchronize()
        ts = []
        r = None
        for _ in range(2 if q == "q10" else reps):
            # the previous result is dropped first, as a query loop that discards its results
            # does (its page-locked result columns go back to the block cache)
            r = None
            if os.environ.get("BENCH_H2O_TRACE"):
                _lib.trace_report()
            t0 = time.perf_counter()
            r = f()
            _lib.synchronize()
            ts.append(time.perf_counter() - t0)
            if os.environ.get("BENCH_H2O_TRACE"):  # per-call C-ABI times (VAEX_AMD_TRACE_CALLS=1)
                top = sorted(_lib.trace_report().items(), key=lambda kv: -kv[1][1])[:5]
                print(f"# h2o {q}: {ts[-1] * 1e3:.1f} ms " + " ".join(f"{k} {1e3 * v[1]:.1f}" for k, v in top),
                      file=sys.stderr, flush=True)
        t = min(ts)
        out[q] = {"ms": round(t * 1e3, 3), "rows_per_s": n / t, "algorithmic_bytes_per_row": H2O_BYTES[q],
                  "GBps": round(H2O_BYTES[q] * n / t / 1e9, 1), "check": h2o_check(q, r, n, sums)}
    del df
    return out


def bench_dist(dist, rank, world, args, repeats=3):
    """The multi-GPU BASELINE configs through the RCCL communicator (every rank runs this;
    times are the max over ranks of the slowest rank, bracketed by barriers):
      groupby_hash -- C3 / C5 shape: each rank its own 1e9-row shard (int32 key, 1e6 distinct,
                      float64 value), the fused hash aggregation, then the hash-partition
                      all-to-all of the groups (vh_hashagg_exchange: every group to owner
                      splitmix64(key) % world, folded there), results left sharded by owner;
      groupby_dense -- the same shards through DataFrame.groupby on ExecutorDistributed
                      (dense key range: BinnerOrdinal grid per rank + RCCL grid all-reduce);
      c4           -- mean(w, binby=[x, y], shape=1024) over one memory-mapped HDF5 file
                      written by rank 0, rows sharded by range across the ranks, grid
                      all-reduce (execution.py:214-289's fan-out at process granularity);
      h2o          -- q1-q5, q7 on per-rank shards through ExecutorDistributed.
    Checks: world-wide count totals and group counts against the rows generated."""
    import shutil
    import tempfile
    import vaex_amd
    from vaex_amd import _lib
    from vaex_amd import distributed as vdist
    from vaex_amd.dataframe import DataFrame
    from vaex_amd.device import DeviceArray
    from vaex_amd.hashagg import HashAgg
    out = {"world": world, "rccl": bool(getattr(dist, "device", False))}

    def timed(f):
        ts = []
        r = None
        for _ in range(repeats):
            vdist.barrier(dist)
            _lib.synchronize()
            t0 = time.perf_counter()
            r = f()
            _lib.synchronize()
            vdist.barrier(dist)
            ts.append(vdist.allreduce_scalar(time.perf_counter() - t0, "max", dist))
        return r, min(ts)

    ng = int(args.dist_groupby_rows)
    keys = DeviceArray.random(ng, "randint", seed=5 + 1000 * rank, a=5, b=5 + 1_000_000, dtype="int32")
    v = DeviceArray.random(ng, "normal", seed=6 + 1000 * rank)

    def hash_exchange():
        ha = HashAgg(keys.dtype, [v.dtype], [False])
        ha.update(keys, [v])
        return ha.finish(dist, gather=False)

    hash_exchange()
    (k, c, s, _), t = timed(hash_exchange)
    groups = int(dist.allreduce(np.array([len(k)], np.int64))[0])
    total = int(dist.allreduce(np.array([int(np.asarray(c).sum())], np.int64))[0])
    out["groupby_hash"] = {"rows_per_rank": ng, "ms": round(t * 1e3, 3), "rows_per_s": ng * world / t,
                           "groups": groups, "count_total": total,
                           "ok": bool(total == ng * world and groups == 1_000_000)}
    ddf = DataFrame({"key": keys, "v": v}, executor=vdist.ExecutorDistributed(dist, shard_rows=False))

    def dense():
        return ddf.groupby("key", agg={"v": ["sum", "count"]}, sort=True)
    dense()
    g, t = timed(dense)
    total = int(np.asarray(g["v"].to_numpy()).sum())
    out["groupby_dense"] = {"rows_per_rank": ng, "ms": round(t * 1e3, 3), "rows_per_s": ng * world / t,
                            "groups": len(g), "count_total": total,
                            "ok": bool(total == ng * world and len(g) == 1_000_000)}
    del ddf, keys, v, g

    if args.dist_h2o_rows > 0:
        nh = int(args.dist_h2o_rows)
        hdf = h2o_frame(nh, seed0=1000 * rank, executor=vdist.ExecutorDistributed(dist, shard_rows=False))
        v1 = int(vdist.allreduce_scalar(float(vaex_amd.from_arrays(v=hdf.columns["i1_10"]).sum("v")), "sum", dist))
        res = {"rows_per_rank": nh}
        for q, f in h2o_queries(hdf).items():
            if q == "q10":
                continue  # the combined-key recursion is single-process
            f()
            r, t = timed(f)
            res[q] = {"ms": round(t * 1e3, 3), "rows_per_s": nh * world / t,
                      "check": h2o_check(q, r, nh * world, {"v1": v1})}
        out["h2o"] = res
        del hdf

    rows = int(args.c4_rows)
    if rows > 0:
        nbytes = 24 * rows
        where = None
        if rank == 0:
            cands = [d for d in ("/dev/shm", tempfile.gettempdir()) if os.path.isdir(d)]
            where = next((d for d in cands if shutil.disk_usage(d).free > 1.15 * nbytes), None)
        where = dist.bcast(where) if hasattr(dist, "bcast") else where
        if where is None:
            out["c4"] = {"skipped": f"needs {1.15 * nbytes / 1e9:.0f} GB of file space"}
            return out
        path = os.path.join(where, f"vaex_amd_c4_dist_{os.environ.get('MASTER_PORT', 'x')}.hdf5")
        try:
            if rank == 0:
                cols = {"x": DeviceArray.random(rows, "normal", seed=12), "y": DeviceArray.random(rows, "normal", seed=13),
                        "w": DeviceArray.random(rows, "uniform", seed=14)}
                vaex_amd.from_arrays(**cols).export_hdf5(path)
                del cols
            vdist.barrier(dist)
            src = vaex_amd.open(path)
            cdf = DataFrame(dict(src.columns), executor=vdist.ExecutorDistributed(dist, shard_rows=True))
            lim = [[-4.0, 4.0], [-4.0, 4.0]]
            cdf.mean("w", binby=["x", "y"], limits=lim, shape=args.bins)
            m, t = timed(lambda: cdf.mean("w", binby=["x", "y"], limits=lim, shape=args.bins))
            cnt = cdf.count(binby=["x", "y"], limits=lim, shape=args.bins, edges=True)
            out["c4"] = {"rows": rows, "ms": round(t * 1e3, 3), "rows_per_s": rows / t,
                         "host_GBps_total": round(nbytes / t / 1e9, 2), "finite_cells": int(np.isfinite(m).sum()),
                         "count_total": int(np.asarray(cnt).sum()), "ok": bool(int(np.asarray(cnt).sum()) == rows)}
            del cdf, src
        finally:
            vdist.barrier(dist)
            if rank == 0 and os.path.exists(path):
                os.remove(path)
    return out


def cpu_baseline(x, y, w, n, bins, target_seconds, repeats=5):
    """oracle/superagg_oracle.c or_bench_grid2d: reference threading model (1 Mi-row chunks,
    max(2, T//8) private grids for a >=1e7-byte part, serial reduce) on a bounded sample;
    the median of `repeats` runs."""
    from oracle import oracle
    L = oracle.lib()
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    nparts = max(2, threads // 8)  # cpu.py:487-499 for a 16.9 MB count+sum part
    cells = (bins + 3) ** 2
    cnt = np.zeros(cells, np.int64)
    sm = np.zeros(cells, np.float64)

    host = {}

    def run_parts(m, parts):
        if host.get("m") != m:
            host.update(m=m, x=x[:m].to_numpy(), y=y[:m].to_numpy(), w=w[:m].to_numpy())
        hx, hy, hw = host["x"], host["y"], host["w"]
        t0 = time.perf_counter()
        used = L.or_bench_grid2d(hx.ctypes.data, hy.ctypes.data, hw.ctypes.data, m, -4.0, 4.0, -4.0, 4.0, bins,
                                 parts, threads, 1 << 20, cnt.ctypes.data, sm.ctypes.data)
        return time.perf_counter() - t0, used

    probe = min(n, 1 << 24)
    t, _ = run_parts(probe, nparts)
    m = int(min(n, 1 << 28, max(probe, probe * (target_seconds / repeats) / max(t, 1e-6))))
    runs = [run_parts(m, nparts) for _ in range(repeats)]
    t = float(np.median([r[0] for r in runs]))
    used = runs[0][1]
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    # the same sample without the ideal_splits cap (one private grid per thread)
    unc = [run_parts(m, threads) for _ in range(repeats)]
    t_unc = float(np.median([r[0] for r in unc]))
    grid = (m, cnt.copy(), sm.copy())  # the oracle's grid of the sample (parity check)
    return {"value": m / t, "unit": "rows/s", "cores": used, "kind": "port",
            "uncapped": {"value": m / t_unc, "cores": unc[0][1], "nparts": threads},
            "sample": f"first {m} rows of the same x,y,w columns, count+sum 1027x1027 grid, median of {repeats} "
                      f"runs ({t:.2f} s each)",
            "runs_s": [round(r[0], 4) for r in runs],
            "threads_available": threads, "nparts_rule": "max(2, T//8) (cpu.py:487-499)",
            "cpu_model": cpu_model, "host": platform.node()}, grid


def prefix_parity_c2(x, y, w, bins, m, cnt, sm):
    """The GPU's count + sum grid of the first m rows (the CPU baseline's sample) against the
    oracle's grid of the same rows (or_bench_grid2d: superagg_binners.cpp:14-56 binning,
    superagg.cpp:155-192,349-389 aggregation): counts exact, sums rtol 1e-6."""
    from vaex_amd import superagg
    bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, bins)
    by = superagg.BinnerScalar_float64("y", -4.0, 4.0, bins)
    bx.set_data(x[:m])
    by.set_data(y[:m])
    grid = superagg.Grid([bx, by])
    count = superagg.AggCount_int64(grid)
    total = superagg.AggSum_float64(grid)
    total.set_data(w[:m], 0)
    grid.bin([count, total])
    shape = (bins + 3, bins + 3)
    gc, gs = np.asarray(count), np.asarray(total)
    oc, osm = cnt.reshape(shape, order="F"), sm.reshape(shape, order="F")
    diff = int(np.count_nonzero(gc != oc))
    nz = osm != 0
    rel = float(np.max(np.abs(gs[nz] - osm[nz]) / np.abs(osm[nz]))) if nz.any() else 0.0
    zero_ok = bool(np.all(gs[~nz] == 0))
    return {"rows": int(m), "cells": int(gc.size), "occupied_cells": int(np.count_nonzero(oc)),
            "count_cells_differing": diff, "sum_max_rel_err": rel,
            "ok": bool(diff == 0 and rel <= 1e-6 and zero_ok)}


def cpu_baseline_groupby(m=1 << 25, repeats=3):
    """C3 on a bounded sample: the first m rows of the bench's key / value columns (the
    counter-based generator gives the same rows), groupby(key).agg({v: [sum, count]}) by the
    oracle's NumPy restatement (oracle.groupby_reference: sort-based, sums in row order; one
    core) -- timed as the C3 CPU baseline -- and through the GPU routes 'auto' (dense grid)
    and assume_sparse=True (first-appearance order), compared group by group: keys and
    counts exact, sums rtol 1e-6."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    from oracle import oracle
    keys = DeviceArray.random(m, "randint", seed=5, a=5, b=5 + 1_000_000, dtype="int32")
    v = DeviceArray.random(m, "normal", seed=6)
    hk, hv = keys.to_numpy(), v.to_numpy()
    ts = []
    for _ in range(repeats):
        t0 = time.perf_counter()
        uk, us, uc = oracle.groupby_reference(hk, hv)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    base = {"value": m / t, "unit": "rows/s", "cores": 1, "kind": "port",
            "sample": f"first {m} rows of the C3 key / value columns, oracle.groupby_reference (NumPy), "
                      f"median of {repeats} runs ({t:.2f} s each)"}
    df = vaex_amd.from_arrays(key=keys, v=v)
    parity = {"rows": m, "groups": int(len(uk))}
    ok = True
    for route, sparse in (("auto", "auto"), ("hash", True)):
        g = df.groupby("key", agg={"v": ["sum", "count"]}, assume_sparse=sparse)
        gk, gc, gs = g["key"].to_numpy(), g["v"].to_numpy(), g["v_sum"].to_numpy()
        o = np.argsort(gk, kind="stable")
        same = len(gk) == len(uk) and bool(np.array_equal(gk[o], uk)) and bool(np.array_equal(gc[o], uc))
        big = np.abs(us) > 1e-6  # near-zero sums of normal values: the absolute bound below
        rel = float(np.max(np.abs(gs[o][big] - us[big]) / np.abs(us[big]))) if same and big.any() else None
        r_ok = same and bool(np.allclose(gs[o], us, rtol=1e-6, atol=1e-9))
        if sparse is True and r_ok:  # first-appearance order: groups sorted by their first row
            _, first = np.unique(hk, return_index=True)
            r_ok = bool(np.array_equal(gk, uk[np.argsort(first, kind="stable")]))
            parity[route + "_first_appearance_order"] = r_ok
        parity[route] = {"keys_counts_equal": same, "sum_max_rel_err": rel, "ok": r_ok}
        ok = ok and r_ok
    parity["ok"] = ok
    return base, parity


def bench_c1(args, repeats=5, gpu_repeats=20):
    """C1 (BASELINE configs[0]): df.count(binby='x', shape=256) on 1e7 float64 rows with no
    limits -- the minmax limits pre-pass, then the bin pass -- end to end
    through the DataFrame API on an HBM column (median of `gpu_repeats`), next to the C
    port of the reference's ExecutorLocal (T threads, private per-thread grids, median of
    `repeats`); also the bin pass alone with limits=[-5, 5]."""
    import vaex_amd
    from vaex_amd.device import DeviceArray
    from oracle import oracle
    n, bins = 10_000_000, 256
    x = DeviceArray.random(n, "normal", seed=1)
    df = vaex_amd.from_arrays(x=x)
    out = {"rows": n, "bins": bins, "algorithmic_bytes_per_row": {"minmax+bin": 16, "bin": 8}}
    for name, lim in (("minmax+bin", None), ("bin", [-5.0, 5.0])):
        df.count(binby="x", shape=bins, limits=lim)
        ts = []
        for _ in range(gpu_repeats):
            t0 = time.perf_counter()
            c = df.count(binby="x", shape=bins, limits=lim)
            ts.append(time.perf_counter() - t0)
        t = float(np.median(ts))
        out[name] = {"gpu_ms": round(t * 1e3, 4), "gpu_rows_per_s": n / t, "count_total": int(np.asarray(c).sum())}
    L = oracle.lib()
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    hx = x.to_numpy()
    lim = np.zeros(2)
    g = np.zeros(bins + 3, np.int64)
    for name, do_mm in (("minmax+bin", 1), ("bin", 0)):
        if not do_mm:
            lim[:] = (-5.0, 5.0)
        ts = []
        for _ in range(repeats):
            t0 = time.perf_counter()
            L.or_bench_count1d(hx.ctypes.data, n, threads, bins, do_mm, lim.ctypes.data, g.ctypes.data)
            ts.append(time.perf_counter() - t0)
        t = float(np.median(ts))
        out[name].update(cpu_ms=round(t * 1e3, 3), cpu_rows_per_s=n / t, cpu_threads=threads,
                         cpu_equal=bool(int(g.sum()) == n))
        out[name]["gpu_over_cpu"] = round(out[name]["gpu_rows_per_s"] / out[name]["cpu_rows_per_s"], 2)
    return out


if __name__ == "__main__":
    main()
