#!/bin/bash
# Round measurement: the default bench line, then rocprofv3 kernel-trace stats and the
# FETCH_SIZE / WRITE_SIZE passes of the same workload (summaries copied into profiles/).
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit 1
tail -1 gpurun_out/bench_$TAG.log
bash scripts/profile.sh $TAG || exit 1
