#!/bin/bash
# Round measurement: rocprofv3 kernel-trace stats + the FETCH_SIZE / WRITE_SIZE passes of the
# bench workload (summary + PMC json written under gpurun_out/), then the default bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r03}
mkdir -p gpurun_out
bash scripts/profile.sh $TAG || exit 1
python3 scripts/prof_summary.py gpurun_out/prof_$TAG gpurun_out/pmc_c2_$TAG.json 1e9 > gpurun_out/${TAG}_bench.txt || exit 1
head -30 gpurun_out/${TAG}_bench.txt
rm -rf gpurun_out/prof_$TAG  # the rocpd databases exceed what gpurun copies back; the summary keeps their numbers
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit 1
python3 scripts/bench_summary.py gpurun_out/bench_$TAG.log
