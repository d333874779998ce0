#!/bin/bash
# the experiment switches exist only in the ablation build (make -C vaex_amd/csrc ablation)
export VAEX_AMD_LIB="${GRAFT_REPO_ROOT:-$(pwd)}/vaex_amd/libvaexhip_ablation.so"
# Pass-A time breakdown: the C2 bench under VH_TILE_DEBUG switches / experiment builds
# (results are wrong by design).  usage: RUNS="lib:dbg lib:dbg ..." scripts/exp_debug.sh
cd "$GRAFT_REPO_ROOT" || exit 1
for run in ${RUNS:-libvaexhip:0}; do
  lib=${run%%:*}; dbg=${run#*:}
  VAEX_AMD_LIB=vaex_amd/$lib.so VH_TILE_DEBUG=$dbg timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --host-rows 0 --no-groupby > gpurun_out/dbg_$lib_$dbg.log 2>&1 || exit 1
  tail -1 gpurun_out/dbg_$lib_$dbg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$run', round(d['ms_per_step'],3), d['roofline']['per_kernel_ms'], 'count_only', round(d['count_only']['ms_per_step'],3), d['count_only']['per_kernel_ms'])"
done
