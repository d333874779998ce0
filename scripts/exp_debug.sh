#!/bin/bash
# Pass-A time breakdown: the C2 bench under VH_TILE_DEBUG switches (1 = no region stores,
# 2 = no commit (sort + stores), 4 = no LDS rank atomics); results are wrong by design.
cd "$GRAFT_REPO_ROOT" || exit 1
for dbg in ${DBGS:-0 1 2 4 0}; do
  VH_TILE_DEBUG=$dbg timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --host-rows 0 --no-groupby > gpurun_out/dbg_$dbg.log 2>&1 || exit 1
  tail -1 gpurun_out/dbg_$dbg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('dbg $dbg', round(d['ms_per_step'],3), d['roofline']['per_kernel_ms'], 'count_only', round(d['count_only']['ms_per_step'],3), d['count_only']['per_kernel_ms'])"
done
