#!/bin/bash
# the experiment switches exist only in the ablation build (make -C vaex_amd/csrc ablation)
export VAEX_AMD_LIB="${GRAFT_REPO_ROOT:-$(pwd)}/vaex_amd/libvaexhip_ablation.so"
# pass A of the C2 tile path with parts switched off (VH_TILE_DEBUG bits, tiled.hip):
# 0 full; 128 no region stores; 32 no commit; 96 no commit + no ranking; 16 no pass-B flush
cd "$GRAFT_REPO_ROOT" || exit 1
for d in ${DBGS:-0 128 32 96}; do
  VH_TILE_DEBUG=$d timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-groupby --host-rows 0 > gpurun_out/abl_$d.log 2>&1
  echo "dbg=$d rc=$?"; python3 - <<PY
import json
l=json.loads(open("gpurun_out/abl_$d.log").read().strip().splitlines()[-1])
print(" count+sum", l["roofline"]["per_kernel_ms"], " count-only", l["count_only"]["per_kernel_ms"])
PY
done
