#!/bin/bash
# C3 dense pass A (k_tile_scatter_ord) with parts switched off (VH_TILE_DEBUG bits, ablation
# build only, results wrong by design): 0 full; 128 no region stores; 32 no commit; 96 no
# commit + no ranking.  Kernel times from HIP events (ab_inproc's c3 workload, one build).
export VAEX_AMD_LIB="${GRAFT_REPO_ROOT:-$(pwd)}/vaex_amd/libvaexhip_ablation.so"
cd "$GRAFT_REPO_ROOT" || exit 1
for d in ${DBGS:-0 128 32 96}; do
  VH_TILE_DEBUG=$d timeout -k 10 200 python3 scripts/ab_inproc.py $VAEX_AMD_LIB --workloads c3 --rounds 4 > gpurun_out/c3abl_$d.log 2>&1
  echo "dbg=$d rc=$?"; grep -E "tile_|c3" gpurun_out/c3abl_$d.log | head -8
done
