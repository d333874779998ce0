#!/bin/bash
# A/B the C2 bench between library builds on one box: ab_bench.sh lib1 lib2 ...
cd "$GRAFT_REPO_ROOT" || exit 1
for round in 1 2; do
  for lib in "$@"; do
    VAEX_AMD_LIB=vaex_amd/$lib.so timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --host-rows 0 --no-groupby > gpurun_out/ab_$lib.log 2>&1 || exit 1
    tail -1 gpurun_out/ab_$lib.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', round(d['ms_per_step'],3), d['roofline']['per_kernel_ms'], 'count_only', round(d['count_only']['ms_per_step'],3), d['count_only']['per_kernel_ms'])"
  done
done
