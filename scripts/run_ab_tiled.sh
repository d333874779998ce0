#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
TMO=400 LOG=gpurun_out/pytest_tiled.log bash scripts/gpu_tests.sh tests/test_gpu_superagg.py tests/test_gpu_groupby.py tests/test_gpu_api.py || exit 1
bash scripts/ab_bench.sh libvaexhip_old libvaexhip || exit 1
for lib in libvaexhip_old libvaexhip; do
  VAEX_AMD_LIB=vaex_amd/$lib.so timeout -k 10 120 python scripts/exp_groupby.py auto > gpurun_out/ord_$lib.log 2>&1 || exit 1
  echo "$lib: $(tail -1 gpurun_out/ord_$lib.log)"
done
