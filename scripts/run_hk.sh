#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
TMO=500 LOG=gpurun_out/pytest_hk.log bash scripts/gpu_tests.sh tests/test_gpu_hashagg.py tests/test_gpu_multikey.py tests/test_gpu_groupby.py || exit 1
for lib in libvaexhip_v1 libvaexhip libvaexhip_v1 libvaexhip; do
  VAEX_AMD_LIB=vaex_amd/$lib.so timeout -k 10 120 python scripts/exp_groupby.py fused > gpurun_out/hk_$lib.log 2>&1 || exit 1
  echo "$lib: $(tail -1 gpurun_out/hk_$lib.log)"
done
KEYDT=int64 timeout -k 10 120 python scripts/exp_groupby.py fused > gpurun_out/hk_i64.log 2>&1 || exit 1
echo "int64: $(tail -1 gpurun_out/hk_i64.log)"
