#!/bin/bash
# correctness of the working-tree library, then an A/B of library builds on one box
cd "$GRAFT_REPO_ROOT" || exit 1
TMO=400 LOG=gpurun_out/pytest_tiled.log bash scripts/gpu_tests.sh tests/test_gpu_superagg.py tests/test_gpu_groupby.py tests/test_gpu_api.py || exit 1
bash scripts/ab_bench.sh ${LIBS:-libvaexhip_old libvaexhip} || exit 1
