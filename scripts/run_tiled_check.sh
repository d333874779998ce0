#!/bin/bash
# tile-path tests + the bench's C2 lines (new pass A)
cd "$GRAFT_REPO_ROOT" || exit 1
TMO=500 LOG=gpurun_out/pytest_tiled.log bash scripts/gpu_tests.sh tests/test_gpu_superagg.py tests/test_gpu_groupby.py tests/test_gpu_api.py tests/test_gpu_multikey.py tests/test_gpu_distributed.py || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --host-rows 0 > gpurun_out/bench_tiled.log 2>&1 || exit 1
tail -1 gpurun_out/bench_tiled.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), d['roofline']['per_kernel_ms'], 'count_only', round(d['count_only']['ms_per_step'],3), d['count_only']['per_kernel_ms']); print({k: v for k, v in d.items() if k.startswith('groupby')})"
