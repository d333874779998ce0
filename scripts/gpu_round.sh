#!/bin/bash
# One GPU session: tests, smoke, bench. Stops at the first crash/timeout (not at test failures).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
STAGE=${1:-all}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
if [ "$STAGE" = all ] || [ "$STAGE" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -15
  ok $rc || exit $rc
fi
if [ "$STAGE" = all ] || [ "$STAGE" = smoke ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
  ok $rc || exit $rc
fi
if [ "$STAGE" = all ] || [ "$STAGE" = bench ]; then
  timeout -k 10 600 python bench.py --rows 1e8 --steps 5 --warmup 2 --no-cpu-baseline --groupby-rows 1e8 > gpurun_out/bench_small.log 2>&1
  rc=$?; echo "bench small rc=$rc"; tail -3 gpurun_out/bench_small.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "$STAGE" = all ] || [ "$STAGE" = fullbench ]; then
  timeout -k 10 900 python bench.py > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
  [ $rc -eq 0 ] || exit $rc
fi
