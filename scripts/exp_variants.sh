cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
EXP_DEBUG=${EXP_DEBUG:-0} timeout -k 10 300 python scripts/exp_tiles.py 1e9 || exit $?
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; tail -c 3000 gpurun_out/bench.log; exit $rc
