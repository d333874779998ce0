#!/bin/bash
# rocprofv3 kernel-trace stats + separate PMC passes (FETCH_SIZE, WRITE_SIZE) for the bench.
# The rocpd databases stay in /tmp on the box (tens of MB each); the summary table and the
# per-kernel JSON bench.py reads come back in gpurun_out/: prof_<tag>.txt, pmc_<tag>.json.
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r01}
ROWS=${2:-1e9}
OUT=/tmp/prof_$TAG
mkdir -p $OUT gpurun_out
ARGS="--rows $ROWS --steps 3 --warmup 1 --no-cpu-baseline --host-rows 0 --c4-rows 0 --h2o-rows 0 --no-aggs --no-layouts --no-set --groupby-rows $ROWS $PROF_ARGS"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $OUT gpurun_out/pmc_$TAG.json $ROWS > gpurun_out/prof_$TAG.txt
echo "summary rc=$?"
