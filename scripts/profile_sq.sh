#!/bin/bash
# SQ/LDS counter pass for the C2 bench kernels (no sys/runtime trace mixed in).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-sq}
ROWS=${2:-1e9}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS="--rows $ROWS --steps 2 --warmup 1 --no-cpu-baseline --no-groupby"
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS --kernel-trace -d $OUT/sq -o run -- python3 bench.py $ARGS > $OUT/sq.log 2>&1
rc=$?; echo "sq rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum --kernel-trace -d $OUT/tcc -o run -- python3 bench.py $ARGS > $OUT/tcc.log 2>&1
rc=$?; echo "tcc rc=$rc"; [ $rc -eq 0 ] || exit $rc
