#!/bin/bash
# rocprofv3 trace + SQ/LDS counters of the ordered_set update (scripts/exp_set.py)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prof_set
mkdir -p $OUT
timeout -k 10 300 python3 scripts/exp_set.py 1e9 3 > $OUT/plain.log 2>&1; echo "plain rc=$?"; cat $OUT/plain.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 scripts/exp_set.py 1e9 2 > $OUT/trace.log 2>&1
echo "trace rc=$?"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_VMEM --kernel-trace -d $OUT/sq -o run -- python3 scripts/exp_set.py 1e9 1 > $OUT/sq.log 2>&1
echo "sq rc=$?"
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM --kernel-trace -d $OUT/sq2 -o run -- python3 scripts/exp_set.py 1e9 1 > $OUT/sq2.log 2>&1
echo "sq2 rc=$?"
find $OUT -name "*.csv" | head
