#!/bin/bash
# Separate rocprofv3 PMC passes over one command: pmc_passes.sh TAG -- cmd...
# (each pass its own run; no trace domains mixed with --pmc)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=$1; shift; shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_VMEM" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_FLAT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d $OUT/p$i -o run -- "$@" > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($ctr) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- "$@" > $OUT/trace.log 2>&1
echo "trace rc=$?"
