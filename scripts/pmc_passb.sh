#!/bin/bash
# SQ counters of pass B for the C2 var and C2 min / max plans (one PMC pass, kernel trace only)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmc_passb
mkdir -p $OUT
for wl in c2var c2mm; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_ANY SQ_INSTS_SALU --kernel-trace --output-format csv -d $OUT/$wl -o run -- python3 scripts/ab_inproc.py vaex_amd/libvaexhip.so --workloads $wl --rounds 1 > $OUT/$wl.log 2>&1
  rc=$?; echo "$wl rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
