#!/bin/bash
# C3 auto query: cProfile of the host side + rocprofv3 kernel/copy timeline of the last query.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/c3tl_${1:-a}
mkdir -p $OUT
timeout -k 10 300 python3 scripts/exp_c3_overhead.py > $OUT/overhead.log 2>&1
rc=$?; echo "overhead rc=$rc"; [ $rc -eq 0 ] || exit $rc
WITH_C2=0 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/tl -o run -- python3 scripts/exp_timeline.py > $OUT/tl.log 2>&1
rc=$?; echo "timeline rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/tl_summary.py $(ls -d $OUT/tl/*/ | head -1)run minmax > $OUT/tl_summary.txt 2>&1 || python3 - <<'PY'
import glob; print(glob.glob("gpurun_out/c3tl_*/tl/**", recursive=True)[:20])
PY
tail -40 $OUT/tl_summary.txt
