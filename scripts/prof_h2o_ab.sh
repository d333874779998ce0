#!/bin/bash
# rocprofv3 kernel traces of h2o queries for the current library and a variant (A/B on one box)
# usage: scripts/prof_h2o_ab.sh <variant.so> <rows> <queries...>
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
VAR=$1; ROWS=$2; shift 2
for tag in new old; do
  OUT=gpurun_out/prof_ab_$tag
  mkdir -p $OUT
  if [ $tag = old ]; then export VAEX_AMD_LIB=$VAR; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 scripts/exp_h2o.py $ROWS "$@" > $OUT/log.txt 2>&1 || exit 1
  echo "== $tag"; grep -E "^q" $OUT/log.txt
  python3 scripts/prof_summary.py $OUT | sed -n 2,8p
done
