#!/bin/bash
# Process-level A/B of the bench's headline step: `bench.py` (C2 leg only) with the current
# library and with a variant (VAEX_AMD_LIB), interleaved ROUNDS times on one box.
# usage: ROUNDS=2 bash scripts/ab_bench_c2.sh OUT variant.so
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$1; VAR=$2
: > $OUT
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-groupby --no-layouts --no-aggs --no-set --no-count-only --no-f32 --no-filtered --host-rows 0 --c4-rows 0 --h2o-rows 0"
for r in $(seq ${ROUNDS:-2}); do
  for tag in cur var; do
    if [ $tag = var ]; then
      VAEX_AMD_LIB="$VAR" timeout -k 10 300 python3 bench.py $ARGS > /tmp/ab_$tag.log 2>&1 || exit 1
    else
      timeout -k 10 300 python3 bench.py $ARGS > /tmp/ab_$tag.log 2>&1 || exit 1
    fi
    echo "$tag $(python3 scripts/bench_brief.py /tmp/ab_$tag.log | head -1)" >> $OUT
  done
done
cat $OUT
