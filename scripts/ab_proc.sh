#!/bin/bash
# Process-level A/B: each variant runs scripts/exp_kernels.py in its own process, variants
# interleaved ROUNDS times.  Variants are "TAG:ENV=VAL,ENV2=VAL2" (VAEX_AMD_LIB selects a
# library build).  usage: ROUNDS=2 bash scripts/ab_proc.sh OUT "a:" "b:VH_TILE_DRAIN=0" ...
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$1; shift
: > $OUT
for r in $(seq ${ROUNDS:-2}); do
  for v in "$@"; do
    tag=${v%%:*}; envs=${v#*:}
    ( IFS=,; for e in $envs; do [ -n "$e" ] && export "$e"; done
      timeout -k 10 240 python3 scripts/exp_kernels.py "$tag" ${ROWS:-1e9} ${REPS:-5} >> $OUT 2>>$OUT.err ) || exit 1
  done
done
cat $OUT
