#!/bin/bash
# Build variants of one HIP source (compile-time tuning macros) as vaex_amd/libvaexhip_<name>.so
# for A/B runs (select one with VAEX_AMD_LIB=vaex_amd/libvaexhip_<name>.so).
# usage: SRC=hashagg scripts/build_variants.sh name:"-DFLAG=.. -DFLAG2=.." ...
set -e
SRC=${SRC:-tiled}
cd "$(dirname "$0")/../vaex_amd/csrc"
make -s
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -munsafe-fp-atomics"
OBJS="runtime binning tiled first hashset hashagg expr nunique comm"
for v in "$@"; do
  name=${v%%:*}; fl=${v#*:}
  mkdir -p build/var_$name
  others=""
  for o in $OBJS; do [ "$o" = "$SRC" ] || others="$others build/$o.o"; done
  ( /opt/rocm/bin/hipcc $F $fl -c $SRC.hip -o build/var_$name/$SRC.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libvaexhip_$name.so $others build/var_$name/$SRC.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib ) &
done
wait
