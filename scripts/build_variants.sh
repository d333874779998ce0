#!/bin/bash
# Build tiled.hip variants (compile-time tuning macros) as vaex_amd/libvaexhip_<name>.so for A/B runs.
# usage: scripts/build_variants.sh name:"-DFLAG=.. -DFLAG2=.." ...
set -e
cd "$(dirname "$0")/../vaex_amd/csrc"
make -s
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -munsafe-fp-atomics"
for v in "$@"; do
  name=${v%%:*}; fl=${v#*:}
  mkdir -p build/var_$name
  /opt/rocm/bin/hipcc $F $fl -c tiled.hip -o build/var_$name/tiled.o &&
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libvaexhip_$name.so build/runtime.o build/binning.o build/hashset.o build/var_$name/tiled.o &
done
wait
