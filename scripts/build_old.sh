#!/bin/bash
# Build libvaexhip_<name>.so from a git revision of ONE source file (A/B against the working tree).
# usage: scripts/build_old.sh <rev> <src-without-.hip> <name>
set -e
REV=$1; SRC=$2; NAME=$3
cd "$(dirname "$0")/../vaex_amd/csrc"
make -s
mkdir -p build/var_$NAME
git show $REV:vaex_amd/csrc/$SRC.hip > build/var_$NAME/$SRC.hip
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -munsafe-fp-atomics -I."
/opt/rocm/bin/hipcc $F -c build/var_$NAME/$SRC.hip -o build/var_$NAME/$SRC.o
others=""
for o in runtime binning tiled hashset hashagg expr nunique comm; do [ "$o" = "$SRC" ] || others="$others build/$o.o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libvaexhip_$NAME.so $others build/var_$NAME/$SRC.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
