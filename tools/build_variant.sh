#!/bin/bash
# Experimental build: libswifthip with swh_hydro.hip compiled under extra
# defines (e.g. -DSWH_TILE_WPE=4), written to swift_subtask_dev_amd/_exp/<name>.so.
# Load it with SWH_LIB_PATH=swift_subtask_dev_amd/_exp/<name>.so.
# usage: tools/build_variant.sh <name> <defines...>   (SRC=swh_grav.hip for the gravity file)
set -e
name="$1"; shift
src="${SRC:-swh_hydro.hip}"
cd "$(dirname "$0")/.."
python -c "from swift_subtask_dev_amd import build as b; b.build()" > /dev/null
pkg=swift_subtask_dev_amd; obj=$pkg/_obj; out=$pkg/_exp
mkdir -p "$out"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function \
  -Wno-unused-variable -Iinclude -I$pkg/csrc -fvisibility=hidden -DSWH_BUILD "$@" \
  -c $pkg/csrc/$src -o "$out/$name.hydro.o"
others=$(ls $obj/*.o | grep -v "${src%.hip}")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/$name.so" "$out/$name.hydro.o" $others -lhipfft
rm -f "$out/$name.hydro.o"
echo "built $out/$name.so"
