#!/bin/bash
# Build an engine variant: ipm.hip recompiled with extra flags, the other objects from _build.
# Usage: bash tools/build_variant.sh NAME "-DFOO=1 ..." [ipm source]  -> mpcc_manipulator_amd/_build_vNAME/libmpcc_engine.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=$ROOT/mpcc_manipulator_amd/_build
V=$ROOT/mpcc_manipulator_amd/_build_v$1
mkdir -p "$V"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I "$ROOT/include" -I "$ROOT/mpcc_manipulator_amd/csrc" \
    -Wno-unused-result $2 -c "${3:-$ROOT/mpcc_manipulator_amd/csrc/ipm.hip}" -o "$V/ipm.o"
objs=""
for o in ipm_wide kernels mlp nn_generic engine host_params host_spline mpc; do objs="$objs $B/$o.o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$V/libmpcc_engine.so" "$V/ipm.o" $objs
echo "built $V"
