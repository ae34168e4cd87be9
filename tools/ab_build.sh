#!/bin/bash
# A/B variant of the Panda engine library: ipm.hip recompiled with extra -D flags and linked with the other
# objects of the regular build (mpcc_manipulator_amd/_build).  Usage: bash tools/ab_build.sh NAME -DFLAG=0 ...
# Output: mpcc_manipulator_amd/_ab/NAME/libmpcc_engine.so (select with MPCC_ENGINE_LIB).
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=$ROOT/mpcc_manipulator_amd/_build
OUT=$ROOT/mpcc_manipulator_amd/_ab/$NAME
mkdir -p "$OUT"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I "$ROOT/include" -I "$ROOT/mpcc_manipulator_amd/csrc" \
    -Wno-unused-result "$@" -c "$ROOT/mpcc_manipulator_amd/csrc/ipm.hip" -o "$OUT/ipm.o"
OBJS="$B/kernels.o $B/ipm_wide.o $B/mlp.o $B/nn_generic.o $B/engine.o $B/host_params.o $B/host_spline.o $B/mpc.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libmpcc_engine.so" "$OUT/ipm.o" $OBJS
echo "$OUT/libmpcc_engine.so"
