#!/bin/bash
# A/B variant of the Panda engine library: one source (SRC, default ipm.hip) recompiled with extra -D flags and
# linked with the other objects of the regular build (mpcc_manipulator_amd/_build).
# Usage: [SRC=mlp.hip] bash tools/ab_build.sh NAME -DFLAG=0 ...
# Output: mpcc_manipulator_amd/_ab/NAME/libmpcc_engine.so (select with MPCC_ENGINE_LIB).
set -e
NAME=$1; shift
SRC=${SRC:-ipm.hip}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=$ROOT/mpcc_manipulator_amd/_build
OUT=$ROOT/mpcc_manipulator_amd/_ab/$NAME
mkdir -p "$OUT"
STEM=${SRC%.*}
EXTRA=""
case $SRC in kernels.hip|mlp.hip|nn_generic.hip) EXTRA="-ffp-contract=off";; esac
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I "$ROOT/include" -I "$ROOT/mpcc_manipulator_amd/csrc" \
    -Wno-unused-result $EXTRA "$@" -c "$ROOT/mpcc_manipulator_amd/csrc/$SRC" -o "$OUT/$STEM.o"
OBJS=""
for o in kernels ipm ipm_wide mlp nn_generic engine host_params host_spline mpc; do
  if [ "$o" = "$STEM" ]; then OBJS="$OBJS $OUT/$o.o"; else OBJS="$OBJS $B/$o.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libmpcc_engine.so" $OBJS
echo "$OUT/libmpcc_engine.so"
