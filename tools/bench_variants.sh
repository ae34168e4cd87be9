#!/bin/bash
# Bench several engine builds (mpcc_manipulator_amd/_build_v<X>) back to back on one GPU box.
# Usage: bash tools/bench_variants.sh A C D ...
set -e
mkdir -p gpurun_out
for v in "$@"; do
  MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_v$v/libmpcc_engine.so timeout -k 10 120 \
      python bench.py --no-cpu-baseline > gpurun_out/bench_v$v.log 2>&1
done
