#!/bin/bash
# Alternating A/B bench of engine-library variants (tools/ab_build.sh) on one box: k_sqp mean launch and solves/s
# per run.  Usage: bash tools/ab_bench.sh OUTDIR "bench args" NAME1 NAME2 ... (ROUNDS rounds, default 3)
set -e
OUT=$1; shift
ARGS=$1; shift
mkdir -p "$OUT"
for r in $(seq 1 ${ROUNDS:-3}); do
  for n in "$@"; do
    MPCC_ENGINE_LIB=mpcc_manipulator_amd/_ab/$n/libmpcc_engine.so timeout -k 10 200 python bench.py --no-cpu-baseline $ARGS \
        > "$OUT/${n}_$r.json" 2> "$OUT/${n}_$r.err"
    python -c "import json,sys; d=json.load(open('$OUT/${n}_$r.json')); r=d['roofline']; m = r.get('mlp') or {}; print('$n', $r, round(d['value']), round(r['avg_launch_ms'], 4), {k: round(v['avg_launch_ms'], 3) for k, v in m.items()}, flush=True)"
  done
done
