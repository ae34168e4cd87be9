#!/bin/bash
# Alternating A/B bench of runtime switches: each variant is "NAME:VAR=VALUE[,VAR=VALUE]" (or "NAME:" for none), on the
# in-tree library (or MPCC_ENGINE_LIB=mpcc_manipulator_amd/_ab/NAME when NAME has a built variant).
# Usage: ROUNDS=3 bash tools/ab_env.sh OUTDIR "bench args" NAME:VARS ...
set -e
OUT=$1; shift
ARGS=$1; shift
mkdir -p "$OUT"
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in "$@"; do
    n=${v%%:*}; vars=${v#*:}
    envs=""; [ -n "$vars" ] && envs=$(echo "$vars" | tr ',' ' ')
    lib=""; [ -f "mpcc_manipulator_amd/_ab/$n/libmpcc_engine.so" ] && lib="MPCC_ENGINE_LIB=mpcc_manipulator_amd/_ab/$n/libmpcc_engine.so"
    env $envs $lib timeout -k 10 300 python bench.py --no-cpu-baseline $ARGS > "$OUT/${n}_$r.json" 2> "$OUT/${n}_$r.err"
    python -c "import json; d=json.load(open('$OUT/${n}_$r.json')); r=d['roofline']; m = r.get('mlp') or {}; print('$n', $r, round(d['value']), round(r['avg_launch_ms'], 4), {k: round(v['avg_launch_ms'], 3) for k, v in m.items()}, flush=True)"
  done
done
