#!/bin/bash
# Round-end verification on one GPU box: the GPU suite, smoke(), the default bench line and every other BASELINE config
# on the same build.  Usage: bash tools/final_round.sh OUTDIR
set -e
OUT=$1
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -1 "$OUT/smoke.log"
b() {  # name, bench args
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err"
  python -c "import json; d=json.load(open('$OUT/bench_$n.json')); print('$n', round(d['value']), round(d['ms_per_step'], 3), flush=True)"
}
b c1 --steps 20 --warmup 3
b c1all --config 1-all-rows --no-cpu-baseline --steps 10 --warmup 2
b c2 --config 2 --no-cpu-baseline --steps 8 --warmup 2
b c3 --config 3 --no-cpu-baseline --steps 8 --warmup 2
b c4share --batch 65536 --no-cpu-baseline --steps 10 --warmup 2
b c1b --steps 20 --warmup 3 --no-cpu-baseline
