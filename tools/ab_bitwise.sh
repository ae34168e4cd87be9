#!/bin/bash
# Bitwise check of engine-library variants (tools/ab_build.sh): the last step's u0 of bench.py for each variant,
# compared with the first.  Usage: bash tools/ab_bitwise.sh OUTDIR "bench args" NAME1 NAME2 ...
set -e
OUT=$1; shift
ARGS=$1; shift
mkdir -p "$OUT"
for n in "$@"; do
  MPCC_ENGINE_LIB=mpcc_manipulator_amd/_ab/$n/libmpcc_engine.so timeout -k 10 200 python bench.py --no-cpu-baseline \
      --steps 3 --warmup 1 $ARGS --dump-u0 "$OUT/u0_$n.npy" > "$OUT/bw_$n.json" 2> "$OUT/bw_$n.err"
done
python - "$OUT" "$@" <<'PY'
import sys, numpy as np
out, names = sys.argv[1], sys.argv[2:]
a = np.load(f"{out}/u0_{names[0]}.npy")
for n in names[1:]:
    b = np.load(f"{out}/u0_{n}.npy")
    print(n, "bitwise" if np.array_equal(a, b) else "DIFFERS max|du0| %.3e" % np.abs(a - b).max(), flush=True)
PY
