#!/bin/bash
# Round profile of the benchmark command (GPU box): rocprofv3 kernel trace + stats of bench.py, then
# separate PMC passes for the dominant kernel (KERNEL, default k_sqp; never combined with trace domains).
# Usage: [KERNEL=k_mlp_env] [NOTRACE=1] bash tools/profile_round.sh OUT [bench.py args, e.g. --config 2]
set -e
OUT=${1:-gpurun_out/prof}
shift || true
EXTRA="$*"
ROOT=$(pwd)
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline $EXTRA"
if [ -z "$NOTRACE" ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace" -o trace -- \
    python3 $BENCH > "$ROOT/$OUT/bench_trace.json" 2> "$ROOT/$OUT/bench_trace.err"
echo "trace done"
fi
PMCB="$ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline $EXTRA"
pmc() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-include-regex "${KERNEL:-k_sqp}" --pmc "$@" --output-format csv \
      -d "$ROOT/$OUT/$name" -o "$name" -- python3 $PMCB > "$ROOT/$OUT/$name.log" 2>&1
}
pmc p1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU
pmc p2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64
pmc p3 FETCH_SIZE
pmc p4 WRITE_SIZE
pmc p5 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA
echo "pmc done"
