#!/bin/bash
# PMC passes for k_ipm on the benchmark workload (one counter group per pass; rocprofv3 on gfx950).
# Usage (GPU box): bash tools/pmc_ipm.sh <outdir>
set -e
OUT=${1:-gpurun_out/pmc}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$ROOT/bench.py --steps 2 --warmup 1 --pool-steps 40 --no-cpu-baseline"
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-include-regex 'k_ipm' --pmc "$@" --output-format csv -d "$ROOT/$OUT/$name" -o "$name" -- python3 $BENCH > "$ROOT/$OUT/$name.log" 2>&1
}
run p1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU
run p2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64
run p3 FETCH_SIZE
run p4 WRITE_SIZE
echo pmc done
