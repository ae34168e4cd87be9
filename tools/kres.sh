#!/bin/bash
# Kernel resource usage (VGPRs, AGPRs, scratch, spills, occupancy) of one device source, as the build compiles it.
# Usage: bash tools/kres.sh ipm.hip [kernel-name regex] [extra flags, e.g. -DMPCC_DOF=10 -Dmpcc=mpcc_m10]
SRC=$1; RE=${2:-.}; shift 2 || true
ROOT=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I "$ROOT/include" -x hip "$@" \
  --offload-device-only -c "$ROOT/mpcc_manipulator_amd/csrc/$SRC" -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -A12 "Function Name: .*$RE" \
  | grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|SGPRs Spill|VGPRs Spill"
