#!/bin/bash
# GPU tests against the bounds-checked engine libraries (MPCC_BOUNDS_CHECK build, mpcc_manipulator_amd/_build_bchk/):
# every computed workspace / QP record / ring / LDS / spline index is tested in the kernels and the autouse
# fixture of tests/conftest.py asserts after each test that none was out of range.
# Build (CPU): MPCC_BOUNDS_CHECK=1 python -m mpcc_manipulator_amd._build
# Usage (GPU box): bash tools/bounds_check.sh tests/test_mobile.py tests/test_bfgs.py ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
export MPCC_ENGINE_LIB=$ROOT/mpcc_manipulator_amd/_build_bchk/libmpcc_engine.so
export MPCC_ENGINE_LIB_MOBILE=$ROOT/mpcc_manipulator_amd/_build_bchk/libmpcc_engine_mobile.so
python - <<EOF
import sys; sys.path.insert(0, "$ROOT")
from mpcc_manipulator_amd import engine
for dof in (7, 10):
    assert engine.lib(dof).mpcc_build_flags() & engine.BUILD_BOUNDS_CHECK, engine.LIB_PATHS[dof]
print("bounds-checked libraries:", engine.build_id(7), engine.build_id(10))
EOF
python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@"
