set -o pipefail
cd $GRAFT_REPO_ROOT
export PROF=mpcc_manipulator_amd/_build_prof/libmpcc_engine.so
timeout -k 10 200 python tools/tail_diff.py --batch 4096 > gpurun_out/r04d_tail_diff.log 2>&1; echo diff_rc=$?
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tail_mode.py > gpurun_out/r04d_tail_tests.log 2>&1; echo tests_rc=$?
MPCC_ENGINE_LIB=$PROF timeout -k 10 200 python tools/ipm_prof.py --batch 1 4 2048 > gpurun_out/r04d_ipm_prof.json 2>&1
echo rc=$?
