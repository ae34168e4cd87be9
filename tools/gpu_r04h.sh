set -o pipefail
cd $GRAFT_REPO_ROOT
DBG2=1 MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_vdbg2/libmpcc_engine.so timeout -k 10 120 python tools/tail_ws_diff.py > gpurun_out/r04h_ws_diff_dbg2.log 2>&1
echo rc=$?
DBG2=1 MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_vstop3/libmpcc_engine.so timeout -k 10 120 python tools/tail_ws_diff.py > gpurun_out/r04h_ws_diff_stop3.log 2>&1
echo rc=$?
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_tail_mode.py > gpurun_out/r04h_tail_tests.log 2>&1
echo rc=$?
MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_vp0/libmpcc_engine.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_tail_mode.py > gpurun_out/r04h_tail_tests_p0.log 2>&1
echo rc=$?
MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_prof/libmpcc_engine.so timeout -k 10 200 python tools/ipm_prof.py --batch 1 > gpurun_out/r04h_ipm_prof.json 2>&1
echo rc=$?
