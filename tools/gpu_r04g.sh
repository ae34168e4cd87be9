set -o pipefail
cd $GRAFT_REPO_ROOT
DBG2=1 MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_vdbg2/libmpcc_engine.so timeout -k 10 120 python tools/tail_ws_diff.py > gpurun_out/r04g_ws_diff_dbg2.log 2>&1
echo rc=$?
MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_prof/libmpcc_engine.so timeout -k 10 200 python tools/ipm_prof.py --batch 1 > gpurun_out/r04g_ipm_prof.json 2>&1
echo rc=$?
