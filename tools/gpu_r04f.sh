set -o pipefail
cd $GRAFT_REPO_ROOT
MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_vdbg1/libmpcc_engine.so timeout -k 10 120 python tools/tail_ws_diff.py > gpurun_out/r04f_ws_diff_dbg1.log 2>&1
echo rc=$?
