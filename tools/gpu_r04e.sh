set -o pipefail
cd $GRAFT_REPO_ROOT
for K in 1 2; do
  MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_vstop$K/libmpcc_engine.so timeout -k 10 120 python tools/tail_ws_diff.py > gpurun_out/r04e_ws_diff_stop$K.log 2>&1 || exit 1
done
timeout -k 10 120 python tools/tail_ws_diff.py > gpurun_out/r04e_ws_diff_full.log 2>&1 || exit 1
MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_prof/libmpcc_engine.so timeout -k 10 200 python tools/ipm_prof.py --batch 1 2048 > gpurun_out/r04e_ipm_prof.json 2>&1
echo rc=$?
