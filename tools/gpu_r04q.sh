set -o pipefail
cd $GRAFT_REPO_ROOT
MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_prof/libmpcc_engine.so timeout -k 10 200 python tools/solo_prof.py --batch 2048 > gpurun_out/r04q_solo_prof.json 2>&1
echo rc=$?
MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_prof/libmpcc_engine.so timeout -k 10 200 python tools/ipm_prof.py --batch 1 > gpurun_out/r04q_ipm_prof.json 2>&1
echo rc=$?
