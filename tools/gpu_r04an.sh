set -o pipefail
cd $GRAFT_REPO_ROOT
MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_vprof/libmpcc_engine.so timeout -k 10 200 python tools/wave_times.py --batch 2048 > gpurun_out/r04an_wave_times.json 2>&1
echo wt_rc=$?
