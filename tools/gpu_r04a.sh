set -o pipefail
cd $GRAFT_REPO_ROOT
export PROF=mpcc_manipulator_amd/_build_prof/libmpcc_engine.so
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err && \
MPCC_ENGINE_LIB=$PROF timeout -k 10 200 python tools/wave_times.py --batch 2048 4096 > gpurun_out/r04a_wave_times.json 2>&1 && \
MPCC_ENGINE_LIB=$PROF timeout -k 10 200 python tools/ipm_prof.py --batch 4 2048 > gpurun_out/r04a_ipm_prof.json 2>&1
echo rc=$?
