set -o pipefail
cd $GRAFT_REPO_ROOT
export PROF=mpcc_manipulator_amd/_build_prof/libmpcc_engine.so
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04i_bench.json 2> gpurun_out/r04i_bench.err
echo bench_rc=$?
MPCC_ENGINE_LIB=$PROF timeout -k 10 200 python tools/wave_times.py --batch 2048 > gpurun_out/r04i_wave_times.json 2>&1
echo wt_rc=$?
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04i_gpu_tests.log 2>&1
echo tests_rc=$?
