set -o pipefail
cd $GRAFT_REPO_ROOT
export PROF=mpcc_manipulator_amd/_build_prof/libmpcc_engine.so
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tail_mode.py > gpurun_out/r04b_tail_tests.log 2>&1
rc=$?
echo tests_rc=$rc
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.err && \
MPCC_TAIL=0 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04b_bench_notail.json 2> gpurun_out/r04b_bench_notail.err && \
MPCC_ENGINE_LIB=$PROF timeout -k 10 200 python tools/wave_times.py --batch 2048 4096 > gpurun_out/r04b_wave_times.json 2>&1
echo rc=$?
