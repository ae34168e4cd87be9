set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tail_mode.py -k "solo and 512-8" > gpurun_out/r04y_solo_quick.log 2>&1
echo quick_rc=$?
[ -f gpurun_out/r04y_solo_quick.log ] && grep -q "1 passed" gpurun_out/r04y_solo_quick.log || exit 1
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tail_mode.py > gpurun_out/r04y_tail_tests.log 2>&1
echo tests_rc=$?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04y_bench.json 2> gpurun_out/r04y_bench.err
echo bench_rc=$?
MPCC_SOLO=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04y_bench_solo1.json 2> gpurun_out/r04y_bench_solo1.err
echo bench1_rc=$?
MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_vprof/libmpcc_engine.so timeout -k 10 200 python tools/wave_times.py --batch 2048 > gpurun_out/r04y_wave_times.json 2>&1
echo wt_rc=$?
