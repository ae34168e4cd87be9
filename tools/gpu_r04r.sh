set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tail_mode.py > gpurun_out/r04r_tail_tests.log 2>&1
echo tests_rc=$?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04r_bench.json 2> gpurun_out/r04r_bench.err
echo bench_rc=$?
MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_prof/libmpcc_engine.so timeout -k 10 200 python tools/solo_prof.py --batch 2048 > gpurun_out/r04r_solo_prof.json 2>&1
echo rc=$?
MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_prof/libmpcc_engine.so timeout -k 10 200 python tools/wave_times.py --batch 2048 > gpurun_out/r04r_wave_times.json 2>&1
echo wt_rc=$?
