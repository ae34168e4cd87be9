set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_tail_mode.py > gpurun_out/r04k_tail_tests.log 2>&1
echo tests_rc=$?
MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_prof/libmpcc_engine.so timeout -k 10 200 python tools/ipm_prof.py --batch 1 > gpurun_out/r04k_ipm_prof.json 2>&1
echo prof_rc=$?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04k_bench.json 2> gpurun_out/r04k_bench.err
echo bench_rc=$?
MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_vpf0/libmpcc_engine.so timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04k_bench_pf0.json 2> gpurun_out/r04k_bench_pf0.err
echo bench0_rc=$?
