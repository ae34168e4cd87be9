set -o pipefail
cd $GRAFT_REPO_ROOT
export SB4=mpcc_manipulator_amd/_build_vsb4/libmpcc_engine.so
MPCC_ENGINE_LIB=$SB4 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tail_mode.py -k "solo" > gpurun_out/r04z_sb4_tests.log 2>&1
echo sb4_tests_rc=$?
grep -q "3 passed" gpurun_out/r04z_sb4_tests.log && MPCC_ENGINE_LIB=$SB4 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04z_sb4_bench.json 2> gpurun_out/r04z_sb4_bench.err
echo sb4_bench_rc=$?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04z_sb2_bench.json 2> gpurun_out/r04z_sb2_bench.err
echo sb2_bench_rc=$?
timeout -k 10 900 bash tools/profile_round.sh gpurun_out/r04z_prof > gpurun_out/r04z_prof.log 2>&1
echo prof_rc=$?
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py > gpurun_out/r04z_bench_default.json 2> gpurun_out/r04z_bench_default.err
echo bench_rc=$?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04z_smoke.log 2>&1
echo smoke_rc=$?
