set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04am_tests.log 2>&1
echo tests=$?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04am_smoke.log 2>&1
echo smoke_rc=$?
timeout -k 10 600 python bench.py > gpurun_out/r04am_bench_default.json 2> gpurun_out/r04am_bench_default.err
echo bench_rc=$?
