set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py > gpurun_out/r04t_bench_default.json 2> gpurun_out/r04t_bench_default.err
echo bench_rc=$?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04t_smoke.log 2>&1
echo smoke_rc=$?
