set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tail_mode.py -k "solo" > gpurun_out/r04aa_solo_tests.log 2>&1
echo tests_rc=$?
grep -q "3 passed" gpurun_out/r04aa_solo_tests.log || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04aa_bench.json 2> gpurun_out/r04aa_bench.err
echo bench_rc=$?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04aa_trace -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r04aa_bench_trace.json 2> $GRAFT_REPO_ROOT/gpurun_out/r04aa_bench_trace.err
echo trace_rc=$?
