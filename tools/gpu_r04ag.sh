set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tail_mode.py > gpurun_out/r04ag_tail_tests.log 2>&1
echo tests_rc=$?
grep -q "10 passed" gpurun_out/r04ag_tail_tests.log || exit 1
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04ag_c1_$i.json 2> gpurun_out/r04ag_c1_$i.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/r04ag_c1_$i.json').read().strip().splitlines()[-1]); print('c1', d['value'], d['ms_per_step'])"
done
bash tools/gpu_r04af.sh
