set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tail_mode.py > gpurun_out/r04ai_tail_tests.log 2>&1
echo tests_rc=$?
grep -q "10 passed" gpurun_out/r04ai_tail_tests.log || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04ai_c1.json 2> gpurun_out/r04ai_c1.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/r04ai_c1.json').read().strip().splitlines()[-1]); print('c1', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --batch 65536 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r04ai_c4.json 2> gpurun_out/r04ai_c4.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/r04ai_c4.json').read().strip().splitlines()[-1]); print('c4', d['value'], d['ms_per_step'])"
