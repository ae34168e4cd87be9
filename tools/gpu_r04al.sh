set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tail_mode.py -k solo > gpurun_out/r04al_solo_tests.log 2>&1
echo tests_rc=$?
grep -q "3 passed" gpurun_out/r04al_solo_tests.log || exit 1
for v in 0 1 0 1; do
MPCC_SOLO_SIDE=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04al_side$v.json 2> gpurun_out/r04al_side$v.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/r04al_side$v.json').read().strip().splitlines()[-1]); print('side$v', d['value'], d['ms_per_step'])"
done
