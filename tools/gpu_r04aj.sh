set -o pipefail
cd $GRAFT_REPO_ROOT
for s in 2 1 4 3 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --sub-batches $s > gpurun_out/r04aj_s$s.json 2> gpurun_out/r04aj_s$s.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/r04aj_s$s.json').read().strip().splitlines()[-1]); print('S$s', d['value'], d['ms_per_step'])"
done
