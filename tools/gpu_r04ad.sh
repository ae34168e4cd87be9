set -o pipefail
cd $GRAFT_REPO_ROOT
for v in n h l n; do
MPCC_SOLO_PRIO=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04ad_$v.json 2> gpurun_out/r04ad_$v.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/r04ad_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
