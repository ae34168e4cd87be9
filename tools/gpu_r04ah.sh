set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 2 1 2 1; do
MPCC_SOLO=$v timeout -k 10 300 python bench.py --batch 65536 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r04ah_c4_$v.json 2> gpurun_out/r04ah_c4_$v.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/r04ah_c4_$v.json').read().strip().splitlines()[-1]); print('solo$v', d['value'], d['ms_per_step'])"
done
