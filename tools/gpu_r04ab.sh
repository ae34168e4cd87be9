set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/r04ab_bench_prio.json 2> gpurun_out/r04ab_bench_prio.err
echo b1=$?
MPCC_SOLO_PRIO=0 timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/r04ab_bench_noprio.json 2> gpurun_out/r04ab_bench_noprio.err
echo b2=$?
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/r04ab_bench_prio2.json 2> gpurun_out/r04ab_bench_prio2.err
echo b3=$?
