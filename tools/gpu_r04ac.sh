set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/r04ac_q8_prio.json 2> gpurun_out/r04ac_q8_prio.err
echo b1=$?
MPCC_SOLO_PRIO=0 timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/r04ac_q8_noprio.json 2> gpurun_out/r04ac_q8_noprio.err
echo b2=$?
GPU_MAX_HW_QUEUES=12 timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/r04ac_q12_prio.json 2> gpurun_out/r04ac_q12_prio.err
echo b3=$?
