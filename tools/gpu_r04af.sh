set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --batch 65536 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r04af_c4share.json 2> gpurun_out/r04af_c4share.err
echo c4=$?
timeout -k 10 300 python bench.py --config 1-all-rows --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04af_c1all.json 2> gpurun_out/r04af_c1all.err
echo c1all=$?
timeout -k 10 400 python bench.py --config 2 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r04af_c2.json 2> gpurun_out/r04af_c2.err
echo c2=$?
timeout -k 10 400 python bench.py --config 3 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r04af_c3.json 2> gpurun_out/r04af_c3.err
echo c3=$?
