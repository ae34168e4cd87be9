set -o pipefail
cd $GRAFT_REPO_ROOT
MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_vmlpprof/libmpcc_engine.so timeout -k 10 200 python tools/mlp_prof.py > gpurun_out/r04u_mlp_prof.json 2>&1
echo mlp=$?
timeout -k 10 400 python bench.py --config 2 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r04u_c2.json 2> gpurun_out/r04u_c2.err
echo c2=$?
timeout -k 10 400 python bench.py --config 3 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r04u_c3.json 2> gpurun_out/r04u_c3.err
echo c3=$?
timeout -k 10 300 python bench.py --config 1-all-rows --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04u_c1all.json 2> gpurun_out/r04u_c1all.err
echo c1all=$?
timeout -k 10 300 python bench.py --batch 65536 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r04u_c4share.json 2> gpurun_out/r04u_c4share.err
echo c4=$?
