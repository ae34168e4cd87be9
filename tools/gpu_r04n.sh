set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/mlp_check.py > gpurun_out/r04n_mlp_check.log 2>&1
echo check_rc=$?
timeout -k 10 400 python bench.py --config 2 --steps 6 --warmup 2 --no-cpu-baseline --sub-batches 1 > gpurun_out/r04n_bench_c2.json 2> gpurun_out/r04n_bench_c2.err
echo c2_rc=$?
MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_vmlp0/libmpcc_engine.so timeout -k 10 400 python bench.py --config 2 --steps 6 --warmup 2 --no-cpu-baseline --sub-batches 1 > gpurun_out/r04n_bench_c2_pf0.json 2> gpurun_out/r04n_bench_c2_pf0.err
echo c2pf0_rc=$?
