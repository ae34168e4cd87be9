set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/mlp_check.py > gpurun_out/r04v_mlp_check.log 2>&1
echo check=$?
MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_vmlpprof/libmpcc_engine.so timeout -k 10 200 python tools/mlp_prof.py > gpurun_out/r04v_mlp_prof.json 2>&1
echo mlp=$?
timeout -k 10 400 python bench.py --config 2 --steps 6 --warmup 2 --no-cpu-baseline --sub-batches 1 > gpurun_out/r04v_c2s1.json 2> gpurun_out/r04v_c2s1.err
echo c2=$?
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_mobile.py tests/test_wrapper.py tests/test_sqp_restate.py > gpurun_out/r04v_tests.log 2>&1
echo tests=$?
