set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bfgs.py > gpurun_out/r04l_bfgs_tests.log 2>&1
echo tests_rc=$?
