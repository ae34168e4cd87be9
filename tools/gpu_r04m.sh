set -o pipefail
cd $GRAFT_REPO_ROOT
for n in 6 12; do
MPCC_ORACLE_IPM_DEBUG=1 MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_vtrace/libmpcc_engine.so timeout -k 10 200 python tools/lr_debug.py $n > gpurun_out/r04m_lr$n.log 2>&1
echo rc=$?
done
