set -o pipefail
cd $GRAFT_REPO_ROOT
KERNEL=k_mlp_env timeout -k 10 1000 bash tools/profile_round.sh gpurun_out/r04o_prof_c2 --config 2 --sub-batches 1 > gpurun_out/r04o_prof.log 2>&1
echo prof_rc=$?
