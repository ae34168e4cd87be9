set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 bash tools/profile_round.sh gpurun_out/r04s_prof > gpurun_out/r04s_prof.log 2>&1
echo prof_rc=$?
