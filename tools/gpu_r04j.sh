set -o pipefail
cd $GRAFT_REPO_ROOT
for S in 4 8; do
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --sub-batches $S > gpurun_out/r04j_bench_s$S.json 2> gpurun_out/r04j_bench_s$S.err
echo s${S}_rc=$?
done
timeout -k 10 900 bash tools/profile_round.sh gpurun_out/r04j_prof > gpurun_out/r04j_prof.log 2>&1
echo prof_rc=$?
