# Round 6: the driver's bench command on the final tree, then the round's profiles (kernel trace + FETCH / WRITE
# passes of the config #3 leg: scripts/gpu_profile.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python bench.py > gpurun_out/r06_bench_final.json 2> gpurun_out/r06_bench_final.err || exit 1
tail -c 300 gpurun_out/r06_bench_final.json
bash scripts/gpu_profile.sh r06
