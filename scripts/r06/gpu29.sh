# Round 6: the driver's bench command with config #4's kernel timer moved into a profile pass (the warm-up step)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 800 python bench.py > gpurun_out/r06_bench_prof.json 2> gpurun_out/r06_bench_prof.err || exit 1
tail -c 400 gpurun_out/r06_bench_prof.json
