# Round 5, final tree: the -m gpu suite and smoke, then the driver's bench command.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_final_check.sh || exit 1
O=gpurun_out/r05last2; rm -rf $O; mkdir -p $O
timeout -k 10 590 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 200 $O/bench.json
