# Round 5, last: the driver's bench command on the final tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05last; rm -rf $O; mkdir -p $O
timeout -k 10 590 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 300 $O/bench.json
