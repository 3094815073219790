# Rehearsal of the multi-rank bench path on a 1-GPU box: 2 ranks (gloo, both on cuda:0) run the driver's
# N=2 command shape (LPT coalition shards, one all_reduce of v(S), max-over-ranks timing, range-sharded N=28
# aggregation).  The N=2..8 scaling runs themselves use nccl (RCCL) on an 8-GPU node.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/rehearse_n2
rm -rf $O; mkdir -p $O
MPLC_DIST_BACKEND=gloo timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --budget-s 300 \
  > $O/bench.json 2> $O/bench.err
rc=$?
echo "rc $rc"
tail -c 1500 $O/bench.json
grep -v "^\[W" $O/bench.err | tail -5
exit $rc
