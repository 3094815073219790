# Multi-rank rehearsal on a 1-GPU box, both launch paths: `bench.py --gpus 2` launching its own ranks, and the
# driver's torchrun shape (gloo: the two ranks share cuda:0; the 8-GPU scaling runs use nccl = RCCL).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/rehearse_r05; rm -rf $O; mkdir -p $O
MPLC_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 1 --warmup 1 --budget-s 240 --no-cpu-baseline > $O/self.json 2> $O/self.err
rc=$?; echo "self-launch rc $rc"; tail -c 600 $O/self.json; [ $rc -eq 0 ] || { tail -5 $O/self.err; exit $rc; }
MPLC_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 1 --warmup 1 --budget-s 240 --no-cpu-baseline \
  > $O/torchrun.json 2> $O/torchrun.err
rc=$?; echo "torchrun rc $rc"; tail -c 600 $O/torchrun.json; exit $rc
