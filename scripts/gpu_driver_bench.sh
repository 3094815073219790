# The driver's exact round-end bench command (N=1), timed like the driver does, plus the GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/driver_bench
rm -rf $O; mkdir -p $O
s=$(date +%s)
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?
echo "bench rc $rc wall $(( $(date +%s) - s ))s" | tee $O/wall.txt
tail -c 3000 $O/bench.json
exit $rc
