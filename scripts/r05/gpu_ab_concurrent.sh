# Round 5: lockstep batches over two HIP streams (MPLC_CONCURRENT_BATCHES=2) against one stream, on the config
# #4-shaped CIFAR probe (52 coalitions x 5 partners) and the config #3-shaped MNIST probe: wall time of the probe's
# timed evaluate and v(S) hashes (bit-identity expected); then the GPU bit-identity test.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab_conc; rm -rf $O; mkdir -p $O
for shape in "52 1 5 cifar" "252 1 5"; do
  for v in 1 2 1 2; do
    MPLC_CONCURRENT_BATCHES=$v timeout -k 10 300 python scripts/probe_train.py $shape > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
    echo "$shape streams=$v: $(grep -h 'v sha1' $O/p.log)"
  done
done
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_concurrent_gpu.py 2>&1 | tail -4
