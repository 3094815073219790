# Round 6: does config #3 gain from two HIP streams (dense1's HBM pass beside the other half's conv MFMA work)?
# Probe wall-clock evals/s, one vs two streams, alternating, at 252 and 1023 coalitions (E=1).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/r06_mnist_streams.txt; : > $O
for i in 1 2; do
  for n in 252 1023; do
    for c in 1 2; do
      MPLC_CONCURRENT_BATCHES=$c timeout -k 10 300 python scripts/probe_train.py $n 1 5 mnist 2>&1 | grep evals | sed "s/^/streams $c n $n: /" >> $O
    done
  done
done
cat $O
