# Round 6: CIFAR lockstep batches on 1-4 HIP streams (probe wall clock, config #4-shaped 52 x 5 and 104 x 5), alternating
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/r06_cifar_streams.txt; : > $O
for i in 1 2; do
  for n in 52 104; do
    for c in 1 2 3 4; do
      MPLC_CONCURRENT_BATCHES=$c timeout -k 10 300 python scripts/probe_train.py $n 1 5 cifar 2>&1 | grep evals | sed "s/^/streams $c n $n: /" >> $O
    done
  done
done
cat $O
