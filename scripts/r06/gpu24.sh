# Round 6 vs round 5 on the SAME box (box-to-box spread is ~8 %): the round-5 tree (607486a, its own library built
# from its sources: gpurun_ab/t605) and HEAD, probe wall-clock evals/s alternating, config #3-shaped (252 coalitions
# x 5 partners, MNIST) and config #4-shaped (52 x 5, CIFAR10; HEAD with its default two streams and with one).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/r06_vs_r05.txt; : > $O
for i in 1 2; do
  for w in mnist cifar; do
    a="252 1 5 mnist"; [ $w = cifar ] && a="52 1 5 cifar"
    (cd gpurun_ab/t605 && timeout -k 10 300 python scripts/probe_train.py $a) 2>&1 | grep evals | sed "s/^/r05 $w: /" >> $O
    timeout -k 10 300 python scripts/probe_train.py $a 2>&1 | grep evals | sed "s/^/r06 $w: /" >> $O
    [ $w = cifar ] && MPLC_CONCURRENT_BATCHES=1 timeout -k 10 300 python scripts/probe_train.py $a 2>&1 | grep evals | sed "s/^/r06 $w 1-stream: /" >> $O
  done
done
cat $O
bash scripts/gpu_profile.sh r06 pmc
