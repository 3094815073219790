# Round 6: config #3 at the reference's defaults (E=40 + early stopping, learnable synthetic MNIST) on the final tree
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
HB=$!
timeout -k 10 700 python bench.py --epochs 40 --early-stopping --mnist-signal 0.2 --steps 1 --warmup 0 --no-cifar \
  --no-titanic --no-tutorial --no-shapley-agg --no-cpu-baseline --budget-s 640 > gpurun_out/r06_es_e40.json 2> gpurun_out/r06_es_e40.err
rc=$?
kill $HB
tail -c 300 gpurun_out/r06_es_e40.json
exit $rc
