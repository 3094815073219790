# Round-end checks on one MI355X: CNN parity (incl. the ranking gate), MNIST PMC summary, and single-GPU
# emulation of rank 0 of an N-GPU config #3 run (N = 2, 4, 8) for the strong-scaling estimate.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/final
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_cnn_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_cnn.log 2>&1 || { tail -30 $O/pytest_cnn.log; exit 1; }
bash scripts/gpu_pmc.sh > $O/pmc.log 2>&1 && python scripts/pmc_summary.py gpurun_out/pmc > $O/pmc_summary.txt || exit 1
for n in 2 4 8; do
  timeout -k 10 300 python scripts/emulate_rank.py $n > $O/emulate_$n.log 2>&1 || exit 1
  tail -1 $O/emulate_$n.log
done
echo EXIT 0
