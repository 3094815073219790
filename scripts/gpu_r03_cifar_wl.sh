# CIFAR10 wave-local Winograd kernels with the next patch read one k-step ahead (new, wlns: SLP off) vs the
# committed kernels (cold, coldns: SLP off): CIFAR GPU tests on the in-tree library, then the A/B probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03wl; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_cifar_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
L=distributed-learning-contributivity_amd/mplc/lib/libmplc_hip.so
cp $L gpurun_ab/keep.so
for v in ${AB_VARIANTS:-cold new wlns coldns cold new wlns}; do
  cp gpurun_ab/$v.so $L
  D=gpurun_out/abc_$v; rm -rf $D; mkdir -p $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- python scripts/probe_train.py 120 1 6 cifar > $D/probe.log 2>&1 || { cp gpurun_ab/keep.so $L; exit 1; }
  echo "== $v"; python scripts/kstats.py $D/trace/run_kernel_stats.csv | head -12; grep -o "evals/s.*sha1 [0-9a-f]*" $D/probe.log
done
cp gpurun_ab/keep.so $L
