# Kernel iteration on one MI355X: CNN parity tests, then a kernel-trace profile of a 1260-replica probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/iter
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_cnn_gpu.py -x -q > $O/pytest.log 2>&1
rc=$?
echo "pytest rc $rc" >> $O/pytest.log
if [ $rc -ne 0 ]; then echo "pytest failed rc $rc"; tail -30 $O/pytest.log; exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python scripts/probe_train.py 252 1 5 > $O/probe.log 2>&1
echo EXIT $?
