# conv_fwd A/B (AB_VARIANTS, default: double-buffered image img2 vs new) after the MNIST GPU tests on the in-tree library
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03c1; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_cnn_gpu.py tests/test_workload_gpu.py::test_config3_round_trajectory_vs_fp64 tests/test_workload_gpu.py::test_config3_batch_invariance -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
AB_VARIANTS="${AB_VARIANTS:-new img2 new img2}" timeout -k 10 700 bash scripts/gpu_ab.sh 252 1 5
for v in ${AB_VARIANTS:-new img2 new img2}; do grep -o "evals/s.*sha1 [0-9a-f]*" gpurun_out/ab_$v/probe.log | sed "s/^/$v /"; done
