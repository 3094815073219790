# dense1_bwd_adam on MFMA (d1m: 3 waves/SIMD, d1m4: held to 128 VGPRs) vs the FMA-loop kernel (new): A/B probe,
# then the MNIST numerics tests with d1m4 in place of the in-tree library (restored after).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
AB_VARIANTS="new d1m d1m4 new d1m4" timeout -k 10 800 bash scripts/gpu_ab.sh 252 1 5 || exit 1
for v in new d1m d1m4; do grep -o "evals/s.*sha1 [0-9a-f]*" gpurun_out/ab_$v/probe.log | sed "s/^/$v /"; done
L=distributed-learning-contributivity_amd/mplc/lib/libmplc_hip.so
O=gpurun_out/r03d1m; rm -rf $O; mkdir -p $O
cp $L gpurun_ab/keep.so; cp gpurun_ab/d1m4.so $L
timeout -k 10 500 python -u -m pytest tests/test_cnn_gpu.py tests/test_workload_gpu.py::test_config3_round_trajectory_vs_fp64 tests/test_workload_gpu.py::test_config3_batch_invariance -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; cp gpurun_ab/keep.so $L; tail -3 $O/pytest.log; exit $rc
