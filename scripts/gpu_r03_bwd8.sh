# conv_bwd_data with 8-channel stages (LDS-DMA Ur, double-buffered, one barrier per stage): parity tests on the
# in-tree library, then the A/B probe against the previous kernel (gpurun_ab/old.so, gpurun_ab/new.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03bwd
rm -rf $O; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_cnn_gpu.py tests/test_workload_gpu.py::test_config3_round_trajectory_vs_fp64 -x -q \
  -k "gradients or fedavg or independent or timer or trajectory or oracle" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
AB_VARIANTS="${AB_VARIANTS:-old new old new}" timeout -k 10 700 bash scripts/gpu_ab.sh 252 1 5
