# CIFAR10 Winograd convolutions: the CIFAR parity tests, then an A/B kernel trace (old direct implicit GEMM vs
# Winograd) on a config #4-shaped probe (80 coalitions x 5 partners of 20, E=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03cifar
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_cifar_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -25 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
AB_VARIANTS="cifar_old cifar_new cifar_new2" bash scripts/gpu_ab.sh 80 1 5 cifar
