# Round 6: the conv2..conv4 weight-gradient kernels (MNIST conv_wgrad, CIFAR wino_wgrad) as ONE loop with the wave's
# transform row as data (runtime +-1 / 0 factors in SGPRs) instead of per-wave compiled copies whose barriers sat in a
# wave-uniform switch.  Bit-identity (model hashes) and kernel time, base vs rsgn.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=distributed-learning-contributivity_amd/mplc/lib/libmplc_hip.so
cp $L gpurun_ab/keep.so
for v in base rsgn; do
  cp gpurun_ab/$v.so $L
  timeout -k 10 300 python scripts/model_hash.py mnist 60 1 > gpurun_out/hash_mnist_$v.log 2>&1 || { cp gpurun_ab/keep.so $L; exit 1; }
  timeout -k 10 300 python scripts/model_hash.py cifar 40 1 > gpurun_out/hash_cifar_$v.log 2>&1 || { cp gpurun_ab/keep.so $L; exit 1; }
  echo "$v $(grep -h sha1 gpurun_out/hash_mnist_$v.log gpurun_out/hash_cifar_$v.log | tr '\n' ' ')"
done
cp gpurun_ab/keep.so $L
KSTATS_ROWS=12 KSTATS_W=44 AB_VARIANTS="base rsgn base rsgn" timeout -k 10 600 bash scripts/gpu_ab.sh 252 1 5 mnist 2>&1 | grep -E "==|conv_wgrad|total"
KSTATS_ROWS=16 KSTATS_W=44 AB_VARIANTS="base rsgn base rsgn" timeout -k 10 600 bash scripts/gpu_ab.sh 52 1 5 cifar 2>&1 | grep -E "==|wino_wgrad|total"
