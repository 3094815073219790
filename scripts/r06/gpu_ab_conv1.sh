# Round 6: CIFAR conv1 forward with the output channels as the MFMA's M rows (16-B stores, the
# bias once per block) - conv1_fwd_kernel - against conv_kernel<32, 32, 3, 32, 1, 8, 4, 2, EPI_FWD>: bit-identity
# (model hashes) and kernel time on the config #4-shaped probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=distributed-learning-contributivity_amd/mplc/lib/libmplc_hip.so
cp $L gpurun_ab/keep.so
for v in fuse c1; do
  cp gpurun_ab/$v.so $L
  timeout -k 10 300 python scripts/model_hash.py cifar 40 1 > gpurun_out/hash_cifar_$v.log 2>&1 || { cp gpurun_ab/keep.so $L; exit 1; }
  echo "$v $(grep -h sha1 gpurun_out/hash_cifar_$v.log)"
done
cp gpurun_ab/keep.so $L
KSTATS_ROWS=18 KSTATS_W=44 AB_VARIANTS="fuse c1 fuse c1" timeout -k 10 600 bash scripts/gpu_ab.sh 52 1 5 cifar 2>&1 | grep -E "==|conv_kernel|conv1_fwd|total"
