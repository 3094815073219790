# Round 6: CIFAR LDS layouts - dense5_fwd16's A tile row stride DF_K + 2 (d5s) and the Winograd
# kernels' staged row stride padded to TXT (mod 16) (wpad: a half-wave's 16 tiles x 2 channels on the 32 banks
# once) - against the conv1 build (c1): bit-identity (model hashes) and kernel time on the config #4-shaped probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=distributed-learning-contributivity_amd/mplc/lib/libmplc_hip.so
cp $L gpurun_ab/keep.so
for v in c1 d5s wpad; do
  cp gpurun_ab/$v.so $L
  timeout -k 10 300 python scripts/model_hash.py cifar 40 1 > gpurun_out/hash_cifar_$v.log 2>&1 || { cp gpurun_ab/keep.so $L; exit 1; }
  echo "$v $(grep -h sha1 gpurun_out/hash_cifar_$v.log)"
done
cp gpurun_ab/keep.so $L
KSTATS_ROWS=18 KSTATS_W=44 AB_VARIANTS="c1 wpad c1 wpad" timeout -k 10 600 bash scripts/gpu_ab.sh 52 1 5 cifar 2>&1 | grep -E "==|wino|dense5|conv1_fwd|total"
