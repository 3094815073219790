# Round 6: CIFAR conv2 wave-local Winograd kernels with 2 tile rows per band (bty2: 8 bands of 2 waves; 8 with 8 rows was slower) - the halo
# rows staged once per 8 tile rows instead of per 4 - counter traffic 1.30x / 1.20x compulsory with 4) against bty4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=distributed-learning-contributivity_amd/mplc/lib/libmplc_hip.so
cp $L gpurun_ab/keep.so
for v in bty4 bty2; do
  cp gpurun_ab/$v.so $L
  timeout -k 10 300 python scripts/model_hash.py cifar 40 1 > gpurun_out/hash_$v.log 2>&1 || { cp gpurun_ab/keep.so $L; exit 1; }
  echo "$v $(grep -h sha1 gpurun_out/hash_$v.log)"
done
cp gpurun_ab/keep.so $L
KSTATS_ROWS=16 KSTATS_W=44 AB_VARIANTS="bty4 bty2 bty4 bty2" timeout -k 10 900 bash scripts/gpu_ab.sh 52 1 5 cifar > gpurun_out/r06_ab_bty.txt 2>&1 || exit 1
grep -E "==|wino_wl|total" gpurun_out/r06_ab_bty.txt
for v in bty4 bty2; do cp gpurun_ab/$v.so $L; MPLC_CONCURRENT_BATCHES=2 timeout -k 10 300 python scripts/probe_train.py 52 1 5 cifar 2>&1 | grep evals | sed "s/^/$v: /"; done
cp gpurun_ab/keep.so $L
