# Round 6: MNIST conv_bwd_data with its staged dZ2 row stride padded to 13 (mod 16) (bwdpad: conflict-free patch
# reads) against the final build (wst): model hash and kernel time on the config #3-shaped probe
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=distributed-learning-contributivity_amd/mplc/lib/libmplc_hip.so
cp $L gpurun_ab/keep.so
for v in wst bwdpad; do
  cp gpurun_ab/$v.so $L
  timeout -k 10 300 python scripts/model_hash.py mnist 60 1 > gpurun_out/hash_$v.log 2>&1 || { cp gpurun_ab/keep.so $L; exit 1; }
  echo "$v $(grep -h sha1 gpurun_out/hash_$v.log)"
done
cp gpurun_ab/keep.so $L
KSTATS_ROWS=10 KSTATS_W=40 AB_VARIANTS="wst bwdpad wst bwdpad" timeout -k 10 900 bash scripts/gpu_ab.sh 252 1 5 mnist > gpurun_out/r06_ab_bwdpad.txt 2>&1 || exit 1
grep -E "==|conv_bwd|total" gpurun_out/r06_ab_bwdpad.txt
