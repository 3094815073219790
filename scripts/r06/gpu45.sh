# Round 6: conv_bwd_data with the next channel quarter's Ur loads issued in the last k-step of the current quarter
# (bwdur, MPLC_BWD_UR_AHEAD) against HEAD's kernel (bhead): model hash (bit-identity) and kernel time on the config #3 probe
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=distributed-learning-contributivity_amd/mplc/lib/libmplc_hip.so
cp $L gpurun_ab/keep.so
for v in bhead bwdur; do
  cp gpurun_ab/$v.so $L
  timeout -k 10 300 python scripts/model_hash.py mnist 60 1 > gpurun_out/hash_$v.log 2>&1 || { cp gpurun_ab/keep.so $L; exit 1; }
  echo "$v $(grep -h sha1 gpurun_out/hash_$v.log)"
done
cp gpurun_ab/keep.so $L
KSTATS_ROWS=10 KSTATS_W=40 AB_VARIANTS="bhead bwdur bhead bwdur" timeout -k 10 900 bash scripts/gpu_ab.sh 252 1 5 mnist > gpurun_out/r06_ab_bwdur.txt 2>&1 || exit 1
grep -E "==|dense1|total" gpurun_out/r06_ab_bwdur.txt
