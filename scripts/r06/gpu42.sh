# Round 6: dense1_bwd_adam_avg_kernel with the next replica's W3 slice and staging loads issued before the current
# replica's pass (apipe, MPLC_D1AVG_PIPE=1, 2 waves per SIMD; measured and not kept) against the shipped
# walk (abase, 3 waves per SIMD): model hash (bit-identity) and kernel time on the config #3 probe, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=distributed-learning-contributivity_amd/mplc/lib/libmplc_hip.so
cp $L gpurun_ab/keep.so
for v in abase apipe; do
  cp gpurun_ab/$v.so $L
  timeout -k 10 300 python scripts/model_hash.py mnist 60 1 > gpurun_out/hash_$v.log 2>&1 || { cp gpurun_ab/keep.so $L; exit 1; }
  echo "$v $(grep -h sha1 gpurun_out/hash_$v.log)"
done
cp gpurun_ab/keep.so $L
KSTATS_ROWS=10 KSTATS_W=40 AB_VARIANTS="abase apipe abase apipe" timeout -k 10 900 bash scripts/gpu_ab.sh 252 1 5 mnist > gpurun_out/r06_ab_apipe.txt 2>&1 || exit 1
grep -E "==|dense1|total" gpurun_out/r06_ab_apipe.txt
