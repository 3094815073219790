# Round 6: dense1_bwd_adam_avg_kernel (the fused W3 average: 0.37 of HBM at 2 waves per SIMD, 172 VGPRs) at 3 waves
# per SIMD (avgw3: 168 VGPRs, 2 spilled) against 2 (avgw2): model hash and kernel time on the config #3 probe
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=distributed-learning-contributivity_amd/mplc/lib/libmplc_hip.so
cp $L gpurun_ab/keep.so
for v in avgw2 avgw3; do
  cp gpurun_ab/$v.so $L
  timeout -k 10 300 python scripts/model_hash.py mnist 60 1 > gpurun_out/hash_$v.log 2>&1 || { cp gpurun_ab/keep.so $L; exit 1; }
  echo "$v $(grep -h sha1 gpurun_out/hash_$v.log)"
done
cp gpurun_ab/keep.so $L
KSTATS_ROWS=10 KSTATS_W=40 AB_VARIANTS="avgw2 avgw3 avgw2 avgw3" timeout -k 10 900 bash scripts/gpu_ab.sh 252 1 5 mnist > gpurun_out/r06_ab_avgw.txt 2>&1 || exit 1
grep -E "==|dense1|total" gpurun_out/r06_ab_avgw.txt
