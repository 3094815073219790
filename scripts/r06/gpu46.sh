# Round 6: CIFAR dense5_fwd16 with W5 streamed in K chunks of 64 / 128 rows (ck64 / ck128, MPLC_D16_K) against 32
# (chead, the shipped form): model hash (bit-identity) and kernel time on the config #4-shaped probe, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=distributed-learning-contributivity_amd/mplc/lib/libmplc_hip.so
cp $L gpurun_ab/keep.so
for v in chead ck64 ck128; do
  cp gpurun_ab/$v.so $L
  timeout -k 10 300 python scripts/model_hash.py cifar 40 1 > gpurun_out/hash_$v.log 2>&1 || { cp gpurun_ab/keep.so $L; exit 1; }
  echo "$v $(grep -h sha1 gpurun_out/hash_$v.log)"
done
cp gpurun_ab/keep.so $L
KSTATS_ROWS=16 KSTATS_W=40 AB_VARIANTS="chead ck64 ck128 chead ck64 ck128" timeout -k 10 900 bash scripts/gpu_ab.sh 52 1 5 cifar > gpurun_out/r06_ab_d16k.txt 2>&1 || exit 1
grep -E "==|dense5_fwd|total" gpurun_out/r06_ab_d16k.txt
