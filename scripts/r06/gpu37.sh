# Round 6: dense1_bwd_adam with W3's loads and stores non-temporal (nt1) vs normal (nt0), on the config #3 leg itself
# (5120 replicas; the in-stream kernel table), alternating; model hash on the MNIST probe
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=distributed-learning-contributivity_amd/mplc/lib/libmplc_hip.so
cp $L gpurun_ab/keep.so
O=gpurun_out/r06_ab_nt.txt; : > $O
for v in nt0 nt1; do
  cp gpurun_ab/$v.so $L
  timeout -k 10 300 python scripts/model_hash.py mnist 60 1 2>&1 | grep sha1 | sed "s/^/$v /" >> $O || { cp gpurun_ab/keep.so $L; exit 1; }
done
for i in 1 2; do
  for v in nt0 nt1; do
    cp gpurun_ab/$v.so $L
    timeout -k 10 400 python bench.py --leg train --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/nt_$v.json 2> gpurun_out/nt_$v.err || { cp gpurun_ab/keep.so $L; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/nt_$v.json').read().strip().splitlines()[-1]); k=d['kernels']
print('$v', d['value'], 'dense1', k['dense1_bwd_adam']['ms_avg'], k['dense1_bwd_adam']['frac'], 'dense_fwd', k['dense_fwd']['ms_avg'])" >> $O
  done
done
cp gpurun_ab/keep.so $L
cat $O
