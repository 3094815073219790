# Round 4: (1) what v_mfma_f32_16x16x4f32 accumulates (scripts/probes/mfma_order), (2) the wave-local data
# gradient's ReLU' operand loaded during the last k-step (MPLC_WL_PRE_RR 0/1/2/4 tile rows; wlpm0 = the peeled
# loop alone) against pdzw (the committed library) on the CIFAR probe, bit-identity by v(S) hash, (3) config #3
# E=40 + early stopping with the stops of an epoch end applied at once (one aggregation-run rebuild, one copy per
# dtype), (4) the early-stopping / compaction / CIFAR GPU tests.  xcd0 / xcd2: the CIFAR kernels in XCD-aware
# block order (csrc/xcd.h) with MPLC_WL_PRE_RR 0 / 2.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 60 ./scripts/probes/mfma_order || exit 31
V="pdzw wlpm0 wlpm1 wlpm2 wlpm4 xcd0 xcd2 pdzw wlpm1 wlpm2 xcd0 xcd2" bash scripts/r04/gpu_ab_cifar.sh 2>&1 | grep -E "==|wino|dense5|conv_kernel|wgrad_kernel|total| v sha1"
h=$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_pdzw/probe.log)
for v in wlpm0 wlpm1 wlpm2 wlpm4 xcd0 xcd2; do [ "$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)" = "$h" ] || { echo "HASH MISMATCH $v"; exit 32; }; done
O=gpurun_out/r04es2
rm -rf $O; mkdir -p $O
timeout -k 10 500 python bench.py --epochs 40 --early-stopping --mnist-signal 0.2 --steps 1 --warmup 0 --no-cifar \
  --no-shapley-agg --no-cpu-baseline --budget-s 480 > $O/es.json 2> $O/es.err || { tail -5 $O/es.err; exit 33; }
python3 -c "
import json; d = json.loads(open('$O/es.json').read().strip().splitlines()[-1])
print('es', d['value'], d['ms_per_step'], json.dumps(d['early_stopping']))"
timeout -k 10 900 python -u -m pytest tests/test_compaction_gpu.py tests/test_cifar_gpu.py tests/test_cnn_gpu.py tests/test_history_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -4
