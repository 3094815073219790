# Round 5: conv_bwd_data A/B on the config #3-shaped MNIST probe: base (HEAD), u (un-pool in two LDS writes per
# window: clear the previous argmax pixel, write the new one), w (conv1 weights for the epilogue loaded up front),
# uw (both).  Kernel totals and the probe's v(S) hash (bit-identity).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
KSTATS_ROWS=6 KSTATS_W=40 AB_VARIANTS="base u w uw base u w uw" timeout -k 10 900 bash scripts/gpu_ab.sh 252 1 5 2>&1 | grep -E "==|conv_bwd|total"
for v in base u w uw; do echo "$v $(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)"; done
