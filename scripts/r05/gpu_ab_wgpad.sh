# Round 5: CIFAR Winograd weight gradients with the LDS channel strides padded to +8 (adjacent tiles 16 banks
# apart) against HEAD, on the config #4-shaped probe (52 coalitions x 5 partners = 260 replicas).  Kernel totals and
# the probe's v(S) hash (bit-identity).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
KSTATS_ROWS=16 KSTATS_W=44 AB_VARIANTS="base pad base pad" timeout -k 10 900 bash scripts/gpu_ab.sh 52 1 5 cifar 2>&1 | grep -E "==|wgrad|total"
for v in base pad; do echo "$v $(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)"; done
