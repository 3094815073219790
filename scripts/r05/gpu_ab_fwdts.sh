# Round 5: MNIST conv_fwd with the T-plane tile stride 68 (C2 + 4: a half-wave's two tile quads on opposite bank
# halves) against HEAD's 65, on the config #3-shaped probe.  Kernel totals and the probe's v(S) hash.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
KSTATS_ROWS=6 KSTATS_W=40 AB_VARIANTS="base ts base ts" timeout -k 10 900 bash scripts/gpu_ab.sh 252 1 5 2>&1 | grep -E "==|conv_fwd|total"
for v in base ts; do echo "$v $(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)"; done
