# Round 5: conv_wgrad in its own translation unit (conv_fwd without spills), barrier-free per-wave k-steps, the
# W1-in-LDS switch removed: the round-4 library (old) vs the new one (new) on the config #3-shaped MNIST probe,
# kernel totals and the probe's v(S) hash (bit-identity).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
KSTATS_ROWS=10 KSTATS_W=40 AB_VARIANTS="old new2 old new2" timeout -k 10 900 bash scripts/gpu_ab.sh 252 1 5 2>&1 | grep -E "==|conv|dense|total|Total"
for v in old new2; do echo "$v $(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)"; done
