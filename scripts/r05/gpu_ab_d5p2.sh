# Round 5: CIFAR dense5_fwd with its K-chunk loads two chunks ahead (A and W5 double-buffered in registers) against
# HEAD's one chunk ahead, on the config #4-shaped probe.  Kernel totals and the probe's v(S) hash.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
KSTATS_ROWS=20 KSTATS_W=44 AB_VARIANTS="base d5p2 base d5p2" timeout -k 10 900 bash scripts/gpu_ab.sh 52 1 5 cifar 2>&1 | grep -E "==|dense5_fwd|total"
for v in base d5p2; do echo "$v $(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)"; done
