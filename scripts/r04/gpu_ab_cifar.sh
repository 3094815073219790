# Round 4: CIFAR kernel A/B on a config #4-shaped probe (92 coalitions x 5 partners = 460 replicas, E=1): the
# round-3 library (d5g4) against the variants named in $V (prebuilt into gpurun_ab/); per variant the kernel trace
# totals and the v(S) hash (bit-identity).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
KSTATS_ROWS=30 KSTATS_W=64 AB_VARIANTS="${V:-d5g4 c2xil cxil cxg1s12 cxg2s12 d5g4 cxil}" bash scripts/gpu_ab.sh 92 1 5 cifar 2>&1 | grep -E "==|wino|conv|dense5|rmsprop|sha1|Total|total" | cut -c1-110
for v in ${V:-d5g4 c2xil cxil cxg1s12 cxg2s12}; do echo "$v $(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)"; done
