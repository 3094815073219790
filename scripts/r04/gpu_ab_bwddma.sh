# Round 4: conv_bwd_data in the LDS-DMA form (MPLC_BWD_DMA) against the current kernel on the config #3-shaped
# probe (252 coalitions x 5 partners, E=1): kernel trace totals and the v(S) hash (bit-identity expected).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
KSTATS_ROWS=8 KSTATS_W=40 AB_VARIANTS="${V:-cur bwddma cur bwddma}" timeout -k 10 900 bash scripts/gpu_ab.sh 252 1 5 2>&1 | grep -E "==|conv_bwd|total"
for v in ${V:-cur bwddma}; do echo "$v $(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)"; done
