# Round 6: where MNIST conv_bwd_data's time goes - timing-experiment builds (garbage results: MPLC_EXPERIMENT) with
# its epilogue, its whole staging, the Ur staging or the dZ2 un-pool compiled out, against the product build (base)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
KSTATS_ROWS=8 KSTATS_W=40 AB_VARIANTS="base xNOEPI xNOSTAGE xNOSTAGE_UR xNOSTAGE_DZ base" timeout -k 10 900 bash scripts/gpu_ab.sh 252 1 5 mnist > gpurun_out/r06_bwd_breakdown.txt 2>&1 || exit 1
grep -E "==|conv_bwd" gpurun_out/r06_bwd_breakdown.txt
