set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/r06/gpu_ab_lds.sh > gpurun_out/r06_ab_lds.txt 2>&1 && \
bash scripts/r06/gpu_pmc4_diag.sh > gpurun_out/r06_pmc4diag.txt 2>&1
