set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/r06/gpu_ab_rsgn.sh > gpurun_out/r06_ab_rsgn.txt 2>&1 && \
timeout -k 10 900 python -u scripts/probe_ranking.py --seeds 3 > gpurun_out/r06_probe_ranking2.log 2>&1
