# Round 5 call A: conv_bwd_data A/B (scripts/r05/gpu_ab_bwd.sh), then the config #4 planner budgets
# (scripts/r05/gpu_plan.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/r05/gpu_ab_bwd.sh && bash scripts/r05/gpu_plan.sh
