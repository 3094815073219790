# PMC passes (one counter group per run) over one probe shape for the given kernels:
#   bash scripts/gpu_pmc_probe.sh <out-name> <kernel regex> <probe args...>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
NAME=$1; K=$2; shift 2
O=gpurun_out/pmc_$NAME
rm -rf $O; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-include-regex "$K" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/p1 -o run --output-format csv -- python scripts/probe_train.py "$@" > $O/p1.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-include-regex "$K" --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS -d $O/p2 -o run --output-format csv -- python scripts/probe_train.py "$@" > $O/p2.log 2>&1
rc=$?
python scripts/pmc_summary.py $O
exit $rc
