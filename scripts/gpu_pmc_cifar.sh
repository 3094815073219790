# PMC passes (separate runs, per MI355X_MICROARCH.md) over the CIFAR probe's training kernels (52 coalitions x 5
# partners: 260 replicas per launch, config #4's TMCS average), then scripts/pmc_summary.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc_cifar
rm -rf $O; mkdir -p $O
K='conv_kernel|wgrad_kernel|wino_kernel|wino_wl_kernel|dense5'
timeout -k 10 200 rocprofv3 --kernel-include-regex "$K" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/p1 -o run --output-format csv -- python scripts/probe_train.py 52 1 5 cifar > $O/p1.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-include-regex "$K" --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $O/p2 -o run --output-format csv -- python scripts/probe_train.py 52 1 5 cifar > $O/p2.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-include-regex "$K" --pmc FETCH_SIZE -d $O/p3 -o run --output-format csv -- python scripts/probe_train.py 52 1 5 cifar > $O/p3.log 2>&1
rc=$?
python scripts/pmc_summary.py $O > $O/summary.txt 2>&1
cat $O/summary.txt
echo EXIT $rc
exit $rc
