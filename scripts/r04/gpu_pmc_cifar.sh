# Round 4: PMC passes (separate runs, MI355X_MICROARCH.md) over the CIFAR10 training kernels on a config #4-shaped
# probe of TMCS-like lockstep batches (92 coalitions x 5 partners = 460 replicas, E=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04pmc_cifar
rm -rf $O; mkdir -p $O
K='wino|wgrad_kernel|conv_kernel|dense5|rmsprop'
P="python scripts/probe_train.py 92 1 5 cifar"
timeout -s KILL 200 rocprofv3 --kernel-include-regex "$K" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/p1 -o run --output-format csv -- $P > $O/p1.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --kernel-include-regex "$K" --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS -d $O/p2 -o run --output-format csv -- $P > $O/p2.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --kernel-include-regex "$K" --pmc FETCH_SIZE -d $O/p3 -o run --output-format csv -- $P > $O/p3.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $P > $O/trace.log 2>&1
rc=$?
python scripts/pmc_summary.py $O > $O/summary.txt 2>&1; cat $O/summary.txt
python scripts/kstats.py $O/trace/run_kernel_stats.csv | head -24
exit $rc
