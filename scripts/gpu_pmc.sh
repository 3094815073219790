set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf gpurun_out/pmc; mkdir -p gpurun_out/pmc
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
K='conv_fwd|conv_bwd_data|conv_wgrad|dense1_bwd_adam|dense_fwd'
timeout -k 10 200 rocprofv3 --kernel-include-regex "$K" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc/p1 -o run --output-format csv -- python scripts/probe_train.py 64 1 5 > gpurun_out/pmc/p1.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-include-regex "$K" --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/pmc/p2 -o run --output-format csv -- python scripts/probe_train.py 64 1 5 > gpurun_out/pmc/p2.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-include-regex "$K" --pmc FETCH_SIZE -d gpurun_out/pmc/p3 -o run --output-format csv -- python scripts/probe_train.py 64 1 5 > gpurun_out/pmc/p3.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-include-regex "$K" --pmc WRITE_SIZE -d gpurun_out/pmc/p4 -o run --output-format csv -- python scripts/probe_train.py 64 1 5 > gpurun_out/pmc/p4.log 2>&1
echo EXIT $?
