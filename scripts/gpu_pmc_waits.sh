# Wave-state PMC passes (separate runs, per the microarch guide) for the MNIST training kernels on a probe run:
# where do the waves' cycles go (parked at s_waitcnt / barrier, issue-stalled, issuing)?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmcw
rm -rf $O; mkdir -p $O
K='conv_fwd|conv_bwd_data|conv_wgrad'
timeout -k 10 200 rocprofv3 --kernel-include-regex "$K" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_BUSY_CYCLES -d $O/p1 -o run --output-format csv -- python scripts/probe_train.py 64 1 5 > $O/p1.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-include-regex "$K" --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $O/p2 -o run --output-format csv -- python scripts/probe_train.py 64 1 5 > $O/p2.log 2>&1
echo EXIT $?
python - <<'PY'
import collections, csv, glob
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob("gpurun_out/pmcw/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in tot.items():
    wc = v["SQ_WAVE_CYCLES"] + 1e-9
    print(f"{k:24s} waves {v['SQ_WAVES']:.0f}  parked(waitcnt/barrier) {v['SQ_WAIT_ANY']/wc:.2f}  issue-stall {v['SQ_WAIT_INST_ANY']/wc:.2f} "
          f"(lds {v['SQ_WAIT_INST_LDS']/wc:.2f})  issuing {v['SQ_ACTIVE_INST_ANY']/wc:.2f}  "
          f"mfma_busy {v['SQ_VALU_MFMA_BUSY_CYCLES']/max(1, v['GRBM_GUI_ACTIVE']/8*1024):.2f}  "
          f"lds/mfma {v['SQ_INSTS_LDS']/(v['SQ_INSTS_MFMA']+1e-9):.2f}  vmem/mfma {v['SQ_INSTS_VMEM_RD']/(v['SQ_INSTS_MFMA']+1e-9):.2f}  "
          f"salu/mfma {v['SQ_INSTS_SALU']/(v['SQ_INSTS_MFMA']+1e-9):.2f}  conflict {v['SQ_LDS_BANK_CONFLICT']/(v['SQ_LDS_IDX_ACTIVE']+1):.2f}")
PY
