"""Summarise PMC passes (rocprofv3 --pmc, one directory per pass) per kernel: MFMA-pipe busy fraction,
VALU/MFMA instruction ratio,
LDS bank-conflict share, wait share, VMEM reads per MFMA, FETCH bytes (x2 gfx950 correction).
python scripts/pmc_summary.py <dir with p1 p2 p3 ...>"""
import collections
import csv
import glob
import sys

tot = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{sys.argv[1]}/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
print(f"{'kernel':44s} {'mfma_busy':>9s} {'valu/mfma':>9s} {'lds_conf':>8s} {'wait/act':>8s} {'vmem/mfma':>9s} {'fetch GB':>9s}")
for k, v in tot.items():
    mf = v["SQ_INSTS_MFMA"] + 1e-9
    # MFMA pipe utilisation: busy cycles over all 1024 SIMDs x the kernel's cycles (GRBM_GUI_ACTIVE sums the
    # 8 XCDs, MI355X_MICROARCH.md)
    busy = v["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1.0, v["GRBM_GUI_ACTIVE"] / 8 * 1024)
    if v["SQ_INSTS_MFMA"] > 0:
        per = f"{v['SQ_INSTS_VALU'] / mf:9.2f}"
        vm = f"{v['SQ_INSTS_VMEM_RD'] / mf:9.2f}"
    else:  # no matrix instructions (HBM-bound kernels): ratios per MFMA are undefined
        per, vm = f"{'-':>9s}", f"{'-':>9s}"
    print(f"{k[:44]:44s} {busy:9.3f} {per} {v['SQ_LDS_BANK_CONFLICT'] / (v['SQ_LDS_IDX_ACTIVE'] + 1):8.3f} "
          f"{v['SQ_WAIT_INST_ANY'] / (v['SQ_ACTIVE_INST_ANY'] + 1):8.2f} {vm} "
          f"{2 * v['FETCH_SIZE'] / 1024 / 1024:9.2f}")

# extra view: where the waves spend their cycles (SQ_WAVE_CYCLES = WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY)
print(f"\n{'kernel':44s} {'waves':>8s} {'wait_any':>8s} {'wait_ins':>8s} {'active':>8s} {'lds/mfma':>8s} {'ldswait':>8s} "
      f"{'valu_use':>8s}")
for k, v in tot.items():
    wc = v["SQ_WAVE_CYCLES"] + 1e-9
    mf = v["SQ_INSTS_MFMA"] + 1e-9
    print(f"{k[:44]:44s} {v['SQ_WAVES']:8.0f} {v['SQ_WAIT_ANY'] / wc:8.3f} {v['SQ_WAIT_INST_ANY'] / wc:8.3f} "
          f"{v['SQ_ACTIVE_INST_ANY'] / wc:8.3f} {(v['SQ_INSTS_LDS'] / mf if v['SQ_INSTS_MFMA'] > 0 else float('nan')):8.2f} "
          f"{v['SQ_WAIT_INST_LDS'] / wc:8.3f} "
          # VALU pipe use: 4 cycles per wave64 VALU instruction over all SIMDs' cycles (an estimate: packed and
          # transcendental ops differ)
          f"{4 * v['SQ_INSTS_VALU'] / max(1.0, v['GRBM_GUI_ACTIVE'] / 8 * 1024):8.3f}")
