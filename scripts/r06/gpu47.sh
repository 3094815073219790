# Round 6: the evaluation's dense_fwd launches (several 32-row tiles per model) with XCD-aware block order (excd)
# against the plain order (ehead): model hash and the eval launches' time on the config #3 probe, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=distributed-learning-contributivity_amd/mplc/lib/libmplc_hip.so
cp $L gpurun_ab/keep.so
for v in ehead excd; do
  cp gpurun_ab/$v.so $L
  timeout -k 10 300 python scripts/model_hash.py mnist 60 1 > gpurun_out/hash_$v.log 2>&1 || { cp gpurun_ab/keep.so $L; exit 1; }
  echo "$v $(grep -h sha1 gpurun_out/hash_$v.log)"
done
cp gpurun_ab/keep.so $L
KSTATS_ROWS=10 KSTATS_W=40 AB_VARIANTS="ehead excd ehead excd" timeout -k 10 900 bash scripts/gpu_ab.sh 252 1 5 mnist > gpurun_out/r06_ab_excd.txt 2>&1 || exit 1
grep -E "==|dense_fwd|total" gpurun_out/r06_ab_excd.txt
python3 - <<'PY'
import csv
for v in ["ehead", "excd"]:
    tot = {}
    for r in csv.DictReader(open(f"gpurun_out/ab_{v}/trace/run_kernel_trace.csv")):
        if "dense_fwd_kernel" in r["Kernel_Name"]:
            g = int(r["Grid_Size_X"]) if "Grid_Size_X" in r else int(r["Grid_Size"])
            k = "eval (grid x %d)" % g if g > 256 else "train"
            n, t = tot.get(k, (0, 0))
            tot[k] = (n + 1, t + int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print(v, {k: (n, round(t / 1e6, 2)) for k, (n, t) in tot.items()})
PY
