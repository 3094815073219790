"""Kernels of a rocprofv3 trace in a time window (seconds from the first kernel), with the idle gap before each:
python scripts/kernels_window.py <run_kernel_trace.csv> <t_from> <t_to>"""
import csv
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                     r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:70]))
rows.sort()
t0 = rows[0][0]
a, b = float(sys.argv[2]), float(sys.argv[3])
prev_end = None
for s, e, k in rows:
    ts = (s - t0) / 1e9
    if a <= ts <= b:
        gap = (s - prev_end) / 1e6 if prev_end is not None else 0.0
        print(f"{ts:9.4f} s  gap {gap:8.2f} ms  dur {(e - s) / 1e3:9.1f} us  {k}")
    prev_end = e if prev_end is None else max(prev_end, e)
print(f"last kernel at {(rows[-1][1] - t0) / 1e9:.3f} s")
