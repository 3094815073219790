"""Summarise a rocprofv3 kernel_stats.csv: per-kernel total ms, calls, and us per replica-step."""
import csv
import sys

path = sys.argv[1]
rs = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0  # replica-steps in the run
tot = 0.0
rows = list(csv.DictReader(open(path)))
for r in rows:
    tot += float(r["TotalDurationNs"])
import os
for r in rows[:int(os.environ.get("KSTATS_ROWS", "12"))]:
    name = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:int(os.environ.get("KSTATS_W", "40"))]
    ms = float(r["TotalDurationNs"]) / 1e6
    extra = f"{ms * 1000 / rs:8.2f} us/replica-step" if rs else ""
    print(f"{name:{int(os.environ.get('KSTATS_W', '40'))}s} {int(r['Calls']):6d} {ms:10.1f} ms {100 * float(r['TotalDurationNs']) / tot:5.1f}% {extra}")
print(f"total {tot / 1e6:.1f} ms")
