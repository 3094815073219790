"""The largest idle gaps of a rocprofv3 kernel trace with the kernels either side of each (where host time goes
between launches).  python scripts/gaps_top.py <run_kernel_trace.csv> [n]"""
import csv
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                     r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:40]))
rows.sort()
gaps = []
end, prev = rows[0][1], rows[0][2]
for s, e, k in rows[1:]:
    if s > end:
        gaps.append((s - end, prev, k, s))
    if e > end:
        end, prev = e, k
t0 = rows[0][0]
gaps.sort(reverse=True)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
print(f"span {(rows[-1][1] - t0) / 1e9:.2f} s, {len(rows)} kernels, gaps >= 1 ms: "
      f"{sum(g for g, *_ in gaps if g >= 1e6) / 1e9:.2f} s in {sum(1 for g, *_ in gaps if g >= 1e6)}")
for g, a, b, s in gaps[:n]:
    print(f"{g / 1e6:9.2f} ms at {(s - t0) / 1e9:7.2f} s  after {a:40s} before {b}")
