"""Idle gaps of a rocprofv3 kernel trace with the kernels on either side: the largest gaps and the gap time
summed by (previous kernel -> next kernel) pair.  python scripts/gaps_context.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                     r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:28]))
rows.sort()
cur_e, prev = rows[0][1], rows[0][2]
pairs = collections.defaultdict(lambda: [0, 0])
big = []
for s, e, k in rows[1:]:
    if s > cur_e:
        g = s - cur_e
        pairs[(prev, k)][0] += 1
        pairs[(prev, k)][1] += g
        big.append((g, prev, k))
    if e > cur_e:
        cur_e, prev = e, k
span = rows[-1][1] - rows[0][0]
tot = sum(v[1] for v in pairs.values())
print(f"span {span / 1e9:.2f} s, idle {tot / 1e9:.3f} s in {sum(v[0] for v in pairs.values())} gaps")
for (a, b), (n, t) in sorted(pairs.items(), key=lambda kv: -kv[1][1])[:14]:
    print(f"  {a:28s} -> {b:28s} {n:6d} gaps {t / 1e6:9.1f} ms  avg {t / n / 1e3:8.1f} us")
print("largest:")
for g, a, b in sorted(big, reverse=True)[:10]:
    print(f"  {g / 1e6:8.1f} ms  {a} -> {b}")
