"""GPU busy fraction from a rocprofv3 kernel trace: span of the trace, union of kernel intervals, and the
idle gaps between consecutive kernels (histogram).  Prints a short summary (the raw trace of a long run is
too large to keep).  python scripts/trace_busy.py <run_kernel_trace.csv>"""
import csv
import sys

iv = []
per = {}
per_grid = {}  # (kernel, grid): a kernel launched by several legs of one command (different batch shapes) apart
with open(sys.argv[1]) as f:
    rd = csv.DictReader(f)
    gcols = [c for c in rd.fieldnames if c.startswith("Grid_Size")]
    for r in rd:
        s_, e_ = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        iv.append((s_, e_))
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "")[:60]
        n, t = per.get(k, (0, 0))
        per[k] = (n + 1, t + e_ - s_)
        g = "x".join(r[c] for c in gcols)
        n, t = per_grid.get((k, g), (0, 0))
        per_grid[(k, g)] = (n + 1, t + e_ - s_)
iv.sort()
span = iv[-1][1] - iv[0][0]
busy, cur_s, cur_e = 0, iv[0][0], iv[0][1]
gaps = []
for s, e in iv[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append(s - cur_e)
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"kernels {len(iv)}  span {span / 1e9:.2f} s  busy {busy / 1e9:.2f} s ({100 * busy / span:.1f} %)")
edges = [1e3, 5e3, 1e4, 2e4, 5e4, 1e5, 1e6, 1e7, 1e12]
lo = 0
for hi in edges:
    sel = [g for g in gaps if lo <= g < hi]
    print(f"  gaps [{lo / 1e3:8.0f}, {hi / 1e3:8.0f}) us: {len(sel):7d}  total {sum(sel) / 1e9:7.2f} s")
    lo = hi
for k, (n, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:16]:
    print(f"  {k:60s} {n:8d} {t / 1e9:8.2f} s  avg {t / n / 1e3:9.1f} us")
print("by launch grid (kernel, grid size):")
for (k, g), (n, t) in sorted(per_grid.items(), key=lambda kv: -kv[1][1])[:24]:
    print(f"  {k:60s} {g:>20s} {n:8d} {t / 1e9:8.2f} s  avg {t / n / 1e3:9.1f} us")
