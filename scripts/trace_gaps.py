"""Where a run's GPU time goes, from a rocprofv3 kernel_trace.csv: the span from the first kernel's start to the
last kernel's end, the busy time (union of kernel intervals), the idle time between kernels, the largest gaps
with the kernels on either side, and idle time summed by the kernel that follows the gap (what the GPU waited
for).  usage: python scripts/trace_gaps.py run_kernel_trace.csv [top]"""
import collections
import csv
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0][:60]


def main(path, top=15):
    ev = []
    with open(path) as f:
        for r in csv.DictReader(f):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    ev.sort()
    t0, t_end = ev[0][0], max(e[1] for e in ev)
    busy, cur_s, cur_e = 0, ev[0][0], ev[0][1]
    gaps = []
    prev = ev[0][2]
    for s, e, n in ev[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev, n, cur_e - t0))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev = n
    busy += cur_e - cur_s
    span = t_end - t0
    idle = span - busy
    print(f"kernels {len(ev)}  span {span / 1e9:.3f} s  busy {busy / 1e9:.3f} s  idle {idle / 1e9:.3f} s "
          f"({100.0 * idle / span:.1f} %)")
    by_next = collections.Counter()
    n_next = collections.Counter()
    for g, p, n, _ in gaps:
        by_next[n] += g
        n_next[n] += 1
    print("idle by the kernel after the gap:")
    for n, g in by_next.most_common(top):
        print(f"  {g / 1e9:8.3f} s  {n_next[n]:7d} gaps  {g / 1e3 / n_next[n]:9.1f} us avg  {n}")
    print("largest gaps:")
    for g, p, n, at in sorted(gaps, reverse=True)[:top]:
        print(f"  {g / 1e6:9.2f} ms at {at / 1e9:8.3f} s  {p} -> {n}")
    hist = collections.Counter()
    for g, *_ in gaps:
        b = "<10us" if g < 1e4 else "<100us" if g < 1e5 else "<1ms" if g < 1e6 else "<10ms" if g < 1e7 else ">=10ms"
        hist[b] += g
    print("idle by gap size:", {k: round(v / 1e9, 3) for k, v in hist.items()})


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 15)
