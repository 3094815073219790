"""Per-launch HBM traffic from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md, HBM section).

FETCH_SIZE and WRITE_SIZE are in KiB.  gfx950 tallies wide coalesced reads at half their bytes, so FETCH is
doubled; WRITE is taken as reported.  Usage: python scripts/pmc_traffic.py <fetch dir> <write dir> <bench json of the profiled run> <out.json>
bench.py fills roofline.traffic from <out.json> when its workload string matches the profiled run's
(profiles/pmc_traffic.json: config #3 + #5; profiles/pmc_traffic_config4.json: the CIFAR10 leg, with the
algorithmic bytes of the same launches when the profiled bench line carries them).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "distributed-learning-contributivity_amd"))


def load(d, counter):
    tot, n = defaultdict(float), defaultdict(set)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            tot[k] += float(r["Counter_Value"]) * 1024.0
            n[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    return tot, {k: len(v) for k, v in n.items()}


def main(fetch_dir, write_dir, bench_json, out):
    f, nf = load(fetch_dir, "FETCH_SIZE")
    w, nw = load(write_dir, "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        launches = max(nf.get(k, 0), nw.get(k, 0), 1)
        rd = 2.0 * f.get(k, 0.0) / max(nf.get(k, 1), 1)
        wr = w.get(k, 0.0) / max(nw.get(k, 1), 1)
        res[k] = {"launches": launches, "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                  "traffic_bytes_per_launch": rd + wr,
                  "note": "FETCH_SIZE x2 (gfx950 half-count of wide reads) + WRITE_SIZE, KiB->bytes"}
    line = json.loads([ln for ln in open(bench_json) if ln.startswith("{")][-1])
    # config #4 leg under --no-kernel-timer: the algorithmic bytes of ALL its launches (bench.py StashOnly), so the
    # counters' bytes and the algorithm's bytes describe the same launches
    alg = line.get("algorithmic_bytes_per_launch_all") or {}
    for k, e in res.items():
        if alg.get(k):
            e["algorithmic_bytes_per_launch"] = alg[k]
            e["traffic_over_algorithmic"] = e["traffic_bytes_per_launch"] / alg[k]
            e["launches_stashed"] = alg["launches"]
    doc = {"workload": line["config"]["workload"], "source": f"{fetch_dir} + {write_dir}", "kernels": res}
    comp = alg.get("compulsory") or {}
    if comp:  # config #4: every launch name's counter bytes beside its compulsory bytes (mplc.cifar.compulsory_bytes)
        from mplc.cifar import launch_name
        by = defaultdict(lambda: [0.0, 0.0, 0, 0])
        for k, v in f.items():
            e = by[launch_name(k) or k]
            e[0] += 2.0 * v
            e[2] += nf[k]
        for k, v in w.items():
            e = by[launch_name(k) or k]
            e[1] += v
            e[3] += nw[k]
        summ = {}
        for name, (rd, wr, lf, lw) in sorted(by.items()):
            rec = {"pmc_read_bytes": rd, "pmc_write_bytes": wr, "pmc_launches": max(lf, lw)}
            c = comp.get(name)
            if c and c["bytes"] > 0:
                rec.update({"compulsory_bytes": c["bytes"], "compulsory_launches": c["launches"],
                            "traffic_over_compulsory": (rd + wr) / c["bytes"]})
            summ[name] = rec
        doc["by_launch"] = summ
        doc["over_1_1"] = sorted(k for k, r in summ.items() if r.get("traffic_over_compulsory", 0) > 1.1)
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
