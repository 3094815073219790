"""Bitwise A/B of two builds of the LR engine (csrc/logreg.hip): run in a child process per library
(MPLC_LIB_PATH), the config #2 sweep (E=3, M=1), an early-stopping sweep (E=15, M=2: the stop rule at epoch >= 10)
and one coalition's learning history; compare correct counts, thetas, epochs and histories bit for bit.

    python scripts/r05/lr_ab.py <lib A> <lib B> <out dir>
"""
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(out):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "distributed-learning-contributivity_amd"))
    import time
    from itertools import combinations

    import torch
    import bench
    from mplc import _native
    from mplc.engine import CoalitionEngine
    res = {}
    for tag, E, M, es in (("c2", 3, 1, False), ("es", 15, 2, True)):
        sc = bench.build_titanic_scenario(epochs=E, M=M)
        sc.is_early_stopping = es
        eng = CoalitionEngine.for_scenario(sc)
        coals = [c for k in range(1, 11) for c in combinations(range(10), k)]
        eng.evaluate(coals[:3], return_details=True, is_early_stopping=es)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d = eng.evaluate(coals, return_details=True, return_models=True, is_early_stopping=es)
        torch.cuda.synchronize()
        res[tag + "_s"] = time.perf_counter() - t0
        res[tag + "_scores"] = np.asarray(d["scores"])
        res[tag + "_epochs"] = np.asarray(d["epochs_done"])
        res[tag + "_theta"] = np.asarray(eng.last_theta)
        h = eng.evaluate([(1, 4, 6)], return_details=True, record_history=True, is_early_stopping=es)["history"]
        for k, v in h.items():
            for n, a in v.items():
                res[f"{tag}_hist_{k}_{n}"] = np.asarray(a)
    np.savez(out, **res)
    print(_native.lib_path(), {k: round(v, 4) for k, v in res.items() if k.endswith("_s")}, flush=True)


def main(a, b, odir):
    os.makedirs(odir, exist_ok=True)
    outs = []
    for i, lib in enumerate((a, b)):
        out = os.path.join(odir, f"lr_ab_{i}.npz")
        env = dict(os.environ, MPLC_LIB_PATH=os.path.abspath(lib))
        subprocess.run([sys.executable, __file__, "--child", out], env=env, check=True, timeout=300)
        outs.append(np.load(out))
    A, B = outs
    diff = [k for k in A.files if not k.endswith("_s") and not np.array_equal(A[k], B[k], equal_nan=True)]
    rep = {"identical": not diff, "differing": diff, "seconds": {k: [float(A[k]), float(B[k])] for k in A.files if k.endswith("_s")},
           "keys": len(A.files)}
    print(json.dumps(rep))
    json.dump(rep, open(os.path.join(odir, "lr_ab.json"), "w"), indent=1)
    return 0 if not diff else 1


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2])
    else:
        sys.exit(main(*sys.argv[1:4]))
