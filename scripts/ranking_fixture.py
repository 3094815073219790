"""ORACLE fixture (test infrastructure; build container only): the 10-partner exact-Shapley partner ranking of the
CNN oracle, for tests/test_ranking_gpu.py ("partner ranking identical" at the 10-partner
exact-Shapley scale north_star names, mplc/contributivity.py:140-171, 1210-1253; tests/end_to_end_tests.py:66-73
ports the reference's own ranking assertion at 2 partners).

    python scripts/ranking_fixture.py [workers] [threads_per_worker]

The scenario (tests/spread_fixtures.py ranking_scenario, chosen on the GPU with scripts/probe_ranking.py: a partner
ranking that survives ~1-ulp perturbations of the data with every adjacent gap several times the perturbations'
spread): MNIST-shaped synthetic data (class templates, signal 0.2), 10 partners with unequal amounts, random split,
a short FedAvg schedule.  Every one of the 1023 coalitions is trained the reference's way, one after the other, by
oracle/cnn.py coalition_value (one CPU thread per worker process, the workers taking coalitions from a shared
list - each value is a function of the coalition alone), and the Shapley values come from the restatement of the
reference's shapley_value in its own fp64 operation order (oracle/shapley.py).  Written: tests/golden/
ranking_10p.json with the v(S) table (bitmask order), the Shapley values, their argsort, the scenario parameters
and a CRC of the data."""
import itertools
import json
import os
import sys
import time
from multiprocessing import get_context

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "distributed-learning-contributivity_amd")):
    sys.path.insert(0, p)

_STATE = {}


def _init(threads=1):
    import torch
    torch.set_num_threads(threads)
    from oracle import cnn as ocnn
    from spread_fixtures import ranking_scenario
    sc = ranking_scenario()
    ds = sc.dataset
    _STATE["data"] = ocnn.Data(ds.x_train, ds.y_train, ds.x_val, ds.y_val, ds.x_test, ds.y_test)
    _STATE["prow"] = [p.train_idx for p in sc.partners_list]
    _STATE["bs"] = [p.batch_size for p in sc.partners_list]
    _STATE["E"], _STATE["M"] = sc.epoch_count, sc.minibatch_count


def _value(coal):
    from oracle import cnn as ocnn
    s = _STATE
    return coal, float(ocnn.coalition_value(s["data"], s["prow"], s["bs"], coal, seed=0, epochs=s["E"], M=s["M"])[0])


def main():
    from oracle import shapley as oshap
    from spread_fixtures import GOLDEN, RANKING, data_crc, ranking_scenario
    workers = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 1  # another summation order: a second oracle sample
    sc = ranking_scenario()
    n = len(sc.partners_list)
    coals = [c for k in range(1, n + 1) for c in itertools.combinations(range(n), k)]
    # long coalitions first: the pool's tail is then short fits
    order = sorted(coals, key=lambda c: -sum(len(sc.partners_list[p].train_idx) for p in c))
    t0 = time.time()
    V = np.zeros(1 << n)
    with get_context("spawn").Pool(workers, initializer=_init, initargs=(threads,)) as pool:
        for i, (coal, v) in enumerate(pool.imap_unordered(_value, order, chunksize=1)):
            V[sum(1 << p for p in coal)] = v
            if i % 50 == 0:
                print(f"{i + 1}/{len(coals)} coalitions, {time.time() - t0:.0f}s", flush=True)
    # the reference's shapley_value takes v(S) in combinations order (mplc/contributivity.py:149-163)
    v_list = [V[sum(1 << p for p in c)] for c in coals]
    sv = [float(x) for x in oshap.shapley_reference_order(n, v_list)]
    out = {"generator": "scripts/ranking_fixture.py", "scenario": RANKING, "data_crc32": data_crc(sc),
           "partner_rows": [len(p.train_idx) for p in sc.partners_list],
           "batch_sizes": [int(p.batch_size) for p in sc.partners_list],
           "values_bitmask": V.tolist(), "shapley": sv, "argsort": [int(i) for i in np.argsort(sv)],
           "threads_per_worker": threads, "wall_s": round(time.time() - t0, 1)}
    path = os.path.join(GOLDEN, "ranking_10p.json" if threads == 1 else f"ranking_10p_t{threads}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path, "shapley", np.round(sv, 4).tolist(), "argsort", out["argsort"], f"{out['wall_s']}s")


if __name__ == "__main__":
    main()
