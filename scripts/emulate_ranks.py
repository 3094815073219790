"""Emulate an N-GPU config #3 exact-Shapley sweep on one GPU: train EVERY rank's LPT shard of the 1023 coalitions
alone, one after the other, and report the max over ranks (the N-rank job waits for its slowest rank at the one
all_reduce of v(S)).  v(S) depends only on (S, seed), so each shard trains exactly what that rank would.

    python scripts/emulate_ranks.py <E> <es 0|1> <signal> N [N ...]

E=2, es 0: the bench's config #3 (fixed epochs).  E=40, es 1, signal 0.2: the reference's defaults with the early-
stopping rule, where a coalition's cost follows its realised epochs (15-28 in round 4), which LPT's cost
(sum of partner rows, mplc.parallel.coalition_cost) does not see.  Prints one JSON line per N with every rank's
seconds, training samples and realised epochs; the all_reduce itself (8 KB over xGMI) is not included."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "distributed-learning-contributivity_amd"))
import threading  # noqa: E402
from itertools import combinations  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from mplc import parallel  # noqa: E402

_T0 = time.time()


def _heartbeat():  # a line on stderr every 30 s: a long shard is not a hung GPU command
    while True:
        time.sleep(30)
        print(f"heartbeat {time.time() - _T0:.0f}s", file=sys.stderr, flush=True)


threading.Thread(target=_heartbeat, daemon=True).start()


def main():
    E, es, signal = int(sys.argv[1]), bool(int(sys.argv[2])), float(sys.argv[3])
    Ns = [int(v) for v in sys.argv[4:]]
    torch.cuda.set_device(0)
    sc = bench.build_scenario(10, E, 20, 8, early_stopping=es, signal=signal)
    from mplc.engine import CoalitionEngine
    eng = CoalitionEngine.for_scenario(sc)
    eng.warmup()
    coals = [c for k in range(1, 11) for c in combinations(range(10), k)]
    sizes = eng.partner_sizes
    eng.evaluate([(0, 1)], epoch_count=1)  # first allocation outside the timed shards
    epochs_by_coal = {}
    for N in Ns:
        shards = parallel.lpt_shard([parallel.coalition_cost(c, sizes) for c in coals], N)
        ranks = []
        for r, sh in enumerate(shards):
            mine = [coals[i] for i in sh]
            s0 = eng.stats.get("samples", 0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = eng.evaluate(mine, return_details=True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            ep = res["epochs_done"]
            for c, e in zip(mine, ep):
                epochs_by_coal[c] = int(e)
            ranks.append({"rank": r, "s": round(dt, 3), "coalitions": len(mine),
                          "lpt_cost": float(sum(parallel.coalition_cost(c, sizes) for c in mine)),
                          "samples": int(eng.stats.get("samples", 0) - s0),
                          "epochs_mean": round(float(np.mean(ep)), 2), "epochs_max": int(np.max(ep))})
            print(f"N={N} rank {r}: {dt:.2f} s, {len(mine)} coalitions, epochs mean {np.mean(ep):.1f} max {np.max(ep)}",
                  file=sys.stderr, flush=True)
        wall = max(x["s"] for x in ranks)
        print(json.dumps({"N": N, "E": E, "early_stopping": es, "signal": signal, "max_rank_s": round(wall, 3),
                          "mean_rank_s": round(float(np.mean([x["s"] for x in ranks])), 3),
                          "evals_per_s": round(1023 / wall, 2), "ranks": ranks}), flush=True)
    if es:
        by_size = {}
        for c, e in epochs_by_coal.items():
            by_size.setdefault(len(c), []).append(e)
        print(json.dumps({"realised_epochs_by_size": {k: [round(float(np.mean(v)), 2), int(np.min(v)), int(np.max(v))]
                                                      for k, v in sorted(by_size.items())}}), flush=True)


if __name__ == "__main__":
    main()
