"""Planner simulation (CPU): the product TMCS / ITMCS (mplc.contributivity) with a table-backed evaluator that
records every batch it is asked to train, for several speculation targets (scenario.mc_plan_replicas).

    python scripts/sim_tmcs_planning.py [values.npz] [--method TMCS] [--targets 0,256,512,1024,2048]

values.npz: bench.py --leg cifar --dump-values (bitmask -> v(S) of a real config #4 run).  Coalitions the dump
does not hold (speculation of another planner) get the mean of the dumped values of their size plus keyed noise
of the dumped spread.  Without a file: a synthetic saturating game.  Reports lockstep batches, replicas per batch,
trained vs counted coalitions and a time estimate from the per-batch cost model t = A + B * replicas (--cost)."""
import argparse
import sys
import types

import numpy as np

sys.path.insert(0, "distributed-learning-contributivity_amd")
from mplc.contributivity import Contributivity  # noqa: E402


def load_table(path, n):
    if path:
        d = np.load(path)
        vals = {int(m): float(v) for m, v in zip(d["masks"], d["values"])}
    else:
        rng = np.random.default_rng(3)
        vals = {}
        for m in range(1, 1 << n):
            k = bin(m).count("1")
            vals[m] = 0.45 - 0.33 * np.exp(-k / 5.0) + rng.normal(0, 0.01)
    by_size = {}
    for m, v in vals.items():
        by_size.setdefault(bin(m).count("1"), []).append(v)
    mean = {k: np.mean(v) for k, v in by_size.items()}
    sd = {k: (np.std(v) if len(v) > 1 else 0.01) for k, v in by_size.items()}

    def value(key):
        m = sum(1 << i for i in key)
        if m in vals:
            return vals[m]
        k = len(key)
        rng = np.random.default_rng(m)
        kk = min(mean, key=lambda s: abs(s - k))
        return float(mean[kk] + rng.normal(0, sd[kk]))
    return value, len(vals)


def run(n, value, method, target, wave_scale=1, adaptive=True, margin=0.5, world=1):
    batches = []
    Contributivity._world_size = lambda self: world  # the planner's per-rank targets and wave scale at N ranks

    class Approach:
        device_planning = False

        @staticmethod
        def evaluate_coalitions(scenario, cs):
            batches.append(sum(len(c) for c in cs))
            return np.array([value(c) for c in cs])

    partners = [types.SimpleNamespace(id=i, y_train=np.zeros(1822)) for i in range(n)]
    sc = types.SimpleNamespace(partners_list=partners, multi_partner_learning_approach=Approach, mc_plan_replicas=target,
                               mc_wave_scale=wave_scale, mc_wave_adaptive=adaptive,
                               mc_plan_overhead=margin)
    np.random.seed(0)
    c = Contributivity(scenario=sc)
    c.compute_contributivity(method)
    trained = len(sc.coalition_values) + 1
    return c, batches, trained


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("values", nargs="?")
    ap.add_argument("--n", type=int, default=20)
    ap.add_argument("--method", default="TMCS")
    ap.add_argument("--targets", default="0,256,512,1024,2048,4096")
    ap.add_argument("--margins", default="16", help="mc_plan_overhead values")
    ap.add_argument("--cost", default="0.09,0.0033", help="A,B of the per-batch time model (s, s per replica)")
    ap.add_argument("--world", type=int, default=1, help="ranks: a batch costs A + B * replicas / world")
    ap.add_argument("--scales", default="0", help="mc_wave_scale values (0: the world size)")
    args = ap.parse_args()
    A, B = (float(x) for x in args.cost.split(","))
    value, held = load_table(args.values, args.n)
    ref = None
    for target, adaptive, margin, scale in [(int(t), a, float(m), int(w)) for a in (False, True)
                                            for t in args.targets.split(",") for m in args.margins.split(",")
                                            for w in args.scales.split(",")]:
        c, batches, trained = run(args.n, value, args.method, target, adaptive=adaptive, margin=margin,
                                  world=args.world, wave_scale=scale)
        if ref is None:
            ref = c.contributivity_scores
        assert np.array_equal(ref, c.contributivity_scores)  # speculation never changes the result
        reps = np.array(batches)
        est = len(reps) * A + np.ceil(reps / args.world).sum() * B
        print(f"{'adaptive' if adaptive else 'fixed   '} scale {scale} target {target:5d} overhead {margin}: batches {len(reps):4d}  replicas/batch {reps.mean():7.1f} (median "
              f"{np.median(reps):6.0f})  counted {c.first_charac_fct_calls_count}  trained {trained}  "
              f"(+{100 * (trained / c.first_charac_fct_calls_count - 1):.1f} %)  replicas {reps.sum()}  "
              f"est {est:6.1f} s -> {c.first_charac_fct_calls_count / est:6.1f} evals/s  "
              f"walks {getattr(c, 'mc_walks', None)} plan {getattr(c, 'plan_stats', {})}", flush=True)


if __name__ == "__main__":
    main()
