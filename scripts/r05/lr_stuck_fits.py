"""CPU restatement of csrc/logreg.hip's fit loop (damped Newton, Armijo 1e-4, <= 40 halvings, <= 100 iterations,
|g| < 1e-10) over the config #2 sweep's multi-partner coalitions (E = 3, M = 1, warm starts from the FedAvg
average): counts the fits that never converge, with and without the full Newton step once g.d <= 1e-10 |f|.

    python scripts/r05/lr_stuck_fits.py
"""
import os
import sys
from itertools import combinations

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "distributed-learning-contributivity_amd"))


def fit(X, y01, w0, full_rule, tol=1e-10):
    y = np.where(y01 > 0.5, 1.0, -1.0)
    n, d = X.shape
    Xa = np.hstack([X, np.ones((n, 1))])
    reg = np.ones(d + 1)
    reg[-1] = 0.0
    w = w0.copy()

    def obj(v):
        return np.sum(np.logaddexp(0.0, -y * (Xa @ v))) + 0.5 * np.sum(reg * v * v)

    f, its = obj(w), 0
    for _ in range(100):
        s = 1 / (1 + np.exp(y * (Xa @ w)))
        g = -(Xa.T @ (y * s)) + reg * w
        if np.max(np.abs(g)) < tol:
            break
        its += 1
        step = np.linalg.solve(Xa.T @ (Xa * (s * (1 - s))[:, None]) + np.diag(reg), g)
        gd = g @ step
        full = full_rule and gd <= 1e-10 * max(1.0, abs(f))
        t = 1.0
        for _l in range(40):
            wn = w - t * step
            fn = obj(wn)
            if full or fn <= f - 1e-4 * t * gd:
                break
            t *= 0.5
        w, f = wn, fn
    return w, its


def main():
    import bench
    from mplc.fedavg import aggregation_weights
    sc = bench.build_titanic_scenario()
    parts = [(np.asarray(p.x_train, dtype=np.float64), np.asarray(p.y_train)) for p in sc.partners_list]
    sizes = [len(p[1]) for p in parts]
    coals = [c for k in range(2, 11) for c in combinations(range(10), k)]
    for full_rule in (False, True):
        its_all = []
        for c in coals:
            ww, scl = aggregation_weights([sizes[p] for p in c])
            theta = None
            for _e in range(3):
                res = [fit(*parts[p], np.zeros(28) if theta is None else theta, full_rule) for p in c]
                its_all += [r[1] for r in res]
                theta = (np.array([r[0] for r in res]) * np.asarray(ww)[:, None]).sum(0) / scl
        its_all = np.array(its_all)
        print(f"full step under rounding: {full_rule}: {len(its_all)} fits, {int((its_all >= 100).sum())} at the "
              f"100-iteration cap, max {its_all.max()}, mean {its_all.mean():.2f}", flush=True)


if __name__ == "__main__":
    main()
