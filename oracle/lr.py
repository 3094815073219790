"""ORACLE (test infrastructure only) - CPU restatement of the reference's Titanic coalition value.

Reference model: mplc/dataset.py:323-394 ``Titanic.LogisticRegression`` = sklearn LogisticRegression
(lbfgs, C=1, L2, fit_intercept, max_iter=1e4, warm_start) whose fit() solves the convex problem
    min_{w,b}  sum_i log(1 + exp(-y_i (w.x_i + b))) + 0.5 ||w||^2      (y_i in {-1,+1}, b unpenalised)
to sklearn's tolerance.  FedAvg (mplc/multi_partner_learning.py:285-334): each round every partner
refits on its minibatch (warm start does not change the optimum of a strictly convex problem), the
(1, 28) weight rows [coef | intercept] are np.average'd with data-volume weights (float64), and the test
score is the accuracy of predict() = [w.x + b > 0].

This restatement solves each fit EXACTLY (Newton, float64).  Pinned against the reference's own FedAvg
runs (tests/golden/fedavg_lr.json: 71 coalitions of 3/5/10-partner scenarios run through
mplc.Scenario/FederatedAverageLearning here) - tests/test_lr.py.
"""
import numpy as np


def fit_exact(X, y01, w0=None, tol=1e-12, max_iter=100):
    """Exact optimum of the sklearn C=1 L2 logistic regression (Newton with backtracking), float64."""
    X = np.asarray(X, dtype=np.float64)
    y = np.where(np.asarray(y01) > 0.5, 1.0, -1.0)
    n, d = X.shape
    Xa = np.hstack([X, np.ones((n, 1))])
    w = np.zeros(d + 1) if w0 is None else np.array(w0, dtype=np.float64)
    reg = np.ones(d + 1)
    reg[-1] = 0.0

    def obj(w):
        z = y * (Xa @ w)
        return np.sum(np.logaddexp(0.0, -z)) + 0.5 * np.sum(reg * w * w)

    f = obj(w)
    for _ in range(max_iter):
        z = y * (Xa @ w)
        s = 1.0 / (1.0 + np.exp(z))           # sigma(-z)
        g = -(Xa.T @ (y * s)) + reg * w
        if np.max(np.abs(g)) < tol:
            break
        h = s * (1.0 - s)
        H = Xa.T @ (Xa * h[:, None]) + np.diag(reg)
        step = np.linalg.solve(H, g)
        t = 1.0
        while True:
            wn = w - t * step
            fn = obj(wn)
            if fn <= f - 1e-4 * t * (g @ step) or t < 1e-10:
                break
            t *= 0.5
        w, f = wn, fn
    return w


def accuracy(w, X, y01):
    X = np.asarray(X, dtype=np.float64)
    pred = (X @ w[:-1] + w[-1]) > 0
    return float(np.mean(pred == (np.asarray(y01) > 0.5)))


def fedavg_value(partners, coalition, X_test, y_test, epochs=1, sizes=None):
    """v(S) of a FedAvg coalition with M = 1 (each round: partner optimum on its full data)."""
    thetas = [fit_exact(partners[p][0], partners[p][1]) for p in coalition]
    if sizes is None:
        sizes = [len(partners[p][1]) for p in coalition]
    w = np.asarray(sizes) / np.sum(sizes)
    theta = np.average(np.array(thetas), axis=0, weights=w)
    return accuracy(theta, X_test, y_test)


def single_value(partners, p, X_test, y_test):
    """Singleton v({p}): the reference crashes here (SinglePartnerLearning passes callbacks= to the LR fit,
    mplc/multi_partner_learning.py:254-260 vs mplc/dataset.py:329); defined as the fit on p's full data."""
    return accuracy(fit_exact(partners[p][0], partners[p][1]), X_test, y_test)
