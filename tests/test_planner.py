"""CPU: the TMCS / ITMCS frontier planner (mplc.mc.plan_frontier, Contributivity._frontier_plan) and the adaptive
permutation waves.  Planning decides only WHICH coalitions are trained together; the estimators' results must not
depend on it (v(S) is a function of (S, seed)): scores, std, call count and memo order are compared with the
reference's one-coalition-at-a-time loop fed the same table, for every planner setting."""
import types

import numpy as np
import pytest

from mplc import mc
from mplc.contributivity import Contributivity


def _game(n, seed=3):
    rng = np.random.default_rng(seed)
    s = rng.uniform(1.0, 3.0, size=n)
    noise = rng.uniform(-0.02, 0.02, size=1 << n)

    def value(key):
        m = sum(1 << i for i in key)
        return float(0.1 + 0.8 * (1 - np.exp(-s[list(key)].sum() / (s.sum() / 3))) + noise[m])
    return value


def _run(n, value, method, **plan):
    batches = []

    class Approach:
        device_planning = False

        @staticmethod
        def evaluate_coalitions(scenario, cs):
            batches.append(list(cs))
            return np.array([value(c) for c in cs])

    partners = [types.SimpleNamespace(id=i, y_train=np.zeros(100 + i)) for i in range(n)]
    sc = types.SimpleNamespace(partners_list=partners, multi_partner_learning_approach=Approach, **plan)
    np.random.seed(0)
    c = Contributivity(scenario=sc)
    c.compute_contributivity(method)
    return c, batches


def _reference(n, value, method):
    """The reference's sequential loop: no batched evaluator, one fit per coalition through the plug-in."""
    import mplc.multi_partner_learning as mpl_mod

    class TableMPL:
        def __init__(self, scenario, partners_list=None, partner=None, **kw):
            self.ids = tuple(sorted(int(p.id) for p in (partners_list if partner is None else [partner])))
            self.history = types.SimpleNamespace(score=None)

        def fit(self):
            self.history.score = value(self.ids)
    saved = mpl_mod.SinglePartnerLearning
    mpl_mod.SinglePartnerLearning = TableMPL
    try:
        partners = [types.SimpleNamespace(id=i, y_train=np.zeros(100 + i)) for i in range(n)]
        np.random.seed(0)
        c = Contributivity(scenario=types.SimpleNamespace(partners_list=partners, multi_partner_learning_approach=TableMPL))
        c.compute_contributivity(method)
    finally:
        mpl_mod.SinglePartnerLearning = saved
    return c


@pytest.mark.parametrize("method", ["TMCS", "ITMCS"])
@pytest.mark.parametrize("plan", [dict(mc_plan_replicas=0, mc_wave_adaptive=False), dict(mc_plan_replicas=0),
                                  dict(mc_plan_overhead=8.0), dict(mc_plan_overhead=1e9, mc_plan_replicas=1 << 20)],
                         ids=["plain", "adaptive", "default", "greedy"])
def test_planning_is_result_neutral(method, plan):
    n = 9
    value = _game(n)
    ref = _reference(n, value, method)
    c, batches = _run(n, value, method, **plan)
    assert np.array_equal(ref.contributivity_scores, c.contributivity_scores)
    assert np.array_equal(ref.scores_std, c.scores_std)
    assert ref.first_charac_fct_calls_count == c.first_charac_fct_calls_count
    assert list(ref.charac_fct_values) == list(c.charac_fct_values)
    assert list(ref.charac_fct_values.values()) == list(c.charac_fct_values.values())
    assert all(len(set(b)) == len(b) for b in batches)  # no coalition twice in a batch
    trained = [k for b in batches for k in b]
    assert len(trained) == len(set(trained))  # and none trained twice


def test_greedy_speculation_uses_fewer_batches():
    n = 9
    value = _game(n)
    _, plain = _run(n, value, "TMCS", mc_plan_replicas=0, mc_wave_adaptive=False)
    _, greedy = _run(n, value, "TMCS", mc_plan_overhead=1e9, mc_plan_replicas=1 << 20, mc_wave_adaptive=False)
    assert len(greedy) < len(plain)


def test_plan_frontier_required_first_and_budget():
    n = 6
    perms = np.array([[0, 1, 2, 3, 4, 5], [5, 4, 3, 2, 1, 0], [2, 0, 4, 1, 5, 3]])
    known = {(0,): 0.3, (5,): 0.3, (4, 5): 0.5, tuple(range(n)): 0.9}  # v_all is always known

    def value(k):
        return known.get(k)
    pred = mc.size_predictor(known.items(), n, 0.9)
    stop = np.array([1, 2, 0])  # first unknown prefixes: (0, 1), (3, 4, 5), (2,)
    keys, req = mc.plan_frontier(perms, stop, value, pred, 0.9, 0.05, target_replicas=0)
    assert req == 3 and keys == [(0, 1), (3, 4, 5), (2,)]  # target 0: nothing speculative
    keys, req = mc.plan_frontier(perms, stop, value, pred, 0.9, 0.05, target_replicas=1 << 20, overhead_replicas=1e9)
    assert keys[:3] == [(0, 1), (3, 4, 5), (2,)]
    # unlimited budget: every deeper prefix of the three walks that is not known yet
    deeper = {tuple(sorted(int(i) for i in p[:j + 1])) for p in perms for j in range(n - 1)} - set(known)
    assert set(keys) == deeper
    keys0, _ = mc.plan_frontier(perms, stop, value, pred, 0.9, 0.05, target_replicas=1 << 20, overhead_replicas=0.0)
    assert keys0[:3] == [(0, 1), (3, 4, 5), (2,)]  # zero budget: only prefixes that are certainly needed
    # a known value inside the truncation band ends its walk's chain: nothing past it is speculated
    known[(0, 2)] = 0.88
    keys, _ = mc.plan_frontier(perms, stop, value, pred, 0.9, 0.05, target_replicas=1 << 20, overhead_replicas=1e9)
    assert not any(set(k) >= {0, 2, 4} and len(k) == 3 and 1 not in k for k in keys)


def test_size_predictor_spread_is_never_overconfident():
    known = [((0,), 0.1), ((1,), 0.9), ((0, 1), 0.5)]
    mean, sd = mc.size_predictor(known, 4, 0.7)
    assert mean[1] == pytest.approx(0.5) and mean[4] == 0.7
    assert np.all(sd >= np.std([0.1, 0.9, 0.5]) - 1e-12)  # few values per size: the pooled spread
