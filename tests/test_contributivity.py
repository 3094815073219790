"""CPU: every coalition-evaluating estimator reproduces the reference on fixed v(S) tables.

tests/golden/estimators.json holds, per (n, seed, method), what the REFERENCE's Contributivity
(mplc/contributivity.py) produced with np.random.seed(seed) on the same table: scores, std, normalized,
calls count, the order coalitions were fitted, the memo keys, the increments and the next draw of the
global RNG.  Host-side estimators must match bit for bit (same RNG stream, same float operations);
"Shapley values" aggregates on the GPU and is checked to 1e-12 in the gpu test below.
"""
import json
import os
import types

import numpy as np
import pytest

import mplc.multi_partner_learning as mpl_mod
from mplc.contributivity import Contributivity

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "estimators.json")


def load_cases():
    with open(GOLDEN) as f:
        return json.load(f)["data"]


CASES = load_cases()


def parse_table(case):
    table = {}
    for k, v in case["table"].items():
        table[tuple(int(x) for x in k.split(",")) if k else ()] = v
    return table


def make_scenario(case, calls, batched=False, device_planning=False):
    table = parse_table(case)

    class FakeMPL:
        def __init__(self, scenario, partners_list=None, partner=None, **kw):
            if partner is not None:
                partners_list = [partner]
            self.ids = tuple(sorted(int(p.id) for p in partners_list))
            self.history = types.SimpleNamespace(score=None)

        def fit(self):
            calls.append(self.ids)
            self.history.score = table[self.ids]

    if batched:
        def evaluate_coalitions(scenario, coalitions):
            for c in coalitions:
                calls.append(tuple(c))
            return np.array([table[tuple(c)] for c in coalitions])
        FakeMPL.evaluate_coalitions = staticmethod(evaluate_coalitions)
        FakeMPL.device_planning = device_planning

    partners = [types.SimpleNamespace(id=i, y_train=np.zeros(s)) for i, s in enumerate(case["sizes"])]
    return types.SimpleNamespace(partners_list=partners, multi_partner_learning_approach=FakeMPL), FakeMPL


def run_case(case, monkeypatch, batched=False, device_planning=False):
    calls = []
    scenario, fake = make_scenario(case, calls, batched, device_planning)
    monkeypatch.setattr(mpl_mod, "SinglePartnerLearning", fake)
    np.random.seed(case["seed"])
    c = Contributivity(scenario=scenario)
    err = None
    try:
        c.compute_contributivity(case["method"])
    except Exception as e:  # noqa: BLE001
        err = f"{type(e).__name__}: {e}"
    return c, calls, err, float(np.random.uniform())


def same(a, b):
    a = np.asarray(a, dtype=float)
    b = np.asarray(b, dtype=float)
    return a.shape == b.shape and np.array_equal(a, b, equal_nan=True)


HOST_CASES = [c for c in CASES if c["method"] != "Shapley values"
              and not (c["method"] == "IS_reg_S" and c["n"] < 4)]


@pytest.mark.parametrize("case", HOST_CASES, ids=lambda c: f"{c['method']}-n{c['n']}")
def test_estimator_matches_reference(case, monkeypatch):
    c, calls, err, nxt = run_case(case, monkeypatch)
    if case["error"]:
        assert err is not None and err.split(":")[0] == case["error"].split(":")[0]
        return
    assert err is None, err
    assert c.name == case["name"]
    assert same(np.atleast_1d(c.contributivity_scores), case["scores"])
    assert same(np.atleast_1d(c.scores_std), case["std"])
    assert same(np.atleast_1d(c.normalized_scores), case["normalized"])
    assert c.first_charac_fct_calls_count == case["calls_count"]
    assert [list(k) for k in c.charac_fct_values.keys()] == case["memo_keys"]
    assert [list(x) for x in calls] == case["fit_order"]
    got_inc = [{",".join(map(str, k)): float(v) for k, v in d.items()} for d in c.increments_values]
    assert got_inc == case["increments"]
    assert nxt == case["rng_next_uniform"]


BATCH_METHODS = ("TMCS", "ITMCS", "IS_lin_S", "IS_reg_S", "SMCS", "WR_SMC", "Independent scores", "AIS_Kriging_S")


@pytest.mark.parametrize("case", [c for c in HOST_CASES if c["method"] in BATCH_METHODS and not c["error"]],
                         ids=lambda c: f"batched-{c['method']}-n{c['n']}")
def test_batched_planning_changes_nothing(case, monkeypatch):
    """With an engine-backed approach the estimators pre-plan and batch their coalitions; memo, call count,
    scores and RNG stream must be identical to the sequential reference."""
    c, calls, err, nxt = run_case(case, monkeypatch, batched=True)
    assert err is None, err
    assert same(np.atleast_1d(c.contributivity_scores), case["scores"])
    assert same(np.atleast_1d(c.scores_std), case["std"])
    assert c.first_charac_fct_calls_count == case["calls_count"]
    assert [list(k) for k in c.charac_fct_values.keys()] == case["memo_keys"]
    assert nxt == case["rng_next_uniform"]
    # every coalition is trained at most once by the engine
    assert len(calls) == len(set(calls))


def test_unknown_method_is_ignored(monkeypatch):
    case = [c for c in CASES if c["method"] == "Not a method"][0]
    c, calls, err, _ = run_case(case, monkeypatch)
    assert err is None and calls == [] and c.first_charac_fct_calls_count == 0


def test_unrank_combination_matches_itertools():
    from itertools import combinations
    items = [0, 2, 3, 5, 7, 8, 9]
    for r in range(len(items) + 1):
        for idx, comb in enumerate(combinations(items, r)):
            assert Contributivity._unrank_combination(items, r, idx) == comb


@pytest.mark.gpu
@pytest.mark.parametrize("case", [c for c in CASES if c["method"] == "Shapley values"
                                  or (c["method"] == "IS_reg_S" and c["n"] < 4)],
                         ids=lambda c: f"{c['method']}-n{c['n']}")
def test_exact_shapley_on_device_matches_reference(case, monkeypatch):
    c, calls, err, nxt = run_case(case, monkeypatch)
    assert err is None
    assert c.name == case["name"]
    ref = np.array(case["scores"])
    assert np.max(np.abs(c.contributivity_scores - ref)) <= 1e-12 * np.max(np.abs(ref))
    assert np.max(np.abs(c.normalized_scores - np.array(case["normalized"]))) <= 1e-11
    assert c.first_charac_fct_calls_count == case["calls_count"]
    assert [list(x) for x in calls] == case["fit_order"]
    assert nxt == case["rng_next_uniform"]


@pytest.mark.parametrize("method,n,max_batches", [("SMCS", 10, 40), ("SMCS", 8, 30), ("WR_SMC", 8, 10),
                                                  ("IS_lin_S", 8, 15)])
def test_speculative_planning_makes_few_large_batches(method, n, max_batches, monkeypatch):
    """SMCS / WR_SMC / IS plan several iterations ahead (one iteration = at most 2N coalitions per
    launch): the whole estimator needs only a few engine batches, and still matches the reference."""
    case = next(c for c in CASES if c["method"] == method and c["n"] == n and not c["error"])
    calls, batches = [], []
    scenario, fake = make_scenario(case, calls, batched=True)
    inner = fake.evaluate_coalitions

    def counting(sc, coalitions):
        batches.append(len(coalitions))
        return inner(sc, coalitions)
    fake.evaluate_coalitions = staticmethod(counting)
    monkeypatch.setattr(mpl_mod, "SinglePartnerLearning", fake)
    np.random.seed(case["seed"])
    c = Contributivity(scenario=scenario)
    c.compute_contributivity(method)
    assert same(np.atleast_1d(c.contributivity_scores), case["scores"])
    assert c.first_charac_fct_calls_count == case["calls_count"]
    assert len(batches) <= max_batches, batches
