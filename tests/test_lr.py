"""Titanic (BASELINE config #2): batched FedAvg logistic regression.

tests/golden/fedavg_lr.json holds the REFERENCE's own v(S) for 71 coalitions (3-, 5- and 10-partner
scenarios on Titanic-shaped data, run through mplc.Scenario / FederatedAverageLearning with
Titanic.LogisticRegression here).  The reference's sklearn lbfgs stops at tol 1e-4; the oracle and the
device kernel solve each fit exactly, so predictions may differ from the reference only on test points
that sit within that tolerance of the decision boundary: 2 of 71 coalitions differ by one test sample.
"""
import json
import os

import numpy as np
import pytest

from oracle import lr as olr

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "fedavg_lr.json")


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)["data"]


def scenario_for(golden, case):
    from mplc.dataset import Titanic
    from mplc.scenario import Scenario
    X = np.array(golden["data"]["X"], dtype=np.float32)
    y = np.array(golden["data"]["y"], dtype=np.float32)
    ds = Titanic(x=X, y=y)
    sc = Scenario(case["partners_count"], case["amounts"], dataset=ds, epoch_count=case["epoch_count"],
                  minibatch_count=case["minibatch_count"], is_early_stopping=False)
    return sc.provision()


def test_oracle_vs_reference_fedavg_lr(golden):
    from sklearn.model_selection import train_test_split
    X = np.array(golden["data"]["X"], dtype=np.float32)
    y = np.array(golden["data"]["y"], dtype=np.float32)
    _, xte, _, yte = train_test_split(X, y, test_size=0.1, random_state=42)
    total, exact, worst = 0, 0, 0
    for case in golden["cases"]:
        parts = [(np.array(p["x_train"]), np.array(p["y_train"])) for p in case["partners"]]
        for k, v in case["values"].items():
            coal = tuple(int(i) for i in k.split(","))
            mine = olr.fedavg_value(parts, coal, xte, yte)
            total += 1
            exact += mine == v
            worst = max(worst, round(abs(mine - v) * len(yte)))
    assert total == 71
    assert exact >= 69 and worst <= 1


def test_titanic_scenario_partitions_match_reference(golden):
    for case in golden["cases"]:
        sc = scenario_for(golden, case)
        for p, gp in zip(sc.partners_list, case["partners"]):
            assert np.array_equal(p.x_train, np.array(gp["x_train"], dtype=np.float32))
            assert np.array_equal(p.y_train, np.array(gp["y_train"], dtype=np.float32))
            assert p.batch_size == gp["batch_size"]


@pytest.mark.gpu
def test_device_lr_fedavg_matches_oracle_and_reference(golden):
    from mplc.engine import CoalitionEngine
    from itertools import combinations
    total, exact_ref = 0, 0
    for case in golden["cases"]:
        sc = scenario_for(golden, case)
        eng = CoalitionEngine.for_scenario(sc)
        ds = sc.dataset
        parts = [(p.x_train, p.y_train) for p in sc.partners_list]
        n = case["partners_count"]
        coals = [tuple(int(i) for i in k.split(",")) for k in case["values"]]
        coals += [(p,) for p in range(n)]
        if n <= 5:
            coals += [c for r in range(2, n + 1) for c in combinations(range(n), r) if c not in coals]
        res = eng.evaluate(coals, return_details=True)
        for ci, c in enumerate(coals):
            if len(c) == 1:
                ref = olr.single_value(parts, c[0], ds.x_test, ds.y_test)
                theta_ref = olr.fit_exact(*parts[c[0]])
            else:
                ref = olr.fedavg_value(parts, c, ds.x_test, ds.y_test)
                sizes = [len(parts[p][1]) for p in c]
                theta_ref = np.average(np.array([olr.fit_exact(*parts[p]) for p in c]), axis=0,
                                       weights=np.asarray(sizes) / np.sum(sizes))
            assert res["scores"][ci] == ref, (c, res["scores"][ci], ref)
            assert np.max(np.abs(eng.last_theta[ci] - theta_ref)) < 1e-8
            key = ",".join(map(str, c))
            if key in case["values"]:
                total += 1
                exact_ref += res["scores"][ci] == case["values"][key]
                assert abs(res["scores"][ci] - case["values"][key]) * len(ds.y_test) <= 1 + 1e-9
        assert np.all(res["epochs_done"] == case["epoch_count"])
    assert total == 71 and exact_ref >= 69


@pytest.mark.gpu
def test_titanic_exact_shapley_all_1023_coalitions():
    """Config #2: 10 partners, exact Shapley over all 1023 coalitions in one launch; efficiency holds."""
    from mplc.dataset import Titanic
    from mplc.scenario import Scenario
    from mplc.contributivity import Contributivity
    sc = Scenario(10, [0.1] * 10, dataset=Titanic(synthetic=True), epoch_count=3, minibatch_count=1,
                  is_early_stopping=False).provision()
    c = Contributivity(scenario=sc)
    c.compute_contributivity("Shapley values")
    assert c.first_charac_fct_calls_count == 1023
    assert abs(np.sum(c.contributivity_scores) - c.charac_fct_values[tuple(range(10))]) < 1e-12


@pytest.mark.gpu
def test_lr_evaluate_in_chunks_equals_one_call():
    """LogRegEngine.evaluate splits long coalition lists into calls of CALL_COALITIONS (the workspace holds every
    coalition's partner fits: ADVICE r5); every value, epoch count and model equals the one-call result."""
    from itertools import combinations
    from mplc.dataset import Titanic
    from mplc.engine import CoalitionEngine
    from mplc.scenario import Scenario
    sc = Scenario(10, [0.1] * 10, dataset=Titanic(synthetic=True), epoch_count=3, minibatch_count=1,
                  is_early_stopping=False).provision()
    eng = CoalitionEngine.for_scenario(sc)
    coals = [c for k in range(1, 11) for c in combinations(range(10), k)]
    one = eng.evaluate(coals, return_details=True, return_models=True)
    eng.CALL_COALITIONS = 100
    parts = eng.evaluate(coals, return_details=True, return_models=True)
    assert np.array_equal(one["scores"], parts["scores"]) and np.array_equal(one["epochs_done"], parts["epochs_done"])
    assert all(np.array_equal(a, b) for a, b in zip(one["models"], parts["models"]))


@pytest.mark.gpu
def test_fedavg_round_is_np_average_of_the_partner_fits():
    """E = 1, M = 1: a coalition's round-0 fits are its partners' singleton fits (same rows, same zero start, same
    code), so its model must be np.average of the singletons' models with the reference's weights, bit for bit
    (mplc/mpl_utils.py:90-115: multiply, then sum in partner order - no fused multiply-add)."""
    from itertools import combinations

    from mplc.dataset import Titanic
    from mplc.engine import CoalitionEngine
    from mplc.fedavg import aggregation_weights
    from mplc.scenario import Scenario
    sc = Scenario(10, [0.1] * 10, dataset=Titanic(synthetic=True), epoch_count=1, minibatch_count=1,
                  is_early_stopping=False).provision()
    eng = CoalitionEngine.for_scenario(sc)
    singles = [(p,) for p in range(10)]
    coals = singles + [c for k in (2, 3, 5, 10) for c in combinations(range(10), k)][::7]
    eng.evaluate(coals)
    theta = eng.last_theta
    sizes = eng.partner_sizes
    for ci, c in enumerate(coals[10:], start=10):
        w, scl = aggregation_weights([sizes[p] for p in c])
        wgt = np.asarray(w, dtype=np.float64).reshape(-1, 1)
        want = np.multiply(np.array([theta[p] for p in c]), wgt).sum(axis=0) / scl
        assert np.array_equal(theta[ci], want), (c, np.abs(theta[ci] - want).max())


def _restated_fedavg(sc, eng, coal, E, M, es, n_val):
    """Host restatement of the device FedAvg with minibatches and the early-stopping rule (mplc/multi_partner_learning.py
    :177-193, 285-334): each round every partner's exact fit (oracle/lr.py) on its minibatch of the keyed epoch
    permutation, np.average with data-volume weights; val loss of the round-0 model of each epoch on hard predictions
    (sklearn eps 1e-15), stop after epoch e >= 10 when it exceeds epoch e - 10's."""
    from mplc.cnn import keyed_perm, minibatch_bounds, shuffle_key, subkey
    from mplc.fedavg import aggregation_weights
    parts = [(np.asarray(p.x_train, dtype=np.float64), np.asarray(p.y_train)) for p in sc.partners_list]
    xv, yv = np.asarray(sc.dataset.x_val, dtype=np.float64), np.asarray(sc.dataset.y_val)
    mask = sum(1 << p for p in coal)
    w, scl = aggregation_weights([len(parts[p][1]) for p in coal])
    theta, have, vh, done = None, False, [], E
    for e in range(E):
        if es and E > 10 and e < 64:
            if have:
                cv = int(round(olr.accuracy(theta, xv, yv) * len(yv)))
                vh.append(((n_val - cv) * -np.log(1e-15) + cv * -np.log(1 - 1e-15)) / n_val)
            else:
                vh.append(0.0)
        for m in range(M):
            fits = []
            for p in coal:
                n_p = len(parts[p][1])
                sp = minibatch_bounds(n_p, M)
                key = subkey(shuffle_key(eng.seed, mask, p), 0x10000 + e, 0)
                pos = [keyed_perm(key, n_p, i) if M > 1 else i for i in range(sp[m], sp[m + 1])]
                fits.append(olr.fit_exact(parts[p][0][pos], parts[p][1][pos]))
            theta = np.multiply(np.array(fits), np.asarray(w).reshape(-1, 1)).sum(axis=0) / scl
            have = True
        if es and E > 10 and 10 <= e < 64 and vh[e] > vh[e - 10]:
            done = e + 1
            break
    return theta, done


@pytest.mark.gpu
def test_device_lr_minibatches_and_early_stopping_vs_restatement(golden):
    """M = 3 (the keyed per-epoch permutation, np.split bounds) and E = 14 with the early-stopping rule, on the
    reference's 5-partner Titanic case: thetas within 1e-8 of the host restatement, the same stop epochs and
    test accuracies."""
    case = [c for c in golden["cases"] if c["partners_count"] == 5][0]
    from mplc.dataset import Titanic
    from mplc.engine import CoalitionEngine
    from mplc.scenario import Scenario
    X = np.array(golden["data"]["X"], dtype=np.float32)
    y = np.array(golden["data"]["y"], dtype=np.float32)
    E, M = 14, 3
    sc = Scenario(5, case["amounts"], dataset=Titanic(x=X, y=y), epoch_count=E, minibatch_count=M,
                  is_early_stopping=True).provision()
    eng = CoalitionEngine.for_scenario(sc)
    coals = [(0, 1), (1, 3), (0, 2, 4), (1, 2, 3, 4), (0, 1, 2, 3, 4)]
    res = eng.evaluate(coals, return_details=True, is_early_stopping=True)
    n_val = len(sc.dataset.y_val)
    stops = []
    for ci, c in enumerate(coals):
        theta, done = _restated_fedavg(sc, eng, c, E, M, True, n_val)
        stops.append(done)
        assert res["epochs_done"][ci] == done, (c, res["epochs_done"][ci], done)
        assert np.max(np.abs(eng.last_theta[ci] - theta)) < 1e-8, (c, np.max(np.abs(eng.last_theta[ci] - theta)))
        assert res["scores"][ci] == olr.accuracy(theta, sc.dataset.x_test, sc.dataset.y_test)
    print("stop epochs", stops)


@pytest.mark.gpu
def test_lr_history_matches_reference(golden):
    """The grand coalition's learning history (mplc/mpl_utils.py:11-27) against the reference's own
    (tests/golden/lr_history.json: FederatedAverageLearning with Titanic.LogisticRegression on the same
    data and partition).  Accuracies are counts over val / minibatch rows: equal, or one sample apart where
    lbfgs' tolerance moves a point across the boundary; losses are those counts through log_loss."""
    with open(os.path.join(os.path.dirname(__file__), "golden", "lr_history.json")) as f:
        hcases = json.load(f)["data"]
    from mplc.engine import CoalitionEngine
    exact, total = 0, 0
    for case, hc in zip(golden["cases"], hcases):
        assert hc["partners_count"] == case["partners_count"]
        sc = scenario_for(golden, case)
        eng = CoalitionEngine.for_scenario(sc)
        n = case["partners_count"]
        res = eng.evaluate([tuple(range(n))], return_details=True, record_history=True)
        h = res["history"]
        ref = {(k if k == "mpl_model" else int(k)): v for k, v in hc["history"].items()}
        assert set(h) == set(ref)
        n_val = len(sc.dataset.y_val)
        for k, metrics in ref.items():
            for m, r in metrics.items():
                r = np.asarray(r, dtype=float)
                d = h[k][m]
                assert d.shape == r.shape
                if m.endswith("accuracy"):
                    rows = n_val if m == "val_accuracy" else len(sc.partners_list[k].y_train)
                    assert np.all(np.abs(d - r) * rows <= 1 + 1e-9), (k, m, d, r)
                    total += d.size
                    exact += int(np.sum(d == r))
        for k in ref:  # loss = f(accuracy): equal wherever the accuracy is
            for m in ("val_loss",) + (("loss",) if k != "mpl_model" else ()):
                acc = "val_accuracy" if m == "val_loss" else "accuracy"
                same = h[k][acc] == np.asarray(ref[k][acc])
                np.testing.assert_allclose(h[k][m][same], np.asarray(ref[k][m])[same], rtol=1e-9)
    assert exact >= 0.9 * total


@pytest.mark.gpu
def test_titanic_scenario_run_records_history_and_federated_sbs(golden):
    sc = scenario_for(golden, golden["cases"][1])
    sc.methods = ["Federated SBS linear", "Federated SBS constant"]
    sc.run()
    hist = sc.mpl.history.history
    assert set(hist) == set(range(5)) | {"mpl_model"}
    assert hist["mpl_model"]["val_accuracy"][0, 0] == 0.0  # the unfitted initial model evaluates to [0, 0]
    lin, const = sc.contributivity_list
    # E*M = 2 rounds: the kept rounds include round 0, whose collective model is the unfitted one (accuracy
    # 0), so the relative performances are inf there - the reference's own arithmetic, reproduced
    E, M = 2, 1
    rel = np.stack([hist[p]["val_accuracy"] for p in range(5)], axis=-1).reshape(E * M, 5)
    with np.errstate(divide="ignore", invalid="ignore"):
        rel = (rel / hist["mpl_model"]["val_accuracy"].reshape(E * M)[:, None])[0:2]
        np.testing.assert_array_equal(const.contributivity_scores, np.nanmean(rel, axis=0))
    assert np.all(np.isinf(const.contributivity_scores))


@pytest.mark.parametrize("n, seed, agg", [(10, 0, "data-volume"), (10, 7, "uniform"), (20, 3, "data-volume"),
                                          (64, 11, "data-volume"), (13, 2 ** 63 + 5, "data-volume")])
def test_launch_tables_equal_the_per_coalition_loop(n, seed, agg):
    """mplc.lr.coalition_tables (vectorised) against the per-coalition loop it replaced: masks, every member's
    shuffle key, the np.average weights and scale, bit for bit."""
    from itertools import combinations

    from mplc.cnn import shuffle_key
    from mplc.fedavg import aggregation_weights
    from mplc.lr import MAXP, coalition_tables
    rng = np.random.default_rng(n + seed % 97)
    sizes = [int(v) for v in rng.integers(1, 500, size=n)]
    if n <= 10:
        coals = [c for k in range(1, n + 1) for c in combinations(range(n), k)]
    else:
        coals = [tuple(sorted(rng.choice(n, size=int(rng.integers(1, n + 1)), replace=False).tolist()))
                 for _ in range(300)]
    C = len(coals)
    masks, keys = np.zeros(C, dtype=np.uint64), np.zeros((C, MAXP), dtype=np.uint64)
    w, scale = np.zeros((C, MAXP)), np.ones(C)
    for ci, c in enumerate(coals):
        mask = sum(1 << p for p in c)
        masks[ci] = mask
        for i, p in enumerate(c):
            keys[ci, i] = shuffle_key(seed, mask, p)
        if len(c) > 1:
            ww, scl = aggregation_weights([sizes[p] for p in c], agg)
            w[ci, :len(c)] = ww
            scale[ci] = scl
    got = coalition_tables(coals, sizes, seed, agg)
    for a, b in zip((masks, keys, w, scale), got):
        assert a.dtype == b.dtype and np.array_equal(a, b)
    with pytest.raises(ValueError):
        coalition_tables([(0, n)], sizes, seed, agg)
