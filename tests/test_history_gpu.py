"""GPU: the learning history of a recorded fit (mplc/mpl_utils.py:11-27 History.history; logged by
mplc/multi_partner_learning.py:130-156) against the oracle's sequential restatement, and the Federated
SBS methods on a Scenario.run history.

Per round (e, m): 'mpl_model' val_loss / val_accuracy of the round-start global model; per partner the
Keras fit history of its round: running training CE / accuracy (the head kernel's hstats) and val
metrics of the partner model after its fit.  The round-0 entries come from bit-identical models (the
keyed init), so they agree to fp32 summation order; later rounds carry the training's fp32 drift and are
held to the +-1 pt (mean) accuracy bar of the v(S) tests."""
import numpy as np
import pytest

from oracle import cnn as ocnn

pytestmark = pytest.mark.gpu

METRICS = ("val_accuracy", "val_loss", "loss", "accuracy")


def make_scenario(approach="fedavg", partners=3, amounts=(0.2, 0.5, 0.3), M=2, E=2):
    from mplc.dataset import ArrayDataset, digits_as_mnist
    from mplc.scenario import Scenario
    x, y = digits_as_mnist()
    ds = ArrayDataset(x[:1500], y[:1500], x[1500:], y[1500:], name="mnist")
    sc = Scenario(partners, list(amounts), dataset=ds, minibatch_count=M, gradient_updates_per_pass_count=4,
                  epoch_count=E, is_early_stopping=False, multi_partner_learning_approach=approach)
    return sc.provision()


def engine_for(sc):
    from mplc.engine import CoalitionEngine
    return CoalitionEngine.for_scenario(sc, memory_budget_bytes=16 << 30, eval_budget_bytes=1 << 30)


def oracle_history(sc, eng, coal, approach):
    ds = sc.dataset
    data = ocnn.Data(ds.x_train, ds.y_train, ds.x_val, ds.y_val, ds.x_test, ds.y_test)
    h = {}
    acc, _ = ocnn.coalition_value(data, [p.train_idx for p in sc.partners_list],
                                  [p.batch_size for p in sc.partners_list], coal, seed=eng.seed,
                                  epochs=eng.epoch_count, M=eng.minibatch_count, approach=approach, history=h)
    return acc, h


def compare(dev, ref, coal):
    assert set(dev) == set(ref)
    for k in ref:
        for metric, r in ref[k].items():
            d = dev[k][metric]
            assert d.shape == r.shape, (k, metric)
            assert np.array_equal(np.isnan(d), np.isnan(r)), (k, metric)
    # round 0: identical starting models (keyed init); fp32 summation order only
    np.testing.assert_allclose(dev["mpl_model"]["val_loss"][0, 0], ref["mpl_model"]["val_loss"][0, 0], rtol=1e-5) \
        if "mpl_model" in ref else None
    if "mpl_model" in ref:
        assert abs(dev["mpl_model"]["val_accuracy"][0, 0] - ref["mpl_model"]["val_accuracy"][0, 0]) <= 2.5e-3
    # round 0's fits: a few optimizer steps (after other members' fits when sequential), each Adam step moving
    # every weight by ~lr * sign(g): summation-order differences (the engine's Winograd conv2 vs the oracle's
    # direct conv) reach a few 1e-3 of the running loss
    for p in coal:
        np.testing.assert_allclose(dev[p]["loss"][0, 0], ref[p]["loss"][0, 0], rtol=1e-2)
    # every entry: accuracies within 3 points, +-1 point on average; losses within 15 %
    accs = []
    for k in ref:
        for metric in ref[k]:
            d, r = dev[k][metric], ref[k][metric]
            ok = ~np.isnan(r)
            if metric.endswith("accuracy"):
                diff = np.abs(d[ok] - r[ok])
                assert np.all(diff <= 0.03), (k, metric, d, r)
                accs.extend(diff.tolist())
            else:
                np.testing.assert_allclose(d[ok], r[ok], rtol=0.15, err_msg=f"{k} {metric}")
    assert np.mean(accs) <= 0.01


@pytest.mark.parametrize("approach", ("fedavg", "seq-pure", "seqavg", "seq-with-final-agg"))
def test_history_vs_oracle(approach):
    sc = make_scenario(approach)
    eng = engine_for(sc)
    coal = (0, 1, 2)
    res = eng.evaluate([coal], return_details=True, record_history=True)
    acc, ref = oracle_history(sc, eng, coal, approach)
    compare(res["history"], ref, coal)
    assert abs(res["scores"][0] - acc) <= 0.03
    # recording reads, never perturbs: the same v(S) without it
    assert eng.evaluate([coal])[0] == res["scores"][0]


def test_singleton_history_vs_oracle():
    sc = make_scenario()
    eng = engine_for(sc)
    res = eng.evaluate([(1,)], return_details=True, record_history=True)
    _, ref = oracle_history(sc, eng, (1,), "fedavg")
    h = res["history"]
    assert set(h) == {1}
    for metric in METRICS:  # the last epoch at [0, 0], NaN elsewhere
        assert not np.isnan(h[1][metric][0, 0])
        assert np.isnan(h[1][metric]).sum() == h[1][metric].size - 1
    assert abs(h[1]["val_accuracy"][0, 0] - ref[1]["val_accuracy"][0, 0]) <= 0.03
    assert abs(h[1]["accuracy"][0, 0] - ref[1]["accuracy"][0, 0]) <= 0.03
    np.testing.assert_allclose(h[1]["loss"][0, 0], ref[1]["loss"][0, 0], rtol=0.15)


def test_scenario_run_history_and_federated_sbs():
    sc = make_scenario(E=3, M=4)
    sc.methods = ["Federated SBS linear", "Federated SBS quadratic", "Federated SBS constant"]
    sc.run()
    hist = sc.mpl.history.history
    assert set(hist) == {0, 1, 2, "mpl_model"}
    assert not np.isnan(hist[2]["val_accuracy"]).any()
    assert np.all(hist["mpl_model"]["val_accuracy"] > 0)
    df = sc.mpl.history.partners_to_dataframe()
    assert len(df) == 3 * 3 * 4 and not df["loss"].isna().any()
    # the scores are the reference's post-processing of that history
    E, M = 3, 4
    rel = np.stack([hist[p]["val_accuracy"] for p in range(3)], axis=-1).reshape(E * M, 3) \
        / hist["mpl_model"]["val_accuracy"].reshape(E * M)[:, None]
    rel = rel[int(np.round(E * M * 0.1)):int(np.round(E * M * 0.9))]
    lin, quad, const = sc.contributivity_list
    np.testing.assert_allclose(lin.contributivity_scores, np.arange(len(rel)).dot(rel), rtol=1e-12)
    np.testing.assert_allclose(quad.contributivity_scores, np.square(np.arange(len(rel))).dot(rel), rtol=1e-12)
    np.testing.assert_allclose(const.contributivity_scores, np.nanmean(rel, axis=0), rtol=1e-12)
    assert lin.name == "Federated step by step linear scores"
    assert abs(np.sum(const.normalized_scores) - 1.0) < 1e-12


@pytest.mark.parametrize("approach", ("fedavg", "seqavg"))
def test_cifar_history_vs_oracle(approach):
    from mplc.dataset import ArrayDataset, digits_as_cifar
    from mplc.scenario import Scenario
    from oracle import cifar_cnn as occ
    x, y = digits_as_cifar()
    ds = ArrayDataset(x[:1500], y[:1500], x[1500:], y[1500:], name="cifar10")
    sc = Scenario(3, [0.2, 0.5, 0.3], dataset=ds, minibatch_count=2, gradient_updates_per_pass_count=4, epoch_count=2,
                  is_early_stopping=False, multi_partner_learning_approach=approach).provision()
    eng = engine_for(sc)
    coal = (0, 1, 2)
    res = eng.evaluate([coal], return_details=True, record_history=True)
    d = sc.dataset
    data = occ.Data(d.x_train, d.y_train, d.x_val, d.y_val, d.x_test, d.y_test)
    ref = {}
    occ.coalition_value(data, [p.train_idx for p in sc.partners_list], [p.batch_size for p in sc.partners_list],
                        coal, seed=eng.seed, epochs=eng.epoch_count, M=eng.minibatch_count, approach=approach,
                        history=ref)
    compare(res["history"], ref, coal)
    assert eng.evaluate([coal])[0] == res["scores"][0]
