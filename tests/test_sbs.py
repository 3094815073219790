"""CPU: Federated step-by-step scores (mplc/contributivity.py:1015-1115) reproduce the reference on the
learning histories of tests/golden/sbs.json (bit for bit: same numpy operations), and the History object
(mplc/mpl_utils.py:11-45) keeps the reference's layout and DataFrame export."""
import json
import os
import types

import numpy as np
import pytest

import mplc.multi_partner_learning as mpl_mod
from mplc.contributivity import Contributivity

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "sbs.json")
METHODS = ("Federated SBS linear", "Federated SBS quadratic", "Federated SBS constant")

with open(GOLDEN) as f:
    CASES = json.load(f)["data"]


def scenario_for(case, approach=mpl_mod.FederatedAverageLearning):
    P, E, M = case["P"], case["E"], case["M"]
    hist = {i: {m: np.asarray(case["partners"][i], dtype=float) if m == "val_accuracy" else np.full((E, M), np.nan)
                for m in mpl_mod.History.metrics} for i in range(P)}
    hist["mpl_model"] = {"val_accuracy": np.asarray(case["collective"], dtype=float), "val_loss": np.zeros((E, M))}
    h = mpl_mod.History()
    h.history = hist
    mpl = types.SimpleNamespace(history=h, partners_count=P, epoch_count=E, minibatch_count=M)
    return types.SimpleNamespace(partners_list=[types.SimpleNamespace(id=i) for i in range(P)], mpl=mpl,
                                 multi_partner_learning_approach=approach)


@pytest.mark.parametrize("ci", range(len(CASES)))
@pytest.mark.parametrize("method", METHODS)
def test_sbs_matches_reference(ci, method):
    case = CASES[ci]
    exp = case[method]
    c = Contributivity(scenario=scenario_for(case))
    c.compute_contributivity(method)
    assert c.name == exp["name"]
    assert np.array_equal(np.asarray(c.contributivity_scores), np.asarray(exp["scores"]), equal_nan=True)
    assert np.array_equal(np.asarray(c.normalized_scores), np.asarray(exp["normalized"]), equal_nan=True)
    assert np.array_equal(np.asarray(c.scores_std), np.asarray(exp["std"]))
    assert c.first_charac_fct_calls_count == 0  # no coalition is evaluated


def test_sbs_warns_for_non_fedavg_approach(caplog):
    c = Contributivity(scenario=scenario_for(CASES[0], approach=mpl_mod.SequentialLearning))
    with caplog.at_level("WARNING", logger="mplc"):
        c.compute_contributivity("Federated SBS constant")
    assert "only suited for federated averaging" in caplog.text
    assert np.array_equal(c.contributivity_scores, CASES[0]["Federated SBS constant"]["scores"])


def test_sbs_without_history_is_an_error():
    sc = types.SimpleNamespace(partners_list=[types.SimpleNamespace(id=0), types.SimpleNamespace(id=1)], mpl=None,
                               multi_partner_learning_approach=mpl_mod.FederatedAverageLearning)
    with pytest.raises(RuntimeError, match="learning history"):
        Contributivity(scenario=sc).compute_contributivity("Federated SBS linear")


def test_history_partners_to_dataframe_layout():
    sc = scenario_for(CASES[0])
    df = sc.mpl.history.partners_to_dataframe()
    P, E, M = CASES[0]["P"], CASES[0]["E"], CASES[0]["M"]
    assert list(df.columns) == ["Partner", "Epoch", "Minibatch", "val_accuracy", "val_loss", "loss", "accuracy"]
    assert len(df) == P * E * M
    row = df[(df.Partner == 1) & (df.Epoch == 2) & (df.Minibatch == 3)].iloc[0]
    assert row.val_accuracy == CASES[0]["partners"][1][2][3]
    assert np.isnan(row.loss)


def test_pvrl_and_lflip_stay_out_of_scope():
    c = Contributivity(scenario=scenario_for(CASES[0]))
    for m in ("PVRL", "LFlip"):
        with pytest.raises(NotImplementedError):
            c.compute_contributivity(m)
