"""GPU: config #4's SMCS half at the config's own 20 partners.

Stratified Monte-Carlo Shapley (mplc/contributivity.py:727-819) on the HIP engine with config #4's 20-partner
partition ([0.05] * 19 + [0.05], FedAvg, E=1, numpy seed 0) on a reduced CIFAR10-shaped set (5,000 training rows
after the 90/10 split, 1,000 test rows, class templates at signal 0.4) and a short training schedule (M=2, G=2:
batch size 50, 4 to 5 steps per partner fit), so that the 21,553 coalition fits the stopping rule needs (780
sampling iterations, as at full size) train in a minute: what is tested is the estimator at 20 partners on the engine, not the training schedule
(bench.py --leg cifar --method SMCS runs config #4's own M=20, G=8 on the full-size set; at 250 rows per partner
that schedule would be batch size 1, ~200 steps per fit).  The v(S) values the batched, speculatively planned run
trained are fed to the reference's sequential loop (one fit per coalition through the plug-in protocol, no
planning): scores, std, call count, memo order and increments must be identical bit for bit, as
tests/test_workload_gpu.py checks at 10 partners."""
import types

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cifar20_small():
    from mplc.dataset import Cifar10
    from mplc.scenario import Scenario
    amounts = [0.05] * 19 + [float(1 - np.sum([0.05] * 19))]
    ds = Cifar10(synthetic=True, signal=0.4, n_train=5556, n_test=1000)
    sc = Scenario(20, amounts, dataset=ds, minibatch_count=2, gradient_updates_per_pass_count=2, epoch_count=1,
                  is_early_stopping=False)
    return sc.provision()


def test_config4_smcs_20_partners_batched_equals_sequential_reference_loop(cifar20_small, monkeypatch):
    import mplc.multi_partner_learning as mpl_mod
    from mplc.contributivity import Contributivity
    sc = cifar20_small
    assert len(sc.dataset.x_train) == 5000 and len(sc.partners_list) == 20
    assert sorted({p.batch_size for p in sc.partners_list}) == [50]
    np.random.seed(0)
    c = Contributivity(scenario=sc)
    c.compute_contributivity("SMCS")
    eng = sc.engine
    print("SMCS 20 partners:", c.first_charac_fct_calls_count, "coalitions counted,", eng.stats, "iterations",
          getattr(c, "sampling_iterations", None))
    assert c.first_charac_fct_calls_count > 2000  # a real stratified sampling run, many strata per player
    table = dict(sc.coalition_values)
    calls = []

    class TableMPL:  # the reference's plug-in protocol, one fit per coalition (mplc/contributivity.py:100-114)
        def __init__(self, scenario, partners_list=None, partner=None, **kw):
            if partner is not None:
                partners_list = [partner]
            self.ids = tuple(sorted(int(p.id) for p in partners_list))
            self.history = types.SimpleNamespace(score=None)

        def fit(self):
            calls.append(self.ids)
            self.history.score = table[self.ids]

    monkeypatch.setattr(mpl_mod, "SinglePartnerLearning", TableMPL)
    plain = types.SimpleNamespace(partners_list=sc.partners_list, multi_partner_learning_approach=TableMPL)
    np.random.seed(0)
    ref = Contributivity(scenario=plain)
    ref.compute_contributivity("SMCS")
    assert ref.name == c.name == "Stratified MC Shapley"
    assert np.array_equal(ref.contributivity_scores, c.contributivity_scores)
    assert np.array_equal(ref.scores_std, c.scores_std)
    assert ref.first_charac_fct_calls_count == c.first_charac_fct_calls_count == len(calls)
    assert list(ref.charac_fct_values) == list(c.charac_fct_values)
    assert all(np.array_equal(ref.increments_values[i], c.increments_values[i]) for i in range(20))
    assert np.all(np.isfinite(c.contributivity_scores))
