"""GPU: early-stopping batch compaction is result-neutral.

With early stopping (mplc/multi_partner_learning.py:177-193 FedAvg rule, Keras EarlyStopping for singletons
:247-260) coalitions of one lockstep batch stop at different epochs.  CnnBatchTrainer compacts the batch once the
live replicas drop to `compact_live_share` of it: the stopped coalitions' final models are test-evaluated and the
live ones continue in a smaller batch with their coalition rows, replica rows, optimizer state and step schedule
gathered unchanged.  Every v(S), realised epoch count and early-stopping trace must therefore be BIT-IDENTICAL to
the same batch trained whole (compact_live_share = 0).  compact_live_share = 1 compacts whenever any replica is
idle: the most compactions, each at a different step.
Cases: MNIST on sklearn digits with 60 % of the labels randomised (the models overfit and the rules fire at
different epochs), 4 partners of unequal size, all 15 coalitions; CIFAR10-shaped random data (RMSprop state and
the keyed dropout masks must survive the gather), 3 partners, all 7 coalitions."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _both(eng, coals):
    out = {}
    for share in (0.0, 1.0):
        eng.compact_live_share = share
        before = eng.stats.get("compactions", 0)
        res = eng.evaluate(coals, return_details=True)
        out[share] = (res, eng.stats.get("compactions", 0) - before)
    return out


def _check(out, min_compactions=2, spread=True):
    (whole, n0), (comp, n1) = out[0.0], out[1.0]
    assert n0 == 0 and n1 >= min_compactions, (n0, n1)
    assert np.array_equal(whole["scores"], comp["scores"]), (whole["scores"], comp["scores"])
    assert np.array_equal(whole["epochs_done"], comp["epochs_done"])
    assert whole["es_val_loss"] == comp["es_val_loss"]
    if spread:
        assert len(set(whole["epochs_done"].tolist())) >= 2, whole["epochs_done"]  # stops at different epochs


def test_mnist_compaction_bit_identical():
    from itertools import combinations
    from mplc.dataset import ArrayDataset, digits_as_mnist
    from mplc.engine import CoalitionEngine
    from mplc.scenario import Scenario
    x, y = digits_as_mnist()
    y = np.argmax(np.array(y), 1)
    rng = np.random.default_rng(0)
    flip = rng.random(1500) < 0.6
    y[np.arange(1500)[flip]] = rng.integers(0, 10, size=int(flip.sum()))
    ds = ArrayDataset(x[:1500], y[:1500], x[1500:], y[1500:])
    sc = Scenario(4, [0.1, 0.2, 0.3, 0.4], dataset=ds, minibatch_count=2, gradient_updates_per_pass_count=16,
                  epoch_count=24, is_early_stopping=True).provision()
    eng = CoalitionEngine.for_scenario(sc, memory_budget_bytes=8 << 30, eval_budget_bytes=1 << 30)
    coals = [c for r in range(1, 5) for c in combinations(range(4), r)]
    out = _both(eng, coals)
    print(out[0.0][0]["epochs_done"], out[1.0][1])
    _check(out)


def test_cifar_compaction_bit_identical():
    from itertools import combinations
    from mplc.dataset import Cifar10
    from mplc.engine import CoalitionEngine
    from mplc.scenario import Scenario
    sc = Scenario(3, [0.2, 0.3, 0.5], dataset=Cifar10(synthetic=True, signal=0.0, n_train=3000, n_test=1000),
                  minibatch_count=2, gradient_updates_per_pass_count=8, epoch_count=14,
                  is_early_stopping=True).provision()
    eng = CoalitionEngine.for_scenario(sc, memory_budget_bytes=8 << 30, eval_budget_bytes=1 << 30)
    coals = [c for r in range(1, 4) for c in combinations(range(3), r)]
    out = _both(eng, coals)
    print(out[0.0][0]["epochs_done"], out[1.0][1])
    _check(out, min_compactions=1, spread=False)  # random labels: the rules fire at epoch 11, at different steps
