"""GPU: lockstep batches split over two HIP streams (CoalitionEngine.concurrent_batches, CnnBatchTrainer.
run_concurrent) give every coalition the value it gets in one batch, bit for bit (v(S) depends only on (S, seed)),
for the CIFAR10 and MNIST trainers."""
import itertools

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _engine(model):
    from mplc.dataset import Cifar10, Mnist
    from mplc.engine import CoalitionEngine
    from mplc.scenario import Scenario
    ds = Cifar10(synthetic=True, n_train=3000, n_test=500, signal=0.3) if model == "cifar10" else Mnist(synthetic=True, signal=0.2)
    sc = Scenario(6, [0.1, 0.15, 0.15, 0.2, 0.2, 0.2], dataset=ds, epoch_count=1, minibatch_count=2,
                  dataset_proportion=1.0 if model == "cifar10" else 0.1, is_early_stopping=False).provision()
    return CoalitionEngine.for_scenario(sc)


@pytest.mark.parametrize("model", ["cifar10", "mnist"])
def test_two_streams_bit_identical(model):
    eng = _engine(model)
    assert eng.concurrent_batches == 1  # opt-in
    coals = [c for k in range(1, 7) for c in itertools.combinations(range(6), k)][:40]
    eng.concurrent_batches = 1
    one = eng.evaluate(coals)
    eng.concurrent_batches = 2
    assert eng._concurrent_ok(coals, eng.epoch_count, eng.is_early_stopping, None, False)
    two = eng.evaluate(coals)
    assert np.array_equal(one, two), np.nonzero(one != two)
    assert len(np.unique(one)) > 5  # trained models, not a constant (small CIFAR runs stay near chance at E=1)
