"""GPU: lockstep batches split over two HIP streams (CoalitionEngine.concurrent_batches, CnnBatchTrainer.
run_concurrent) give every coalition the value it gets in one batch, bit for bit (v(S) depends only on (S, seed)),
for the CIFAR10 and MNIST trainers.  Two streams are the CIFAR10 default; a batch the bench's kernel timer samples
runs as one lockstep batch on one stream, so its launches are timed without overlap."""
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
    assert eng.concurrent_batches == (2 if model == "cifar10" else 1)  # the default
    coals = [c for k in range(1, 7) for c in itertools.combinations(range(6), k)][:40]
    eng.concurrent_batches = 1
    one = eng.evaluate(coals)
    eng.concurrent_batches = 2
    assert eng._concurrent_ok(coals, eng.epoch_count, eng.is_early_stopping, None, False)
    two = eng.evaluate(coals)
    assert np.array_equal(one, two), np.nonzero(one != two)
    assert len(np.unique(one)) > 5  # trained models, not a constant (small CIFAR runs stay near chance at E=1)


def test_timed_batch_runs_as_one_lockstep_batch():
    """With the kernel timer switched on at the batch's start (bench.py's progress hook), a two-stream batch trains
    as one batch: one launch of every kernel per step, each covering all the batch's replicas, the values
    unchanged; the start is reported once."""
    from mplc.profiling import KernelTimer
    from mplc.cifar import KERNEL_IDS
    from mplc.cnn import schedule_geometry
    eng = _engine("cifar10")
    coals = [c for k in range(1, 7) for c in itertools.combinations(range(6), k)][:40]
    eng.concurrent_batches = 1
    one = eng.evaluate(coals)
    eng.concurrent_batches = 2
    timer = KernelTimer("all", list(KERNEL_IDS), stash=True)
    starts = []

    def progress(s, total, R):
        if s == 0:
            starts.append((total, R))
            eng.profiler = timer
    eng.progress = progress
    two = eng.evaluate(coals)
    eng.progress, eng.profiler = None, None
    assert np.array_equal(one, two)
    steps = schedule_geometry(eng, [tuple(c) for c in coals], eng.epoch_count)[2]
    assert starts == [(steps, sum(len(c) for c in coals))]
    assert timer.launches("dense5_bwd") == steps  # one launch per step: not one per part
    units = eng.model_impl.algorithmic_units(timer.stash)
    assert units["samples"] == sum(eng.partner_sizes[p] for c in coals for p in c) * eng.epoch_count


def test_two_stream_batches_stay_within_the_memory_budget():
    """the caching allocator keeps freed blocks per stream, so blocks the two-stream parts left on the
    side streams cannot serve a batch on the caller's stream (the bench's timer-sampled batches) - without a release
    the device would hold both, about twice memory_budget_bytes.  CoalitionEngine._within_budget returns the cache
    when idle + need would pass the budget: the peak reserved memory of a run alternating two-stream and one-stream
    batches stays within the resident data + the training budget + the evaluation budget (+ allocator rounding)."""
    import torch
    from mplc.dataset import Cifar10
    from mplc.engine import CoalitionEngine
    from mplc.profiling import KernelTimer
    from mplc.cifar import KERNEL_IDS
    from mplc.scenario import Scenario
    ds = Cifar10(synthetic=True, n_train=3000, n_test=500, signal=0.3)
    sc = Scenario(6, [0.1, 0.15, 0.15, 0.2, 0.2, 0.2], dataset=ds, epoch_count=1, minibatch_count=2,
                  is_early_stopping=False).provision()
    coals = [c for k in range(1, 7) for c in itertools.combinations(range(6), k)][:60]
    probe = CoalitionEngine.for_scenario(sc)
    per = max(len(c) * probe.replica_bytes(max(probe.batch_sizes[p] for p in c)) for c in coals)
    budget, eval_budget = 12 * per, 64 << 20
    del probe
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    eng = CoalitionEngine.for_scenario(sc, memory_budget_bytes=budget, eval_budget_bytes=eval_budget)
    assert eng.concurrent_batches == 2 and len(eng.plan_batches(coals)) >= 3
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    first = eng.evaluate(coals)  # two-stream batches: the side streams keep their parts' blocks cached
    timer = KernelTimer("all", list(KERNEL_IDS), stash=True)

    def progress(s, total, R):
        if s == 0:
            eng.profiler = timer  # every batch sampled: one lockstep batch on the caller's stream
    eng.progress = progress
    second = eng.evaluate(coals)
    eng.progress, eng.profiler = None, None
    third = eng.evaluate(coals)  # back to two streams
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_reserved() - base
    print(f"budget {budget >> 20} MiB + eval {eval_budget >> 20} MiB, peak reserved above the data {peak >> 20} MiB, "
          f"cache releases {eng.stats.get('cache_releases', 0)}")
    assert np.array_equal(first, second) and np.array_equal(first, third)
    assert eng.stats.get("cache_releases", 0) >= 1
    assert peak <= 1.1 * (budget + eval_budget) + (64 << 20), (peak, budget)
