"""Host-side accounting of the bench's per-kernel rates (bench.py kernel_table, MnistModel.algorithmic_units):
the dense kernels' algorithmic HBM bytes follow the Adam schedule flags exactly as csrc/mnist_cnn.hip
dense1_bwd_adam_kernel moves them.  No GPU needed."""
import os
import sys

import pytest

torch = pytest.importorskip("torch")

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "distributed-learning-contributivity_amd"))

from mplc import cnn  # noqa: E402

W3 = 9216 * 128 * 4


def test_dense_bytes_follow_adam_schedule():
    L = cnn.ADAM_LAST
    # replicas: fresh step (t=1), idle, step 2, step 5, last step of an optimizer (t=8), t=1 that is also last
    cnt = torch.tensor([27, 0, 27, 10, 27, 5], dtype=torch.int32)
    at = torch.tensor([1, 0, 2, 5, 8 | L, 1 | L], dtype=torch.int32)
    src = torch.full((6,), -1, dtype=torch.int32)
    u = cnn.MnistModel.algorithmic_units([(cnt, at, src)])
    per_sample_bwd = 2 * 9216 * 4 + 128 * 4
    # W3 read+write (2) + moments: t1 -> write g (1); t2 -> read g, write m, v (3); t5 -> 4; last t8 -> read 2;
    # t1 last -> nothing
    moments = [1, None, 3, 4, 2, 0]
    exp = sum((2 + m) * W3 + c * per_sample_bwd for c, m in zip([27, 0, 27, 10, 27, 5], moments) if m is not None)
    assert u["dense1_bwd_adam_bytes"] == exp
    assert u["dense_fwd_bytes"] == 5 * W3 + 96 * (9216 * 4 + 128 * 4)
    assert u["samples"] == 96


def test_kernel_table_picks_rates():
    import bench

    class FakeTimer:
        def total_ms(self, k):
            return {"dense1_bwd_adam": 20.0, "conv_bwd_data": 10.0}.get(k, 1.0)

        def launches(self, k):
            return 2

    units = {"samples": 1000.0, "dense1_bwd_adam_bytes": 1.2e11, "dense_fwd_bytes": 3e10}
    tab = bench.kernel_table(FakeTimer(), units)
    d1 = tab["dense1_bwd_adam"]
    assert d1["bound"] == "hbm" and d1["achieved"] == pytest.approx(1.2e11 / 0.02 / 1e9)
    assert d1["frac"] == pytest.approx(d1["achieved"] / 8000.0, abs=1e-4)
    cb = tab["conv_bwd_data"]
    assert cb["achieved"] == pytest.approx(1000 * bench.CONV_BWD_DATA_FLOP_PER_SAMPLE / 0.01 / 1e12, abs=0.01)
    assert "frac" not in tab["head"]
    assert sum(e["time_share"] for e in tab.values()) == pytest.approx(1.0, abs=1e-3)


def test_shared_coalition_rows_count_once():
    """A FedAvg round's first step: the replicas of a coalition read W3 from one coalition row."""
    cnt = torch.tensor([27, 27, 27, 10], dtype=torch.int32)
    at = torch.tensor([1, 1, 1, 1], dtype=torch.int32)
    src = torch.tensor([4, 4, 4, 7], dtype=torch.int32)  # coalition 4 has three partners, coalition 7 one
    u = cnn.MnistModel.algorithmic_units([(cnt, at, src)])
    per_sample_bwd = 2 * 9216 * 4 + 128 * 4
    # W3 write + g write per replica, two distinct coalition rows read
    assert u["dense1_bwd_adam_bytes"] == 4 * 2 * W3 + 91 * per_sample_bwd + 2 * W3
    assert u["dense_fwd_bytes"] == 91 * (9216 * 4 + 128 * 4) + 2 * W3


def test_steps_of_batches_with_different_replica_counts():
    """A job split into several lockstep batches (memory budget) stashes per-step schedules of different
    lengths: the totals are the sums of the per-step counts (torch.stack raised here)."""
    L = cnn.ADAM_LAST
    a = (torch.tensor([27, 27, 0], dtype=torch.int32), torch.tensor([1, 2, 0], dtype=torch.int32),
         torch.tensor([3, -1, -1], dtype=torch.int32))
    b = (torch.tensor([11, 27, 27, 5, 9], dtype=torch.int32), torch.tensor([3, 4 | L, 1, 1, 2], dtype=torch.int32),
         torch.tensor([-1, -1, 0, 0, -1], dtype=torch.int32))
    both = cnn.MnistModel.algorithmic_units([a, b])
    ua, ub = cnn.MnistModel.algorithmic_units([a]), cnn.MnistModel.algorithmic_units([b])
    for k in ("samples", "dense1_bwd_adam_bytes", "dense_fwd_bytes"):
        assert both[k] == ua[k] + ub[k]
    assert both["samples"] == 27 + 27 + 11 + 27 + 27 + 5 + 9
    # batch b's step: coalition row 0 read once by its two first-step replicas
    per_sample_fwd = 9216 * 4 + 128 * 4
    assert ub["dense_fwd_bytes"] == 3 * W3 + W3 + 79 * per_sample_fwd  # three own rows + the shared one


def test_cifar_table_puts_conv1_on_its_hbm_roof():
    """conv1 (K = 27) sits under the fp32 MFMA / HBM ridge: its row is HBM-bound on its compulsory bytes, with the
    MFMA rate beside it; the Winograd convolutions stay MFMA-bound."""
    import bench
    from mplc.cifar import BYTES_PER_SAMPLE, FLOP_PER_SAMPLE

    class FakeTimer:
        def total_ms(self, k):
            return 2.0

        def launches(self, k):
            return 4

    units = {"samples": 10000.0, "dense5_bwd_bytes": 1e10, "dense5_fwd_bytes": 2e9}
    tab = bench.cifar_kernel_table(FakeTimer(), units)
    c1 = tab["conv1_fwd"]
    assert c1["bound"] == "hbm" and c1["unit"] == "GB/s"
    assert c1["achieved"] == pytest.approx(10000 * BYTES_PER_SAMPLE["conv1_fwd"] / 0.002 / 1e9, rel=1e-6)
    assert FLOP_PER_SAMPLE["conv1_fwd"] / BYTES_PER_SAMPLE["conv1_fwd"] < bench.FP32_MFMA_PEAK_TFLOPS / bench.HBM_PEAK_GBS * 1e3
    assert c1["mfma_rate"]["achieved"] == pytest.approx(10000 * FLOP_PER_SAMPLE["conv1_fwd"] / 0.002 / 1e12, abs=0.01)
    assert tab["conv1_wgrad"]["bound"] == "hbm" and tab["conv4_fwd"]["bound"] == "mfma"
    assert tab["dense5_bwd"]["bound"] == "hbm"


def test_tutorial_leg_is_the_reference_notebook_workload():
    """bench.py's tutorial leg (vs_baseline against the reference's one published timing) runs the notebook's
    experiment: notebooks/tutorials/Tutorial-2_Add_contributivity_measurement.ipynb prints the partner split of its
    Scenario(3, [0.001, 0.699, 0.3], MNIST, epoch_count=10, minibatch_count=3) as 43 / 30573 / 13122 samples
    (output lines 546-549) and its time, 1525.8 s for the 7 coalitions of exact Shapley.  The same split comes out
    of this package's split_data on the synthetic MNIST at the full sizes."""
    import bench
    from mplc.dataset import Mnist
    from mplc.scenario import Scenario
    assert (bench.REFERENCE_TUTORIAL_S, bench.REFERENCE_TUTORIAL_COALITIONS) == (1525.8, 7)
    sc = Scenario(3, [0.001, 0.699, 0.3], dataset=Mnist(synthetic=True, signal=0.2), epoch_count=10,
                  minibatch_count=3).provision()
    assert [len(p.y_train) for p in sc.partners_list] == [43, 30573, 13122]
    # batch size = rows / (minibatch_count * gradient_updates_per_pass_count 8), at least 1
    assert [p.batch_size for p in sc.partners_list] == [1, 1273, 546]
    # Tutorial-1_Run_your_first_scenario.ipynb (the leg's timed grand-coalition fit, 179.283 s): its printed split
    assert bench.REFERENCE_TUTORIAL1_FIT_S == 179.283
    sc1 = Scenario(3, [0.2, 0.5, 0.3], dataset=Mnist(synthetic=True, signal=0.2), epoch_count=10, minibatch_count=3,
                   dataset_proportion=0.1).provision()
    assert [len(p.y_train) for p in sc1.partners_list] == [874, 2186, 1312]
