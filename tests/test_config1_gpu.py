"""GPU: BASELINE config #1 exactly as the reference writes it, through the reference's command line.

Input: /root/reference/tests/config_end_to_end_test_contrib.yml, unchanged (tests/golden/
config_end_to_end_test_contrib.yml: MNIST, 2 partners [0.1, 0.9], basic random split, FedAvg, "Shapley values" and
"Independent scores", E=1, M=10, G=8, dataset_proportion 0.1), plus the 3-partner variant SURVEY 8 names for
BASELINE's "3 partners" ([0.2, 0.5, 0.3], tests/unit_tests.py:115-116), otherwise the same yml.

Data: MNIST cannot be downloaded here, so mnist.npz (MPLC_DATA_DIR) holds the engine's learnable synthetic MNIST
(mplc.dataset._synthetic_images: class templates + noise, signal 0.3, 60000 / 10000 rows) quantised to uint8 like
the real file; main.py loads it as it would the real one, and dataset_proportion 0.1 shortens it as the reference
does (mplc/dataset.py:83-106).  Signal 0.3 was chosen before the test (scripts/probe_config1_signal.py, oracle
only): the 0.9 partner learns (0.99+), the 0.1 partner (437 rows at bs 5) is still in the steep part (~0.27).

Checks:
  - every partner's rows and batch size equal the reference's own split (tests/golden/splits.json, cfg1_mnist_2p /
    cfg1b_mnist_3p: 437 / 3936 rows at bs 5 / 49; 874 / 2186 / 1312 at 10 / 27 / 16);
  - the reference test's assertions (tests/end_to_end_tests.py:54-73): 4 rows, and for each method the 0.1
    partner's score below the 0.9 partner's; for the 3-partner variant 6 rows and the 0.2 partner lowest;
  - v(S) of every coalition (the memo of the Shapley run) against the oracle (oracle/cnn.py: the same partition,
    keys and schedule, sequential like the reference): each coalition within the oracle's OWN spread over fp32
    summation orders widened by 1 pt (north star: +-1 pt), and the mean signed difference to the oracle's median
    within 1 pt.  The spread is the oracle run at 1, 2, 3, 4, 6, 8, 12 and 16 CPU threads (committed fixture
    tests/golden/oracle_spread_config1_*.json, scripts/oracle_spread.py) plus one live run at the box's thread
    count.  Why a spread: one epoch leaves some of these models in the steep part of learning, where a near-tie (a
    max-pool window or a ReLU input at ~0) breaks either way with the summation order.  Round 4's failing
    (0, 1) = 0.9585 (the band was then widened to 1.5 pt) is such a case: scripts/diag_config1.py
    on the box (profiles/r05_diag_config1.json) gave the fp32 oracle 0.9717 / 0.9597 / 0.9708 / 0.9712 / 0.9695 /
    0.9734 / **0.9585** / 0.9694 at 1 / 2 / 3 / 4 / 6 / 8 / 12 / 16 threads (fp64: 0.9718) - the device's value
    exactly, at 12 threads.  The band is back to spread + 1 pt;
  - deterministic numerics of the ragged bs-10 path: every FedAvg round of the coalitions
    with partner 0 (874 rows at bs 10: each round 8 steps of 10 and one of 7 or 8; partner 1's rounds end with 2
    or 3 samples at bs 27, partner 2's with 3 at bs 16) started from the device's global model, against the
    oracle's fp64 restatement of the same round (test_config1_three_partner_round_trajectories_vs_fp64).
"""
import os
from itertools import combinations

import numpy as np
import pandas as pd
import pytest

from spread_fixtures import golden_split, load_spread, oracle_values


def _dump_rounds(tag, errs):
    """Per-round (device, fp32-oracle) errors of a round-trajectory test, to $MPLC_TRAJ_DUMP/<tag>.json when set."""
    import json
    import os
    d = os.environ.get("MPLC_TRAJ_DUMP")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"{tag}.json"), "w") as f:
            json.dump(errs, f)

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
SIGNAL = 0.3


@pytest.fixture(scope="module")
def mnist_dir(tmp_path_factory):
    from mplc.dataset import _synthetic_images
    d = tmp_path_factory.mktemp("cfg1")
    x, y, xt, yt = _synthetic_images((28, 28, 1), 60000, 10000, 0, SIGNAL)
    q = lambda a: np.round(a[..., 0] * 255).astype(np.uint8)  # noqa: E731  (the real file's uint8 pixels)
    np.savez(d / "mnist.npz", x_train=q(x), y_train=np.argmax(y, 1).astype(np.uint8), x_test=q(xt),
             y_test=np.argmax(yt, 1).astype(np.uint8))
    return d


def _run_main(mnist_dir, yml_text, name):
    """main.py -f <yml> (the reference's command line); returns results.csv and the scenario it ran."""
    import main
    from mplc import scenario as scenario_mod
    ran = []
    orig = scenario_mod.Scenario.run

    def run(self):  # keep the scenario main.py builds, to compare its split and memo
        ran.append(self)
        return orig(self)
    with pytest.MonkeyPatch.context() as mp:
        mp.setenv("MPLC_DATA_DIR", str(mnist_dir))
        mp.chdir(mnist_dir)
        mp.setattr(scenario_mod.Scenario, "run", run)
        cfg = mnist_dir / name
        cfg.write_text(yml_text)
        assert main.main(["-f", str(cfg)]) == 0
    runs = sorted((mnist_dir / "experiments").glob("*end_to_end_test*"), key=lambda p: p.stat().st_mtime)
    assert len(ran) == 1
    return pd.read_csv(runs[-1] / "results.csv"), ran[0]


def _reference_yml():
    with open(os.path.join(HERE, "golden", "config_end_to_end_test_contrib.yml")) as f:
        return f.read()


@pytest.fixture(scope="module")
def run_2p(mnist_dir):
    return _run_main(mnist_dir, _reference_yml(), "config_end_to_end_test_contrib.yml")


@pytest.fixture(scope="module")
def run_3p(mnist_dir):
    text = _reference_yml().replace("partners_count:\n     - 2", "partners_count:\n     - 3")
    text = text.replace("- [0.1, 0.9]", "- [0.2, 0.5, 0.3]")
    assert "- [0.2, 0.5, 0.3]" in text and "     - 3" in text
    return _run_main(mnist_dir, text, "config_end_to_end_test_contrib_3p.yml")


def _check_split_images(sc, mnist_dir, tag):
    rec = golden_split(tag)
    with np.load(mnist_dir / "mnist.npz") as f:
        full = f["x_train"].reshape(-1, 28, 28, 1).astype("float32") / 255
    assert len(sc.partners_list) == len(rec["partners"])
    for p, gp in zip(sc.partners_list, rec["partners"]):
        assert len(p.train_idx) == len(gp["x_train"])
        assert p.batch_size == gp["batch_size"]
        # the partner's images are the reference's rows of the original 60000 (random images: no duplicates)
        assert np.array_equal(sc.dataset.x_train[p.train_idx], full[np.asarray(gp["x_train"])])


def _check_vs_oracle(sc, name):
    """Each coalition within the oracle's spread over summation orders + 1 pt; mean signed difference to the
    oracle's median within 1 pt."""
    import torch
    shap = next(c for c in sc.contributivity_list if c.name == "Shapley")
    rec = load_spread(name, sc)
    assert sc.engine.seed == rec.get("seed", 0)
    coals = [tuple(k) for k in rec["coalitions"]]
    n = len(sc.partners_list)
    assert set(k for k in shap.charac_fct_values if k) == set(coals) == \
        {k for r in range(1, n + 1) for k in combinations(range(n), r)}
    dev = np.array([shap.charac_fct_values[k] for k in coals])
    refs = [rec["fp32"][str(t)] for t in rec["threads"]]
    refs.append(oracle_values(sc, coals, torch.get_num_threads()))  # the box's own summation order
    refs = np.array(refs)
    lo, hi = refs.min(axis=0) - 0.01, refs.max(axis=0) + 0.01
    print(list(zip(coals, dev.tolist(), refs.min(axis=0).tolist(), refs.max(axis=0).tolist(), rec["fp64"])))
    assert abs(np.mean(dev - np.median(refs, axis=0))) <= 0.01, (coals, dev, refs)  # no systematic bias
    assert np.all((lo <= dev) & (dev <= hi)), (coals, dev, refs)
    return dev


def test_config1_reference_yml_unchanged(run_2p, mnist_dir):
    import yaml
    p = yaml.safe_load(_reference_yml())["scenario_params_list"][0]  # the reference's values, unchanged
    assert (p["partners_count"], p["amounts_per_partner"], p["epoch_count"], p["minibatch_count"],
            p["gradient_updates_per_pass_count"], p["dataset_proportion"]) == ([2], [[0.1, 0.9]], [1], [10], [8], [0.1])
    df, sc = run_2p
    assert (sc.epoch_count, sc.minibatch_count, sc.gradient_updates_per_pass_count) == (1, 10, 8)
    _check_split_images(sc, mnist_dir, "cfg1_mnist_2p")
    # tests/end_to_end_tests.py:54-73
    assert len(df) == 4
    for method in df.contributivity_method.unique():
        cur = df[df.contributivity_method == method]
        small = cur.loc[cur.dataset_fraction_of_partner == 0.1, "contributivity_score"].values
        big = cur.loc[cur.dataset_fraction_of_partner == 0.9, "contributivity_score"].values
        assert small < big, (method, small, big)
    dev = _check_vs_oracle(sc, "config1_2p")
    assert dev[1] > 0.9  # the 0.9 partner's model has learned


def test_config1_three_partner_variant(run_3p, mnist_dir):
    df, sc = run_3p
    _check_split_images(sc, mnist_dir, "cfg1b_mnist_3p")
    assert len(df) == 6
    for method in df.contributivity_method.unique():
        cur = df[df.contributivity_method == method].sort_values("dataset_fraction_of_partner")
        scores = cur["contributivity_score"].values
        assert scores[0] < scores[1] and scores[0] < scores[2], (method, cur)  # the 0.2 partner lowest
    _check_vs_oracle(sc, "config1_3p")


def test_config1_three_partner_round_trajectories_vs_fp64(run_3p):
    """Every one of the 10 FedAvg rounds of the coalitions holding partner 0 ((0, 1), (0, 2), (0, 1, 2)), each
    started from the device's global model at the round's start, against oracle/cnn.py fedavg_round(precise=True):
    the same round (keys, ragged batches, fresh Keras Adam per partner, data-volume average) with every tensor
    operation in fp64.  Per round and tensor the error on the round's update, ||dev - ref64|| / ||ref64 - start||,
    beside the fp32 oracle's own error (the largest over 2, 3 and the box's CPU threads).

    The errors are bimodal (profiles/r05_diag_config1.json, all four FedAvg coalitions, 40 rounds): ~1e-6 in a
    round without a near-tie - device and fp32 oracle alike - and 1e-4 .. 1e-2 in a round where a max-pool window or
    a ReLU input near 0 breaks the other way; such rounds hit the device and the oracle at different rounds.  So the
    gate is per coalition and tensor on the LOWER QUARTILE round (the clean-mode floor, the kernels' own rounding):
    device error <= 4x the fp32 oracle's, and at most 4 of the 10 rounds with any tensor outside 4x (measured 1, 1
    and 0 for these coalitions; 3 for (1, 2)).  A defect of the ragged path (a short batch averaged over bs instead
    of its count, a dropped remainder) would put every round at ~1e-1.  (Through round 6 the gate sat on the median
    round, which lies on the boundary of the two modes when about half the rounds meet a tie - config #3's (2, 9)
    test showed a 10x swing of the median from one tie round; tests/test_workload_gpu.py.  Quartile ratios with the
    round's final numerics 0.1 .. 1.3, profiles/r06_traj_rounds.json.)"""
    import torch
    from oracle import cnn as ocnn
    from mplc.engine import CoalitionEngine
    _, sc = run_3p
    eng = CoalitionEngine.for_scenario(sc, memory_budget_bytes=8 << 30, eval_budget_bytes=1 << 30)
    ds = sc.dataset
    data = ocnn.Data(ds.x_train, ds.y_train, ds.x_val, ds.y_val, ds.x_test, ds.y_test)
    prow = [p.train_idx for p in sc.partners_list]
    bs = [p.batch_size for p in sc.partners_list]
    assert [len(r) for r in prow] == [874, 2186, 1312] and bs == [10, 27, 16]
    M = sc.minibatch_count
    threads0 = torch.get_num_threads()
    report, bad = [], []
    for coal in [(0, 1), (0, 2), (0, 1, 2)]:
        st = eng.trainer.prepare([coal], 1)
        errs = []  # [round] -> {tensor: (dev, cpu)}
        for m in range(M):
            start = st.glob[0].cpu().numpy().copy()
            for s in range(m * st.round_len, (m + 1) * st.round_len):
                st.step(s)
            st.aggregate(epoch_end=(m == M - 1))
            torch.cuda.synchronize()
            dev = st.glob[0].cpu().numpy()
            glob = ocnn.unpack(start)
            g64 = ocnn.fedavg_round(data, prow, bs, coal, glob, seed=eng.seed, M=M, e=0, m=m, precise=True)
            g32s = []
            for th in sorted({2, 3, threads0}):
                torch.set_num_threads(th)
                g32s.append(ocnn.fedavg_round(data, prow, bs, coal, glob, seed=eng.seed, M=M, e=0, m=m))
            torch.set_num_threads(threads0)
            row = {}
            for name, (off, shape) in ocnn.OFF.items():
                n = int(np.prod(shape))
                ref = g64[name].numpy().reshape(-1)
                upd = np.linalg.norm(ref - start[off:off + n].astype(np.float64))
                e_dev = np.linalg.norm(dev[off:off + n].astype(np.float64) - ref) / upd
                e_cpu = max(np.linalg.norm(g[name].numpy().reshape(-1).astype(np.float64) - ref) / upd for g in g32s)
                row[name] = (float(e_dev), float(e_cpu))
            errs.append(row)
        del st
        outliers = sum(any(r[k][0] > 4 * r[k][1] for k in r) for r in errs)
        _dump_rounds(f"config1_{'_'.join(map(str, coal))}", errs)
        for name in ocnn.OFF:
            q_dev = float(np.percentile([r[name][0] for r in errs], 25))
            q_cpu = float(np.percentile([r[name][1] for r in errs], 25))
            report.append((coal, name, q_dev, q_cpu))
            if not q_dev <= 4 * q_cpu:
                bad.append(report[-1])
        report.append((coal, "outlier rounds", outliers))
        if outliers > 4:
            bad.append(report[-1])
    print(report)
    assert not bad, (bad, report)
