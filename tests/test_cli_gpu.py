"""GPU: the reference's command line end to end (main.py -f <yaml> -> experiments/<name>_<date>/results.csv),
ported from tests/end_to_end_tests.py:54-73 (test_contrib): 2 partners [0.1, 0.9], "Shapley values" and
"Independent scores" -> 4 rows, the 10% partner scores below the 90% partner for each method.
Data: a local mnist.npz written from sklearn's digits (MPLC_DATA_DIR), since MNIST cannot be downloaded."""
import os

import numpy as np
import pandas as pd
import pytest

pytestmark = pytest.mark.gpu

CONFIG = """experiment_name: end_to_end_test_contrib
n_repeats: 1
scenario_params_list:
 - dataset_name:
    'mnist':
     - 'random_initialization'
   partners_count:
     - 2
   amounts_per_partner:
     - [0.1, 0.9]
   samples_split_option:
     - ['basic', 'random']
   multi_partner_learning_approach:
     - 'fedavg'
   methods:
    - ["Shapley values", "Independent scores"]
   epoch_count:
     - 2
   minibatch_count:
     - 4
   gradient_updates_per_pass_count:
     - 4
   dataset_proportion:
     - 1
"""


@pytest.fixture()
def digits_mnist(tmp_path, monkeypatch):
    from mplc.dataset import digits_as_mnist
    x, y = digits_as_mnist()
    xi = np.round(x[..., 0] * 255).astype(np.uint8)
    yi = np.argmax(y, 1).astype(np.uint8)
    np.savez(tmp_path / "mnist.npz", x_train=xi[:1500], y_train=yi[:1500], x_test=xi[1500:], y_test=yi[1500:])
    monkeypatch.setenv("MPLC_DATA_DIR", str(tmp_path))
    monkeypatch.chdir(tmp_path)
    return tmp_path


def test_main_contrib_results_csv(digits_mnist):
    import main
    cfg = digits_mnist / "config_end_to_end_test_contrib.yml"
    cfg.write_text(CONFIG)
    assert main.main(["-f", str(cfg)]) == 0
    runs = sorted((digits_mnist / "experiments").glob("*end_to_end_test*"), key=lambda p: p.stat().st_ctime)
    df = pd.read_csv(runs[-1] / "results.csv")
    assert len(df) == 4
    assert df["mpl_test_score"].min() > 0.5
    for method in df.contributivity_method.unique():
        cur = df[df.contributivity_method == method]
        small = cur.loc[cur.dataset_fraction_of_partner == 0.1, "contributivity_score"].values
        big = cur.loc[cur.dataset_fraction_of_partner == 0.9, "contributivity_score"].values
        assert small < big, (method, small, big)
    assert set(df.columns) >= {"scenario_name", "dataset_name", "partners_count", "contributivity_method",
                               "contributivity_scores", "first_characteristic_calls_count", "partner_id",
                               "random_state", "scenario_id"}
    assert (runs[-1] / "info.log").exists()


def test_persisted_table_skips_training(digits_mnist):
    from mplc.dataset import Mnist
    from mplc.scenario import Scenario
    f = str(digits_mnist / "values.npz")

    def run():
        sc = Scenario(3, [0.2, 0.5, 0.3], dataset=Mnist(synthetic=False), minibatch_count=2, epoch_count=1,
                      methods=["Shapley values", "TMCS"], coalition_values_file=f)
        np.random.seed(0)
        sc.run()
        return sc
    a = run()
    b = run()
    assert b.engine is None or b.engine.stats["coalitions"] == 0  # every v(S) came from the table
    for ca, cb in zip(a.contributivity_list, b.contributivity_list):
        assert np.array_equal(ca.contributivity_scores, cb.contributivity_scores)
        assert ca.first_charac_fct_calls_count == cb.first_charac_fct_calls_count
