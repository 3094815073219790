"""CPU: the reference's experiment YAML schema and results layer (mplc/utils.py, main.py, to_dataframe)
and the persisted v(S) table.  The reference's own config files are the fixtures (tests/golden/*.yml)."""
import os

import numpy as np
import pytest

from mplc import utils

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_contrib_config_expands_like_the_reference():
    cfg = utils.load_cfg(os.path.join(GOLDEN, "config_end_to_end_test_contrib.yml"))
    assert cfg["experiment_name"] == "end_to_end_test_contrib" and cfg["n_repeats"] == 1
    sl = utils.get_scenario_params_list(cfg["scenario_params_list"])
    assert len(sl) == 1
    sc = sl[0]
    assert sc["dataset_name"] == "mnist" and sc["init_model_from"] == "random_initialization"
    assert sc["partners_count"] == 2 and sc["amounts_per_partner"] == [0.1, 0.9]
    assert sc["methods"] == ["Shapley values", "Independent scores"]
    assert sc["samples_split_option"] == ["basic", "random"] and sc["dataset_proportion"] == 0.1


def test_mnist_and_reference_configs_cartesian_product():
    cfg = utils.load_cfg(os.path.join(GOLDEN, "config_end_to_end_test_mnist.yml"))
    sl = utils.get_scenario_params_list(cfg["scenario_params_list"])
    assert [s["multi_partner_learning_approach"] for s in sl] == ["fedavg", "seq-pure"]
    cfg = utils.load_cfg(os.path.join(GOLDEN, "config_reference.yml"))
    sl = utils.get_scenario_params_list(cfg["scenario_params_list"])
    # block 1: 2 datasets x 3 splits x 4 approaches x 2 aggregations; block 2: 2 aggregations
    assert len(sl) == 2 * 3 * 4 * 2 + 2


def test_bad_lengths_raise():
    with pytest.raises(Exception, match="amounts_per_partner"):
        utils.get_scenario_params_list([{"dataset_name": ["mnist"], "partners_count": [3],
                                         "amounts_per_partner": [[0.5, 0.5]],
                                         "samples_split_option": [["basic", "random"]]}])


def test_duplicate_yaml_keys_are_an_error(tmp_path):
    p = tmp_path / "dup.yml"
    p.write_text("experiment_name: a\nexperiment_name: b\n")
    with pytest.raises(ValueError, match="duplicated"):
        utils.load_cfg(str(p))


def test_result_folder_and_yaml_copy(tmp_path):
    src = os.path.join(GOLDEN, "config_end_to_end_test_contrib.yml")
    cfg = utils.get_config_from_file(src, root=tmp_path)
    p = cfg["experiment_path"]
    assert p.exists() and p.name.startswith("end_to_end_test_contrib_") and (p / os.path.basename(src)).exists()
    cfg2 = utils.get_config_from_file(src, root=tmp_path)
    assert cfg2["experiment_path"] != p  # "_bis" when the minute-stamped folder exists


def _scenario():
    from mplc.dataset import ArrayDataset
    from mplc.scenario import Scenario
    rng = np.random.default_rng(0)
    x = rng.random((200, 28, 28, 1), dtype=np.float32)
    y = np.eye(10, dtype=np.float32)[rng.integers(0, 10, 200)]
    ds = ArrayDataset(x[:150], y[:150], x[150:], y[150:])
    return Scenario(3, [0.2, 0.5, 0.3], dataset=ds, minibatch_count=2, epoch_count=1).provision()


def test_persisted_table_round_trip_and_fingerprint(tmp_path):
    sc = _scenario()
    sc.coalition_values = {(0,): 0.25, (0, 2): 0.5, (0, 1, 2): 0.75}
    f = str(tmp_path / "v.npz")
    sc.save_coalition_values(f)
    sc2 = _scenario()
    assert sc2.load_coalition_values(f) == 3
    assert sc2.coalition_values == {(0,): 0.25, (0, 2): 0.5, (0, 1, 2): 0.75}
    with np.load(f, allow_pickle=False) as z:
        assert sorted(int(m) for m in z["masks"]) == [0b1, 0b101, 0b111]
    sc3 = _scenario()
    sc3.epoch_count = 2  # another training configuration: the table must not be reused
    with pytest.raises(ValueError):
        sc3.load_coalition_values(f)
    assert sc3.load_coalition_values(str(tmp_path / "none.npz"), missing_ok=True) == 0
