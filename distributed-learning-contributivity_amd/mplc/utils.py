"""Experiment configuration and logging helpers - drop-in for mplc/utils.py (used by main.py).

YAML experiment files keep the reference's schema (experiment_name, n_repeats, scenario_params_list with
one list of values per scenario parameter; the cartesian product of the lists is the scenario list,
mplc/utils.py:40-87).  Differences: YAML is read with PyYAML's safe loader (the reference uses ruamel's
YAML(typ='safe'); same result on these plain documents), logging goes through the standard library, and
there is no TensorFlow GPU setup (init_gpu_config reports the HIP device instead).
"""
import argparse
import datetime
import logging
import sys
from itertools import product
from pathlib import Path
from shutil import copyfile

from . import constants

logger = logging.getLogger("mplc")


def load_cfg(yaml_filepath):
    """mplc/utils.py:20-37: safe-load the experiment YAML (duplicated keys are an error)."""
    import yaml

    class _UniqueKeyLoader(yaml.SafeLoader):
        def construct_mapping(self, node, deep=False):
            keys = [self.construct_object(k, deep=deep) for k, _ in node.value]
            dup = {k for k in keys if keys.count(k) > 1}
            if dup:
                raise ValueError(f"duplicated keys in {yaml_filepath}: {sorted(map(str, dup))}")
            return super().construct_mapping(node, deep)

    logger.info("Loading experiment yaml file")
    with open(yaml_filepath, "r") as stream:
        cfg = yaml.load(stream, Loader=_UniqueKeyLoader)
    logger.info(cfg)
    return cfg


def get_scenario_params_list(config):
    """mplc/utils.py:40-87: expand each scenario block into the cartesian product of its value lists.
    A dataset_name mapping {name: init_model_from or None} yields one block per dataset."""
    blocks = []
    for block in config:
        names = block["dataset_name"]
        if isinstance(names, dict):
            for name, init in names.items():
                b = dict(block)
                b["dataset_name"] = [name]
                b["init_model_from"] = ["random_initialization"] if init is None else init
                blocks.append(b)
        else:
            blocks.append(block)
    out = []
    for block in blocks:
        keys = list(block.keys())
        for combo in product(*block.values()):
            sc = dict(zip(keys, combo))
            if sc["partners_count"] != len(sc["amounts_per_partner"]):
                raise Exception("Length of amounts_per_partner does not match number of partners.")
            split = sc.get("samples_split_option")
            if split is not None and split[0] == "advanced" and sc["partners_count"] != len(split[1]):
                raise Exception("Length of samples_split_option does not match number of partners.")
            if "corrupted_datasets" in keys and sc["partners_count"] != len(sc["corrupted_datasets"]):
                raise Exception("Length of corrupted_datasets does not match number of partners.")
            out.append(sc)
    logger.info(f"Number of scenario(s) configured: {len(out)}")
    return out


def init_result_folder(yaml_filepath, cfg, root=None):
    """mplc/utils.py:90-128: experiments/<experiment_name>_<date>[_bis...] with a copy of the YAML."""
    now_str = datetime.datetime.now().strftime("%Y-%m-%d_%Hh%M")
    base = Path(root) if root is not None else Path.cwd() / constants.EXPERIMENTS_FOLDER_NAME
    experiment_path = base / (cfg["experiment_name"] + "_" + now_str)
    while experiment_path.exists():
        logger.warning(f"Experiment folder, {experiment_path} already exists")
        experiment_path = Path(str(experiment_path) + "_bis")
    experiment_path.mkdir(parents=True, exist_ok=False)
    cfg["experiment_path"] = experiment_path
    copyfile(yaml_filepath, experiment_path / Path(yaml_filepath).name)
    logger.info("experiment folder " + str(experiment_path) + " created.")
    return cfg


def get_config_from_file(config_filepath, root=None):
    return init_result_folder(config_filepath, load_cfg(config_filepath), root)


def parse_command_line_arguments(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("-f", "--file", help="input config file")
    parser.add_argument("-v", "--verbose", help="verbose output", action="store_true")
    return parser.parse_args(argv)


def init_logger(debug=False):
    """Console logging at INFO (DEBUG with -v), as mplc/utils.py:150-160."""
    logger.handlers.clear()
    h = logging.StreamHandler(sys.stdout)
    h.setFormatter(logging.Formatter("%(asctime)s | %(levelname)-8s | %(message)s"))
    logger.addHandler(h)
    logger.setLevel(logging.DEBUG if debug else logging.INFO)


def set_log_file(path):
    """mplc/utils.py:179-186: info.log and debug.log in the experiment folder, plus the console."""
    path = Path(path)
    for name, level in ((constants.INFO_LOGGING_FILE_NAME, logging.INFO),
                        (constants.DEBUG_LOGGING_FILE_NAME, logging.DEBUG)):
        h = logging.FileHandler(path / name)
        h.setLevel(level)
        h.setFormatter(logging.Formatter("%(asctime)s | %(levelname)-8s | %(message)s"))
        logger.addHandler(h)
    if logger.level > logging.DEBUG:
        logger.setLevel(logging.DEBUG)
        for h in logger.handlers:
            if isinstance(h, logging.StreamHandler) and not isinstance(h, logging.FileHandler):
                h.setLevel(logging.INFO)


def init_gpu_config():
    """The reference configures TF's GPU memory growth (mplc/utils.py:131-144); here: report the HIP device."""
    try:
        import torch
        if torch.cuda.is_available():
            logger.info(f"Found GPU: {torch.cuda.get_device_name(0)}")
            return
    except Exception:  # noqa: BLE001
        pass
    logger.info("No GPU found")


__all__ = ["load_cfg", "get_scenario_params_list", "init_result_folder", "get_config_from_file",
           "parse_command_line_arguments", "init_logger", "set_log_file", "init_gpu_config"]
