"""Scenario - drop-in for mplc/scenario.py on the coalition path.

Keeps the reference's constructor keywords and validation (mplc/scenario.py:28-128, 216-261), the basic
random / stratified split (mplc/scenario.py:571-681, index-identical: tests/test_scenario.py vs
tests/golden/splits.json), batch sizes (mplc/scenario.py:705-724), ``run()`` (mplc/scenario.py:845-879)
and ``to_dataframe()`` (mplc/scenario.py:788-843).  Training goes through the batched MI355X engine.

Out of scope: the advanced split (:392-569), label corruption (:726-786), plots.
"""
import datetime
import logging
import uuid
from pathlib import Path
from timeit import default_timer as timer

import numpy as np
from sklearn.preprocessing import LabelEncoder

from . import constants
from . import dataset as dataset_module
from .fedavg import AGGREGATION_SCHEMES
from .multi_partner_learning import MULTI_PARTNER_LEARNING_APPROACHES
from .partner import Partner

logger = logging.getLogger("mplc")

PARAMS_KNOWN = ["dataset", "dataset_name", "dataset_proportion", "methods", "multi_partner_learning_approach",
                "aggregation", "partners_count", "amounts_per_partner", "corrupted_datasets", "samples_split_option",
                "gradient_updates_per_pass_count", "epoch_count", "minibatch_count", "is_early_stopping",
                "init_model_from", "is_quick_demo", "engine_seed", "coalition_values_file"]



def _label_codes(y):
    """LabelEncoder().fit_transform([str(row) for row in y]) (the reference's label encoding for the split,
    mplc/scenario.py:573), with str() taken once per distinct row instead of once per sample: equal rows give
    equal strings, so the codes are identical."""
    y = np.asarray(y)
    uniq, inverse = np.unique(y, axis=0, return_inverse=True) if y.ndim > 1 else np.unique(y, return_inverse=True)
    inverse = np.asarray(inverse).reshape(-1)
    names = [str(u) for u in uniq]
    order = LabelEncoder().fit(names)
    return order.transform(names)[inverse]

class Scenario:
    def __init__(self, partners_count, amounts_per_partner, dataset=None, dataset_name=constants.MNIST,
                 dataset_proportion=1, samples_split_option=None, corrupted_datasets=None,
                 init_model_from="random_initialization", multi_partner_learning_approach="fedavg",
                 aggregation_weighting="data-volume",
                 gradient_updates_per_pass_count=constants.DEFAULT_GRADIENT_UPDATES_PER_PASS_COUNT,
                 minibatch_count=constants.DEFAULT_BATCH_COUNT, epoch_count=constants.DEFAULT_EPOCH_COUNT,
                 is_early_stopping=True, methods=None, is_quick_demo=False, experiment_path=Path("./experiments"),
                 scenario_id=1, repeats_count=1, is_dry_run=True, engine_seed=0, coalition_values_file=None,
                 **kwargs):
        unknown = [k for k in kwargs if k not in PARAMS_KNOWN]
        if unknown:
            raise Exception(f"Unrecognised parameters {unknown}, check your configuration")
        if isinstance(dataset, dataset_module.Dataset):
            self.dataset = dataset
        elif dataset_name == constants.MNIST:
            self.dataset = dataset_module.Mnist()
        elif dataset_name == constants.CIFAR10:
            self.dataset = dataset_module.Cifar10()
        elif dataset_name == constants.TITANIC:
            self.dataset = dataset_module.Titanic()
        else:
            raise Exception(f"Dataset named '{dataset_name}' is not supported by the MI355X engine (yet)")
        self.dataset_proportion = dataset_proportion
        assert self.dataset_proportion > 0, "Error in the config file, dataset_proportion should be > 0"
        assert self.dataset_proportion <= 1, "Error in the config file, dataset_proportion should be <= 1"
        if self.dataset_proportion < 1:
            self.dataset.shorten_dataset_proportion(self.dataset_proportion)
        self.nb_samples_used = len(self.dataset.x_train)
        self.final_relative_nb_samples = []
        self.partners_list = []
        self.partners_count = partners_count
        self.amounts_per_partner = amounts_per_partner
        if samples_split_option is not None:
            self.samples_split_type, self.samples_split_description = samples_split_option
        else:
            self.samples_split_type, self.samples_split_description = "basic", "random"
        self.corrupted_datasets = corrupted_datasets or ["not_corrupted"] * self.partners_count
        if any(c != "not_corrupted" for c in self.corrupted_datasets):
            raise NotImplementedError("label corruption is outside the engine's scope (DESIGN.md)")
        self.mpl = None
        try:
            self.multi_partner_learning_approach = MULTI_PARTNER_LEARNING_APPROACHES[multi_partner_learning_approach]
        except KeyError:
            raise KeyError(f"Multi-partner learning approach '{multi_partner_learning_approach}' is not a valid "
                           f"approach. List of supported approach : {', '.join(MULTI_PARTNER_LEARNING_APPROACHES)}, ")
        if aggregation_weighting == "local-score":
            # registered in the reference (mplc/mpl_utils.py:132-136) but its aggregate_model_weights returns
            # None (:118-128), so the next round's models are None: rejected here instead of failing mid-run
            raise NotImplementedError("'local-score' aggregation is broken in the reference (its aggregator "
                                      "returns no weights); use 'data-volume' or 'uniform' (DESIGN.md)")
        if aggregation_weighting not in AGGREGATION_SCHEMES:
            raise ValueError(f"aggregation approach '{aggregation_weighting}' is not a valid approach. ")
        self.aggregation_weighting = aggregation_weighting
        self.aggregation = aggregation_weighting
        self.epoch_count = epoch_count
        assert self.epoch_count > 0, "Error: in the provided config file, epoch_count should be > 0"
        self.minibatch_count = minibatch_count
        assert self.minibatch_count > 0, "Error: in the provided config file, minibatch_count should be > 0"
        self.gradient_updates_per_pass_count = gradient_updates_per_pass_count
        assert self.gradient_updates_per_pass_count > 0
        self.is_early_stopping = is_early_stopping
        self.init_model_from = init_model_from
        if init_model_from != "random_initialization":
            raise NotImplementedError("warm start from saved weights is outside the engine's scope")
        self.use_saved_weights = False
        self.methods = list(methods) if methods else []
        for m in self.methods:
            if m not in constants.CONTRIBUTIVITY_METHODS:
                raise Exception(f"Contributivity method '{m}' is not in methods list.")
        self.is_quick_demo = is_quick_demo
        self.engine_seed = int(engine_seed)
        self.contributivity_list = []
        self.scenario_id = scenario_id
        self.repeats_count = repeats_count
        self.n_repeat = 0
        now = datetime.datetime.now().strftime("%Y-%m-%d_%Hh%M")
        self.scenario_name = f"scenario_{scenario_id}_repeat_{self.n_repeat}_{now}_{uuid.uuid4().hex[:3]}"
        self.short_scenario_name = f"{self.partners_count} {self.amounts_per_partner}"
        self.save_folder = Path(experiment_path) / self.scenario_name
        self.is_dry_run = is_dry_run
        if not is_dry_run:
            self.save_folder.mkdir(parents=True, exist_ok=True)
        self.engine = None
        self.coalition_values = {}
        # opt-in persisted v(S) table shared across methods and runs (npz, bitmask order)
        self.coalition_values_file = coalition_values_file

    # --------------------------------------------------------------------------------------------
    def instantiate_scenario_partners(self):
        if self.partners_list != []:
            raise Exception("self.partners_list should be []")
        self.partners_list = [Partner(i) for i in range(self.partners_count)]

    def split_data(self, is_logging_enabled=True):
        """mplc/scenario.py:571-681 (basic split), plus each partner's row indices (train_idx)."""
        y_train = _label_codes(self.dataset.y_train)
        assert len(self.amounts_per_partner) == self.partners_count, \
            "Error: amounts_per_partner list should have a size equals to partners_count"
        assert np.sum(self.amounts_per_partner) == 1, \
            "Error: the sum of the proportions you provided isn't equal to 1"
        if self.partners_count == 1:
            cut = 1
        else:
            cum = np.empty((self.partners_count - 1,))
            cum[0] = self.amounts_per_partner[0]
            for i in range(self.partners_count - 2):
                cum[i + 1] = cum[i] + self.amounts_per_partner[i + 1]
            cut = (cum * len(y_train)).astype(int)
        if self.samples_split_description == "stratified":
            order = y_train.argsort()
        elif self.samples_split_description == "random":
            order = np.arange(len(y_train))
            np.random.seed(42)
            np.random.shuffle(order)
        else:
            raise NameError("This samples_split option [" + self.samples_split_description + "] is not recognized.")
        for p, idx in zip(self.partners_list, np.split(order, cut)):
            tr, _te, _, _ = self.dataset.train_test_split_local(idx, idx)
            tr, _va, _, _ = self.dataset.train_val_split_local(tr, tr)
            p.train_idx = np.asarray(tr, dtype=np.int64)
            p.x_train = self.dataset.x_train[p.train_idx]
            p.y_train = self.dataset.y_train[p.train_idx]
            p.final_nb_samples = len(p.train_idx)
            p.clusters_list = list(set(y_train[idx]))
        assert self.minibatch_count <= (min(self.amounts_per_partner) * len(y_train)), \
            "Error: a partner doesn't have enough data samples to create the minibatches"
        self.nb_samples_used = sum(len(p.train_idx) for p in self.partners_list)
        self.final_relative_nb_samples = [p.final_nb_samples / self.nb_samples_used for p in self.partners_list]
        if is_logging_enabled:
            for p in self.partners_list:
                logger.info(f"   Partner #{p.id}: {p.final_nb_samples} samples")
        return 0

    def compute_batch_sizes(self):
        """mplc/scenario.py:705-724."""
        lo, hi = 1, constants.MAX_BATCH_SIZE
        if self.partners_count == 1:
            p = self.partners_list[0]
            p.batch_size = int(np.clip(int(len(p.train_idx) / self.gradient_updates_per_pass_count), lo, hi))
        else:
            for p in self.partners_list:
                bs = int(len(p.train_idx) / (self.minibatch_count * self.gradient_updates_per_pass_count))
                p.batch_size = int(np.clip(bs, lo, hi))

    def provision(self):
        """Partners, split and batch sizes (the part of run() that fixes every v(S)'s inputs)."""
        if not self.partners_list:
            self.instantiate_scenario_partners()
            self.split_data(is_logging_enabled=False)
            self.compute_batch_sizes()
        return self

    # --------------------------------------------------------------------------------------------
    def run(self):
        """mplc/scenario.py:845-879: grand-coalition learning, then each contributivity method."""
        from .contributivity import Contributivity
        self.provision()
        if self.coalition_values_file:
            self.load_coalition_values(self.coalition_values_file, missing_ok=True)
        # the main learning run records its history (mplc/mpl_utils.py:11-27), which the Federated SBS
        # methods read (mplc/contributivity.py:1079-1115) - unless its value comes from a persisted table,
        # whose point is to skip training (the history is then empty)
        grand = tuple(range(self.partners_count))
        record = grand not in getattr(self, "persisted_coalitions", ())
        self.mpl = self.multi_partner_learning_approach(self, is_save_data=True, record_history=record)
        self.mpl.fit()
        if self.is_early_stopping or self.epoch_count <= constants.PATIENCE:  # same v(N) as Contributivity's
            self.coalition_values[tuple(range(self.partners_count))] = self.mpl.history.score
        for method in self.methods:
            contrib = Contributivity(scenario=self)
            contrib.compute_contributivity(method)
            self.contributivity_list.append(contrib)
            logger.info(f"## Evaluating contributivity with {method}: {contrib}")
        if self.coalition_values_file:
            self.save_coalition_values(self.coalition_values_file)
        return 0

    # --------------------------------------------------------------------------------------------
    # persisted v(S) table
    # --------------------------------------------------------------------------------------------
    def coalition_values_fingerprint(self):
        """Everything a v(S) depends on; a table saved under another fingerprint is never reused."""
        import json
        import zlib
        approach = self.multi_partner_learning_approach
        ds = self.dataset
        content = zlib.crc32(np.ascontiguousarray(ds.y_train).tobytes())
        content = zlib.crc32(np.ascontiguousarray(np.asarray(ds.x_train)[::97]).tobytes(), content)
        content = zlib.crc32(np.ascontiguousarray(np.asarray(ds.x_test)[::97]).tobytes(), content)
        return json.dumps({
            "content_crc32": int(content),
            "dataset": self.dataset.name, "synthetic": bool(getattr(self.dataset, "synthetic", False)),
            "n_train": int(len(self.dataset.x_train)), "n_val": int(len(self.dataset.x_val)),
            "n_test": int(len(self.dataset.x_test)),
            "partners": [int(len(p.train_idx)) for p in self.partners_list],
            "batch_sizes": [int(p.batch_size) for p in self.partners_list],
            "split": [self.samples_split_type, str(self.samples_split_description)],
            "approach": getattr(approach, "__name__", str(approach)), "aggregation": self.aggregation,
            "epoch_count": self.epoch_count, "minibatch_count": self.minibatch_count,
            "gradient_updates_per_pass_count": self.gradient_updates_per_pass_count,
            "is_early_stopping": bool(self.is_early_stopping), "engine_seed": self.engine_seed,
            "dataset_proportion": self.dataset_proportion}, sort_keys=True)

    def save_coalition_values(self, path):
        """Write the known v(S) as npz: masks (uint64, bit i = partner i), values (float64), fingerprint."""
        keys = sorted(k for k in self.coalition_values if len(k))
        masks = np.array([sum(1 << int(i) for i in k) for k in keys], dtype=np.uint64)
        values = np.array([float(self.coalition_values[k]) for k in keys], dtype=np.float64)
        np.savez(path, masks=masks, values=values, n=np.int64(self.partners_count),
                 fingerprint=np.array(self.coalition_values_fingerprint()))

    def load_coalition_values(self, path, missing_ok=False):
        """Merge a saved table into the coalition cache (the memo and call counts of each method are
        unaffected: only the training is skipped).  Returns the number of entries loaded."""
        import os
        if not os.path.exists(path):
            if missing_ok:
                return 0
            raise FileNotFoundError(path)
        with np.load(path, allow_pickle=False) as f:
            if str(f["fingerprint"]) != self.coalition_values_fingerprint() or int(f["n"]) != self.partners_count:
                raise ValueError(f"{path} was computed for another scenario configuration")
            loaded = getattr(self, "persisted_coalitions", set())
            for m, v in zip(f["masks"], f["values"]):
                m = int(m)
                key = tuple(i for i in range(self.partners_count) if (m >> i) & 1)
                self.coalition_values[key] = float(v)
                loaded.add(key)
            self.persisted_coalitions = loaded
            return int(len(f["values"]))

    def append_contributivity(self, contributivity):
        self.contributivity_list.append(contributivity)

    def to_dataframe(self):
        """Results table with the reference's columns (mplc/scenario.py:788-843)."""
        import pandas as pd
        base = {
            "scenario_name": self.scenario_name, "short_scenario_name": self.short_scenario_name,
            "dataset_name": self.dataset.name, "train_data_samples_count": len(self.dataset.x_train),
            "test_data_samples_count": len(self.dataset.x_test), "partners_count": self.partners_count,
            "dataset_fraction_per_partner": self.amounts_per_partner,
            "samples_split_description": self.samples_split_description, "nb_samples_used": self.nb_samples_used,
            "final_relative_nb_samples": self.final_relative_nb_samples,
            "multi_partner_learning_approach": self.multi_partner_learning_approach,
            "aggregation": self.aggregation, "epoch_count": self.epoch_count, "minibatch_count": self.minibatch_count,
            "gradient_updates_per_pass_count": self.gradient_updates_per_pass_count,
            "is_early_stopping": self.is_early_stopping, "mpl_test_score": self.mpl.history.score,
            "mpl_nb_epochs_done": self.mpl.history.nb_epochs_done,
            "learning_computation_time_sec": self.mpl.learning_computation_time,
        }
        if getattr(self.dataset, "synthetic", False):  # not a reference column: only present when true
            base["synthetic_data"] = True
        rows = []
        if not self.contributivity_list:
            rows.append(dict(base))
        for contrib in self.contributivity_list:
            d = dict(base)
            d["contributivity_method"] = contrib.name
            d["contributivity_scores"] = contrib.contributivity_scores
            d["contributivity_stds"] = contrib.scores_std
            d["computation_time_sec"] = contrib.computation_time_sec
            d["first_characteristic_calls_count"] = contrib.first_charac_fct_calls_count
            for i in range(self.partners_count):
                r = dict(d)
                r["partner_id"] = i
                r["dataset_fraction_of_partner"] = self.amounts_per_partner[i]
                r["contributivity_score"] = contrib.contributivity_scores[i]
                r["contributivity_std"] = contrib.scores_std[i]
                rows.append(r)
        return pd.DataFrame(rows)


__all__ = ["Scenario", "timer"]
