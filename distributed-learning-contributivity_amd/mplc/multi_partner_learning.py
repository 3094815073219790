"""Multi-partner learning approaches - drop-in for mplc/multi_partner_learning.py on the coalition path.

The reference trains one Keras model per partner per round, one coalition at a time
(mplc/multi_partner_learning.py:195-334).  Here the approach classes keep the reference's constructor
and ``fit()`` / ``history.score`` contract (used by Contributivity.not_twice_characteristic,
mplc/contributivity.py:100-114) but delegate to the scenario's batched MI355X engine
(mplc/engine.py), and additionally expose ``evaluate_coalitions(scenario, coalitions)`` so that
contributivity estimators can have many coalitions trained at once.
"""
import operator
from timeit import default_timer as timer

import numpy as np

from . import constants

ALLOWED_PARAMETERS = ('partners_list', 'epoch_count', 'minibatch_count', 'dataset', 'aggregation_method',
                      'is_early_stopping', 'is_save_data', 'save_folder', 'init_model_from', 'use_saved_weights')


class History:
    """mplc/mpl_utils.py:11-45: score (test accuracy of the final model), nb_epochs_done, and the learning
    history ``history[partner_id][metric]`` / ``history['mpl_model'][metric]`` as [epoch_count,
    minibatch_count] arrays (partners: 'val_accuracy', 'val_loss', 'loss', 'accuracy', NaN until logged;
    the collective model: 'val_accuracy', 'val_loss', zeros until logged).  Filled by a recorded fit
    (MultiPartnerLearning.fit with record_history, the scenario's main learning run); a fit served from
    the coalition-value cache leaves it empty."""
    metrics = ['val_accuracy', 'val_loss', 'loss', 'accuracy']

    def __init__(self, mpl=None):
        self.mpl = mpl
        self.save_folder = getattr(mpl, "save_folder", None)
        self.score = None
        self.nb_epochs_done = 0
        self.history = {}

    def partners_to_dataframe(self):
        """mplc/mpl_utils.py:29-43: one row per (partner, epoch, minibatch) with the four metrics."""
        import pandas as pd
        temp = {'Partner': [], 'Epoch': [], 'Minibatch': []}
        for key in self.metrics:
            temp[key] = []
        for pid, hist in [(k, v) for k, v in self.history.items() if k != 'mpl_model']:
            E, M = next(iter(hist.values())).shape
            for epoch in range(E):
                for mb in range(M):
                    temp['Partner'].append(pid)
                    temp['Epoch'].append(epoch)
                    temp['Minibatch'].append(mb)
                    for metric, matrix in hist.items():
                        temp[metric].append(matrix[epoch, mb])
        return pd.DataFrame.from_dict(temp)


def _engine(scenario):
    eng = getattr(scenario, "engine", None)
    if eng is None:
        from .engine import CoalitionEngine
        eng = CoalitionEngine.for_scenario(scenario)
        scenario.engine = eng
    return eng


class MultiPartnerLearning:
    """Common constructor (mplc/multi_partner_learning.py:34-91): attributes come from the scenario and
    may be overridden by ALLOWED_PARAMETERS kwargs."""

    def __init__(self, scenario, **kwargs):
        self.scenario = scenario
        self.dataset = getattr(scenario, "dataset", None)
        self.partners_list = scenario.partners_list
        self.epoch_count = getattr(scenario, "epoch_count", constants.DEFAULT_EPOCH_COUNT)
        self.minibatch_count = getattr(scenario, "minibatch_count", constants.DEFAULT_BATCH_COUNT)
        self.is_early_stopping = getattr(scenario, "is_early_stopping", True)
        self.aggregation_method = getattr(scenario, "aggregation", None)
        self.is_save_data = False
        self.save_folder = getattr(scenario, "save_folder", None)
        self.__dict__.update((k, v) for k, v in kwargs.items() if k in ALLOWED_PARAMETERS)
        for partner in self.partners_list:
            if not hasattr(partner, "id"):
                raise TypeError("partners_list must hold Partner objects")
        self.epoch_index = 0
        self.minibatch_index = 0
        self.learning_computation_time = 0
        self.record_history = bool(kwargs.get("record_history", False))
        self.history = History(self)

    @property
    def partners_count(self):
        return len(self.partners_list)

    def _coalition(self):
        return tuple(sorted(int(p.id) for p in self.partners_list))

    def fit(self):
        start = timer()
        key = self._coalition()
        cache = getattr(self.scenario, "coalition_values", None)
        # the cache holds v(S) as Contributivity defines it: the scenario's epochs, early stopping ON
        # (mplc/contributivity.py:100-112); reuse it only for a fit with the same semantics
        same = (self.epoch_count == getattr(self.scenario, "epoch_count", self.epoch_count)
                and (self.is_early_stopping or self.epoch_count <= constants.PATIENCE))
        if same and cache is not None and key in cache and not self.record_history:  # evaluated earlier (or persisted)
            self.history.score = float(cache[key])
            self.history.nb_epochs_done = int(getattr(self.scenario, "coalition_epochs", {}).get(key, self.epoch_count))
            self.learning_computation_time = timer() - start
            return
        eng = _engine(self.scenario)
        record = self.record_history and getattr(eng, "supports_history", False)
        kw = dict(record_history=True) if record else {}
        # a dry-run scenario writes nothing (the reference's is_dry_run skips the experiment folder)
        save = self.is_save_data and self.save_folder is not None and not getattr(self.scenario, "is_dry_run", False)
        if save:
            kw["return_models"] = True
        res = eng.evaluate([self._coalition()], epoch_count=self.epoch_count,
                           is_early_stopping=self.is_early_stopping, return_details=True, **kw)
        self.history.score = float(res["scores"][0])
        self.history.nb_epochs_done = int(res["epochs_done"][0])
        if record:  # keyed by partner.id (== the engine's partner index) and 'mpl_model'
            self.history.history = res["history"]
            self.epoch_index = self.history.nb_epochs_done - 1
        if save:
            self.model_weights = res["models"][0]
            self.save_final_model()
        self.learning_computation_time = timer() - start

    def save_final_model(self):
        """mplc/multi_partner_learning.py:117-128: <save_folder>/model/<dataset>_final_weights.npy, the final
        model's get_weights() list saved with np.save (an object array, as the reference writes it).  The
        reference saves after EVERY fit - each coalition of a contributivity run overwrites the same file, so
        what survives is an arbitrary coalition's model; here the learners that save are the ones built with
        is_save_data=True (Scenario.run's main fit), so the file holds the grand coalition's final model.
        The Keras .h5 copy is not written: h5py / Keras are not available."""
        import os
        folder = os.path.join(str(self.save_folder), "model")
        os.makedirs(folder, exist_ok=True)
        name = getattr(self.dataset, "name", "model")
        w = self.model_weights
        if isinstance(w, np.ndarray):  # Titanic LR: one (1, 28) array
            np.save(os.path.join(folder, name + "_final_weights.npy"), w)
            return
        arr = np.empty(len(w), dtype=object)
        arr[:] = list(w)
        np.save(os.path.join(folder, name + "_final_weights.npy"), arr, allow_pickle=True)

    # Contributivity plans TMCS/ITMCS permutation waves with the device walk (mplc.mc) for this approach
    device_planning = True

    @classmethod
    def evaluate_coalitions(cls, scenario, coalitions):
        """Batched v(S) for many coalitions (test accuracy of the trained coalition model), float64 array.
        Under torch.distributed the coalitions are LPT-sharded over the ranks (mplc.parallel)."""
        from .parallel import EpochModel, sharded_evaluate
        eng = _engine(scenario)

        # Contributivity always builds its learners with is_early_stopping=True (mplc/contributivity.py:101-112),
        # whatever the scenario's own flag: that is the flag the training below uses
        es_flag = True

        def local(cs):
            return eng.evaluate(cs, is_early_stopping=es_flag)
        # with early stopping a coalition's cost follows its realised epochs: the LPT plan learns them per size
        # (from the flag the evaluation is actually given, not the scenario's)
        es = es_flag and int(getattr(eng, "epoch_count", 0)) > constants.PATIENCE
        model = None
        if es:
            model = getattr(eng, "epoch_model", None)
            if model is None:
                model = eng.epoch_model = EpochModel(eng.epoch_count)
        return sharded_evaluate(local, list(coalitions), eng.partner_sizes, eng.device,
                                epochs_local=(lambda: eng.last_epochs_done) if es else None, epoch_model=model)


class SinglePartnerLearning(MultiPartnerLearning):
    """mplc/multi_partner_learning.py:230-275: one model, fit(epochs=E, bs=partner.batch_size)."""

    def __init__(self, scenario, partner, **kwargs):
        if type(partner) == list:
            raise ValueError('More than one partner is provided')
        kwargs['partners_list'] = [partner]
        super().__init__(scenario, **kwargs)
        self.partner = partner


class FederatedAverageLearning(MultiPartnerLearning):
    """mplc/multi_partner_learning.py:278-334: FedAvg rounds over minibatches, fresh optimizer per partner fit."""
    engine_approach = "fedavg"

    def __init__(self, scenario, **kwargs):
        super().__init__(scenario, **kwargs)
        if self.partners_count == 1:
            raise ValueError('Only one partner is provided. Please use the dedicated SinglePartnerLearning class')


class SequentialLearning(MultiPartnerLearning):
    """seq-pure, mplc/multi_partner_learning.py:337-381: per round one model (fresh optimizer) trained on
    each member's minibatch in a shuffled member order; the model after the last member goes on.  On the
    engine: one MPLC_REP_SEQ replica per coalition (csrc/keyed.h seq_locate)."""
    engine_approach = "seq-pure"

    def __init__(self, scenario, **kwargs):
        super().__init__(scenario, **kwargs)
        if self.partners_count == 1:
            raise ValueError('Only one partner is provided. Please use the dedicated SinglePartnerLearning class')


class SequentialWithFinalAggLearning(SequentialLearning):
    """seq-with-final-agg, mplc/multi_partner_learning.py:384-405: as seq-pure, and at each epoch end the
    model is the aggregate of the members' weights after their last fit (csrc/seq.hip snapshots)."""
    engine_approach = "seq-with-final-agg"


class SequentialAverageLearning(SequentialLearning):
    """seqavg, mplc/multi_partner_learning.py:408-430: as seq-pure, aggregating the members' weights after
    every round."""
    engine_approach = "seqavg"


MULTI_PARTNER_LEARNING_APPROACHES = {
    "fedavg": FederatedAverageLearning,
    "seq-pure": SequentialLearning,
    "seq-with-final-agg": SequentialWithFinalAggLearning,
    "seqavg": SequentialAverageLearning,
}

__all__ = ["MultiPartnerLearning", "SinglePartnerLearning", "FederatedAverageLearning", "SequentialLearning",
           "SequentialWithFinalAggLearning", "SequentialAverageLearning", "MULTI_PARTNER_LEARNING_APPROACHES",
           "operator", "np"]
