"""Coalition-evaluation engine: v(S) for many coalitions at once on the MI355X.

Replaces the reference's one-coalition-at-a-time loop (Contributivity.not_twice_characteristic ->
FederatedAverageLearning/SinglePartnerLearning(...).fit() -> history.score,
mplc/contributivity.py:92-136, mplc/multi_partner_learning.py:195-334) with batched training of every
requested coalition in lockstep (mplc/cnn.py + csrc/mnist_cnn.hip for MNIST, mplc/cifar.py +
csrc/cifar_cnn.hip for CIFAR10).

Data live in HBM for the engine's lifetime: the dataset's train/val/test arrays (fp32 images, int32
labels), and each partner's row indices into the train array (the reference's partner.x_train copies,
mplc/scenario.py:571-681).

Determinism: v(S) depends only on (S, seed) - initial weights are keyed by (seed, S) and each
replica's sample order by (seed, S, partner, epoch, round) - so a coalition evaluated alone or inside
any batch, on any GPU, gets the same value.  (The reference's values are not reproducible at all:
TF is never seeded, mplc/scenario.py:614 only seeds numpy for the split.)
"""
import os

import numpy as np

from . import constants
from .cnn import CnnBatchTrainer, MnistModel, minibatch_bounds

MODELS = {"mnist_cnn": MnistModel}


def model_class(name):
    if name == "cifar10_cnn" and name not in MODELS:
        from .cifar import CifarModel
        MODELS[name] = CifarModel
    if name not in MODELS:
        raise NotImplementedError(f"model '{name}' has no batched MI355X kernels (see DESIGN.md)")
    return MODELS[name]


class CoalitionEngine:
    """Batched v(S) evaluator bound to one scenario's partners, data and training hyper-parameters."""

    def __init__(self, *, x_train, y_train, x_val, y_val, x_test, y_test, partner_rows, batch_sizes,
                 epoch_count, minibatch_count, aggregation="data-volume", is_early_stopping=True, seed=0,
                 model="mnist_cnn", device=None, memory_budget_bytes=None, eval_budget_bytes=8 << 30,
                 approach="fedavg"):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("MI355X (HIP) device required: the MPLC engine has no CPU fallback")
        self.model_impl = model_class(model)()
        if approach not in ("fedavg", "seq-pure", "seq-with-final-agg", "seqavg"):
            raise NotImplementedError(f"multi-partner learning approach '{approach}' has no batched MI355X path")
        self.approach = approach
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.model = model
        self.seed = int(seed)
        self.epoch_count = int(epoch_count)
        self.minibatch_count = int(minibatch_count)
        self.aggregation = aggregation
        self.is_early_stopping = bool(is_early_stopping)
        self.eval_budget_bytes = int(eval_budget_bytes)

        shape = self.model_impl.input_shape

        def images(x):
            x = np.asarray(x, dtype=np.float32)
            return torch.from_numpy(np.ascontiguousarray(x.reshape((x.shape[0],) + shape))).to(self.device)

        def labels(y):
            y = np.asarray(y)
            if y.ndim == 2:
                y = np.argmax(y, axis=1)  # one-hot (keras.utils.to_categorical) -> class id
            return torch.from_numpy(np.ascontiguousarray(y.astype(np.int32))).to(self.device)

        self.x_train_d, self.y_train_d = images(x_train), labels(y_train)
        self.x_val_d, self.y_val_d = images(x_val), labels(y_val)
        self.x_test_d, self.y_test_d = images(x_test), labels(y_test)
        self.partner_sizes = [int(len(r)) for r in partner_rows]
        self.batch_sizes = [int(b) for b in batch_sizes]
        rows, splits, self.rows_off, self.split_off, self.bounds = [], [], [], [], []
        for r in partner_rows:
            self.rows_off.append(len(rows))
            rows.extend(int(i) for i in r)
            b = minibatch_bounds(len(r), self.minibatch_count)
            self.bounds.append(b)
            self.split_off.append(len(splits))
            splits.extend(b)
        self.rows_d = torch.tensor(rows, dtype=torch.int32, device=self.device)
        self.splits_d = torch.tensor(splits, dtype=torch.int32, device=self.device)
        if memory_budget_bytes is None:
            free, _ = torch.cuda.mem_get_info(self.device)
            # memory the caching allocator holds but no tensor uses (an earlier engine's lockstep batches) is
            # as good as free for this engine's batches; mem_get_info does not count it
            free += torch.cuda.memory_reserved(self.device) - torch.cuda.memory_allocated(self.device)
            memory_budget_bytes = int(free * 0.8) - self.eval_budget_bytes
            if memory_budget_bytes < (256 << 20):
                raise RuntimeError(f"not enough free device memory for the coalition engine: {free >> 20} MiB free, "
                                   f"{self.eval_budget_bytes >> 20} MiB reserved for evaluation")
        self.memory_budget_bytes = int(memory_budget_bytes)
        self.trainer = CnnBatchTrainer(self)
        self.profiler = None  # optional KernelTimer (bench.py): in-stream HIP events around the step kernels
        # lockstep batches split over this many HIP streams (MPLC_CONCURRENT_BATCHES overrides): 2 for the CIFAR10
        # model, whose ~0.3 ms step kernels leave tails and launch gaps a second batch fills (config #4 TMCS +7 %,
        # DESIGN.md 8); 1 for MNIST (+1 % there: its 5120-replica launches already fill the chip)
        default_streams = "2" if model == "cifar10_cnn" else "1"
        self.concurrent_batches = max(1, int(os.environ.get("MPLC_CONCURRENT_BATCHES", default_streams)))
        # FedAvg rounds leave the large dense layer out of the broadcast (the next round's first step reads it
        # from the coalition row); False broadcasts every layer (the plain copy-back, for A/B tests)
        self.bcast_skip = True
        # the round's last step averages W3 in its dense pass (MNIST; ABI 4): MPLC_FUSE_AVG=0 keeps the
        # separate aggregation of every layer (A/B and bit-identity tests)
        self.fuse_avg = os.environ.get("MPLC_FUSE_AVG", "1") != "0"
        self.stats = {"coalitions": 0, "batches": 0, "replicas": 0, "samples": 0}

    # --------------------------------------------------------------------------------------------
    @classmethod
    def for_scenario(cls, scenario, **overrides):
        """Engine for the scenario's dataset: the batched CNN for MNIST, the batched logistic regression for
        Titanic (mplc/dataset.py:323-394)."""
        ds = scenario.dataset
        name = getattr(ds, "name", "mnist")
        if name == "titanic" and cls is CoalitionEngine:
            from .lr import LogRegEngine
            target = LogRegEngine
        else:
            target = cls
        model = {"mnist": "mnist_cnn", "cifar10": "cifar10_cnn"}.get(name, name)
        parts = scenario.partners_list
        rows = []
        for p in parts:
            if getattr(p, "train_idx", None) is None:
                raise ValueError("partners need train_idx (row indices into dataset.x_train); use mplc.scenario")
            rows.append(np.asarray(p.train_idx))
        kw = dict(x_train=ds.x_train, y_train=ds.y_train, x_val=ds.x_val, y_val=ds.y_val, x_test=ds.x_test,
                  y_test=ds.y_test, partner_rows=rows, batch_sizes=[int(p.batch_size) for p in parts],
                  epoch_count=scenario.epoch_count, minibatch_count=scenario.minibatch_count,
                  aggregation=getattr(scenario, "aggregation_weighting", "data-volume"),
                  is_early_stopping=getattr(scenario, "is_early_stopping", True),
                  seed=getattr(scenario, "engine_seed", int(os.environ.get("MPLC_ENGINE_SEED", "0"))), model=model)
        approach = getattr(getattr(scenario, "multi_partner_learning_approach", None), "engine_approach", "fedavg")
        if target is cls:
            kw["approach"] = approach
        elif approach != "fedavg":
            raise NotImplementedError(f"'{approach}' is not available for the {name} model (FedAvg only)")
        kw.update(overrides)
        if target is not cls:
            kw.pop("batch_sizes", None)
        return target(**kw)

    # --------------------------------------------------------------------------------------------
    def replica_bytes(self, bmax):
        return self.model_impl.replica_bytes(bmax)

    def plan_batches(self, coalitions):
        """Split coalitions into lockstep batches that fit the HBM budget (cost-sorted so that a batch holds
        coalitions of similar size; every coalition's replicas stay together)."""
        order = sorted(range(len(coalitions)), key=lambda i: (len(coalitions[i]) == 1, -len(coalitions[i])))
        batches, cur, cur_bytes = [], [], 0
        for i in order:
            c = coalitions[i]
            bmax = max(self.batch_sizes[p] for p in c)
            need = len(c) * self.replica_bytes(bmax) + self.model_impl.STRIDE * 4
            if cur and (cur_bytes + need > self.memory_budget_bytes or len(cur) >= 65535):
                batches.append(cur)
                cur, cur_bytes = [], 0
            cur.append(i)
            cur_bytes += need
        if cur:
            batches.append(cur)
        return batches

    def warmup(self):
        """Load the HIP code object (one tiny init_params launch) without running any training kernel."""
        import torch
        from . import _native
        buf = torch.empty((1, self.model_impl.STRIDE), dtype=torch.float32, device=self.device)
        keys = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.model_impl.init_params(buf, keys, _native.stream_handle(self.device))
        torch.cuda.synchronize(self.device)

    def release(self):
        """Return the cached device memory of finished lockstep batches to the driver (the data stay)."""
        import gc
        import torch
        gc.collect()
        torch.cuda.empty_cache()

    supports_history = True
    # Lockstep batches trained at once on separate HIP streams (CnnBatchTrainer.run_concurrent): 1 = off.  A
    # batch of at least 2 * CONCURRENT_MIN_COALITIONS coalitions is split into that many cost-balanced parts.
    concurrent_batches = 1
    CONCURRENT_MIN_COALITIONS = 8

    def _concurrent_ok(self, coal, E, es, history, return_models):
        from .cnn import PATIENCE
        return (self.concurrent_batches > 1 and len(coal) >= 2 * self.CONCURRENT_MIN_COALITIONS
                and not (es and E > PATIENCE) and history is None and not return_models
                and self.approach == "fedavg"
                and hasattr(self.trainer, "run_concurrent"))

    def _within_budget(self, coal):
        """Keep the device memory of a lockstep batch within the engine's budget across HIP streams.
        The caching allocator keeps freed blocks per stream, so the blocks a two-stream batch left on the side
        streams cannot serve a batch on the caller's stream (the bench's timed batches) and vice versa: when the
        cached-but-unused memory plus this batch's need would pass memory_budget_bytes (what the batches may
        use beside the resident data), the cache is returned to the driver first.  TMCS-sized batches (a few GB)
        never trigger it."""
        import torch
        if self.concurrent_batches <= 1:
            return
        need = sum(len(c) * self.replica_bytes(max(self.batch_sizes[p] for p in c)) for c in coal)
        idle = torch.cuda.memory_reserved(self.device) - torch.cuda.memory_allocated(self.device)
        if idle > 0 and idle + need > self.memory_budget_bytes:
            self.release()
            self.stats["cache_releases"] = self.stats.get("cache_releases", 0) + 1

    def _run_concurrent(self, coal, E):
        from .parallel import coalition_cost, lpt_shard
        parts = [p for p in lpt_shard([coalition_cost(c, self.partner_sizes) for c in coal], self.concurrent_batches)
                 if p]
        accs = self.trainer.run_concurrent([[coal[i] for i in p] for p in parts], E)
        s = np.zeros(len(coal))
        for p, a in zip(parts, accs):
            s[p] = a
        self.trainer.last_es_trace = [[] for _ in coal]
        return s, np.full(len(coal), E, dtype=np.int64)

    def evaluate(self, coalitions, epoch_count=None, is_early_stopping=None, return_details=False,
                 record_history=False, return_models=False):
        """v(S) (test accuracy, float64) for each coalition (sorted tuple of partner indices).  With
        record_history (one coalition) the details also hold its learning history (cnn.HistoryRecorder);
        with return_models, the final models as Keras get_weights() lists (details["models"])."""
        coalitions = [tuple(sorted(int(i) for i in c)) for c in coalitions]
        for c in coalitions:
            if len(c) == 0 or c[0] < 0 or c[-1] >= len(self.partner_sizes) or len(set(c)) != len(c):
                raise ValueError(f"invalid coalition {c}")
        E = self.epoch_count if epoch_count is None else int(epoch_count)
        es = self.is_early_stopping if is_early_stopping is None else bool(is_early_stopping)
        scores = np.zeros(len(coalitions))
        epochs_done = np.zeros(len(coalitions), dtype=np.int64)
        es_trace = [[] for _ in coalitions]
        models = [None] * len(coalitions)
        history = None
        if record_history:
            if len(coalitions) != 1:
                raise ValueError("record_history takes exactly one coalition")
            history = {}
        for batch in self.plan_batches(coalitions):
            coal = [coalitions[i] for i in batch]
            self._within_budget(coal)
            if self._concurrent_ok(coal, E, es, history, return_models):
                s, e = self._run_concurrent(coal, E)
            else:
                s, e = self.trainer.run(coal, E, es, history=history, keep_models=return_models)
            scores[batch] = s
            epochs_done[batch] = e
            for i, tr in zip(batch, getattr(self.trainer, "last_es_trace", [[]] * len(batch))):
                es_trace[i] = list(tr)
            if return_models:
                from .cnn import keras_weights
                for j, i in enumerate(batch):
                    models[i] = keras_weights(self.trainer.last_models[j], self.model_impl.KERAS_LAYERS)
            self.stats["batches"] += 1
            self.stats["replicas"] += sum(len(c) for c in coal)
            # samples trained (every replica sees all its partner's rows once per epoch done)
            self.stats["samples"] += int(sum(int(ep) * sum(self.partner_sizes[p] for p in c)
                                             for c, ep in zip(coal, e)))
        self.stats["coalitions"] += len(coalitions)
        self.last_epochs_done = epochs_done  # realised epochs of this call's coalitions (early stopping)
        if return_details:
            # es_val_loss: the val losses the early-stopping rule compared (start-of-epoch global model for
            # FedAvg, end-of-epoch model for singletons); empty when early stopping is inactive
            out = {"scores": scores, "epochs_done": epochs_done, "es_val_loss": es_trace}
            if return_models:
                out["models"] = models
            if history is not None:
                out["history"] = history
            return out
        return scores


def default_seed():
    return int(os.environ.get("MPLC_ENGINE_SEED", "0"))


__all__ = ["CoalitionEngine", "constants"]
