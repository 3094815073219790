"""Generate the committed golden fixtures under tests/golden/ from the REFERENCE implementation.

Run ONLY in the build container (where /root/reference exists):

    python tests/golden/make_golden.py

The reference (mshuaic/distributed-learning-contributivity, package ``mplc``) is imported read-only with
stand-ins for the third-party modules that are absent from this image (tensorflow, keras, loguru,
librosa, ruamel.yaml); none of those stand-ins touch the code paths whose outputs are recorded here
(SURVEY.md Appendix A).  Nothing under tests/ imports the reference at test time: the tests read the
JSON files this script writes.

Fixtures written (all data, no reference source):
  shapley_value.json   - mplc/contributivity.py:1210-1253 ``shapley_value`` on seeded v(S) tables, n=1..13
  estimators.json      - mplc/contributivity.py:1134-1198 every coalition-evaluating estimator on fixed
                         v(S) tables with np.random.seed(s): scores, std, normalized, calls count, memo order
  splits.json          - mplc/scenario.py:571-724 + mplc/dataset.py:62-106 partner index arrays and bs_p
  fedavg_lr.json       - mplc/multi_partner_learning.py:195-334 FedAvg with the Titanic LogisticRegression
                         model (mplc/dataset.py:323-394) on synthetic Titanic-shaped data: v(S) per coalition
  lr_history.json      - mplc/mpl_utils.py:11-27 the learning history of the grand coalition's FedAvg fit on the
                         fedavg_lr.json data
  sbs.json             - mplc/contributivity.py:1015-1115 Federated SBS linear / quadratic / constant on seeded
                         learning histories
"""
import itertools
import json
import os
import sys
import time
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


# --------------------------------------------------------------------------------------------------
# Import recipe: stand-ins for modules absent from the image.
# --------------------------------------------------------------------------------------------------
def import_reference():
    np.Inf = np.inf  # numpy>=2 removed np.Inf, used at mplc/contributivity.py:807,919

    def stub(name, **kw):
        m = types.ModuleType(name)
        m.__dict__.update(kw)
        sys.modules[name] = m
        return m

    class _Any:
        def __init__(self, *a, **k):
            pass

    class _Log:
        def __getattr__(self, k):
            return lambda *a, **kw: None

        def level(self, name):
            return types.SimpleNamespace(no=20)

        def opt(self, *a, **k):
            return self

    stub("loguru", logger=_Log())
    stub("keras")
    stub("keras.backend", clear_session=lambda: None)
    stub("keras.callbacks", EarlyStopping=_Any)
    stub("keras.utils", to_categorical=lambda y, num_classes=None: np.eye(
        num_classes or int(np.max(y)) + 1, dtype="float32")[np.asarray(y, int).ravel()])
    stub("keras.datasets", cifar10=None, mnist=None, imdb=None)
    stub("keras.layers", **{k: _Any for k in (
        "Activation Conv2D GlobalAveragePooling2D MaxPooling2D Dense Dropout Embedding Conv1D "
        "MaxPooling1D Flatten").split()})
    stub("keras.losses", categorical_crossentropy=None)
    stub("keras.models", Sequential=_Any)
    stub("keras.optimizers", RMSprop=_Any)
    stub("keras.preprocessing", sequence=None)
    stub("librosa", load=None)
    stub("librosa.feature", mfcc=None)
    stub("ruamel")
    stub("ruamel.yaml", YAML=_Any)
    tf = stub("tensorflow")
    tf.config = types.SimpleNamespace(
        experimental=types.SimpleNamespace(list_physical_devices=lambda k: []))
    sys.path.insert(0, REF)
    import mplc  # noqa: F401
    import mplc.contributivity
    import mplc.multi_partner_learning
    import mplc.scenario
    import mplc.dataset
    return mplc


# --------------------------------------------------------------------------------------------------
# Synthetic characteristic-function tables
# --------------------------------------------------------------------------------------------------
def make_table(n, seed, sizes=None, noise=0.02):
    """Deterministic v(S) for all non-empty S, keyed by sorted tuple.  Concave in data volume plus
    seeded noise, in [0, 1] - the shape of a test-accuracy characteristic function."""
    rng = np.random.default_rng(seed)
    if sizes is None:
        sizes = rng.integers(20, 200, size=n)
    sizes = np.asarray(sizes, dtype=np.int64)
    total = float(sizes.sum())
    table = {(): 0.0}
    for r in range(1, n + 1):
        for c in itertools.combinations(range(n), r):
            x = sizes[list(c)].sum() / total
            v = 0.95 * (1.0 - np.exp(-4.0 * x)) / (1.0 - np.exp(-4.0)) + noise * rng.uniform(-1, 1)
            table[c] = float(min(max(v, 0.0), 1.0))
    return table, sizes


def combination_order(n):
    return [c for r in range(1, n + 1) for c in itertools.combinations(range(n), r)]


# --------------------------------------------------------------------------------------------------
# (a) shapley_value
# --------------------------------------------------------------------------------------------------
def gen_shapley(mplc):
    out = []
    for n in range(1, 14):
        for seed in (0, 1):
            if n >= 12 and seed == 1:
                continue
            table, _ = make_table(n, 1000 + 17 * n + seed)
            v_list = [table[c] for c in combination_order(n)]
            t0 = time.time()
            sv = mplc.contributivity.shapley_value(n, v_list)
            dt = time.time() - t0
            out.append({"n": n, "seed": seed, "v_combination_order": v_list, "shapley": list(map(float, sv)),
                        "ref_seconds": dt})
            print(f"shapley n={n} seed={seed} {dt:.3f}s", flush=True)
    return out


# --------------------------------------------------------------------------------------------------
# (b) estimators on fixed tables
# --------------------------------------------------------------------------------------------------
class _FakeHistory:
    def __init__(self):
        self.score = None


def _fake_learning(table, calls):
    class FakeMPL:
        def __init__(self, scenario, partners_list=None, partner=None, **kw):
            if partner is not None:
                partners_list = [partner]
            self.ids = tuple(sorted(int(p.id) for p in partners_list))
            self.history = _FakeHistory()

        def fit(self):
            calls.append(self.ids)
            self.history.score = table[self.ids]
    return FakeMPL


def gen_estimators(mplc):
    methods = ["Shapley values", "Independent scores", "TMCS", "ITMCS", "IS_lin_S", "IS_reg_S",
               "AIS_Kriging_S", "SMCS", "WR_SMC", "Not a method"]
    cases = []
    big = {8: ["TMCS", "ITMCS", "IS_lin_S", "IS_reg_S", "SMCS", "WR_SMC"], 10: ["TMCS", "ITMCS", "SMCS"]}
    for n, seed in ((2, 3), (3, 5), (4, 7), (5, 11), (6, 13), (8, 17), (10, 19)):
        table, sizes = make_table(n, seed, noise=0.03)
        for method in methods:
            if method in ("SMCS", "WR_SMC") and n == 6:
                continue
            if n in big and method not in big[n]:
                continue
            calls = []
            fake = _fake_learning(table, calls)
            partners = []
            for i in range(n):
                p = types.SimpleNamespace(id=i, y_train=np.zeros(int(sizes[i])))
                partners.append(p)
            scenario = types.SimpleNamespace(partners_list=partners, multi_partner_learning_approach=fake)
            orig_single = mplc.multi_partner_learning.SinglePartnerLearning
            mplc.multi_partner_learning.SinglePartnerLearning = fake
            try:
                np.random.seed(seed)
                contrib = mplc.contributivity.Contributivity(scenario=scenario)
                t0 = time.time()
                try:
                    contrib.compute_contributivity(method)
                    err = None
                except Exception as e:  # record reference failures as data
                    err = f"{type(e).__name__}: {e}"
                dt = time.time() - t0
            finally:
                mplc.multi_partner_learning.SinglePartnerLearning = orig_single
            rng_after = float(np.random.uniform())
            case = {
                "n": n, "seed": seed, "method": method, "sizes": [int(s) for s in sizes],
                "table": {",".join(map(str, k)): v for k, v in table.items()},
                "error": err,
                "name": contrib.name,
                "scores": [float(x) for x in np.atleast_1d(contrib.contributivity_scores)],
                "std": [float(x) for x in np.atleast_1d(contrib.scores_std)],
                "normalized": [float(x) for x in np.atleast_1d(contrib.normalized_scores)],
                "calls_count": int(contrib.first_charac_fct_calls_count),
                "fit_order": [list(c) for c in calls],
                "memo_keys": [list(map(int, k)) for k in contrib.charac_fct_values.keys()],
                "increments": [{",".join(map(str, map(int, k))): float(v) for k, v in d.items()}
                               for d in contrib.increments_values],
                "rng_next_uniform": rng_after,
                "ref_seconds": dt,
            }
            cases.append(case)
            print(f"estimator n={n} {method}: {dt:.2f}s calls={case['calls_count']} err={err}", flush=True)
    return cases


# --------------------------------------------------------------------------------------------------
# (c) partner splits and batch sizes
# --------------------------------------------------------------------------------------------------
def gen_splits(mplc):
    from mplc.dataset import Dataset, Mnist, Cifar10, Titanic

    def make_ds(base_cls, name, n_train, n_test, num_classes, input_shape):
        class IdxDataset(Dataset):
            train_test_split_local = staticmethod(base_cls.train_test_split_local)
            train_val_split_local = staticmethod(base_cls.train_val_split_local)

            def __init__(self):
                x_train = np.arange(n_train, dtype=np.int64).reshape(-1, 1)
                y_train = np.eye(num_classes, dtype="float32")[np.arange(n_train) % num_classes]
                x_test = np.arange(n_test, dtype=np.int64).reshape(-1, 1)
                y_test = np.eye(num_classes, dtype="float32")[np.arange(n_test) % num_classes]
                super().__init__(name, input_shape, num_classes, x_train, y_train, x_test, y_test)

            def generate_new_model(self):
                raise NotImplementedError
        return IdxDataset()

    configs = [
        ("cfg1_mnist_2p", Mnist, "mnist", 60000, 10000, 10, (28, 28, 1), 2, [0.1, 0.9], 0.1, 10, 8),
        ("cfg1b_mnist_3p", Mnist, "mnist", 60000, 10000, 10, (28, 28, 1), 3, [0.2, 0.5, 0.3], 0.1, 10, 8),
        ("cfg2_titanic_10p", Titanic, "titanic", 798, 89, 2, (27,), 10, [0.1] * 10, 1, 1, 8),
        ("cfg3_mnist_10p", Mnist, "mnist", 60000, 10000, 10, (28, 28, 1), 10, [0.1] * 10, 1, 20, 8),
        ("cfg4_cifar_20p", Cifar10, "cifar10", 50000, 10000, 10, (32, 32, 3), 20,
         [0.05] * 19 + [float(1 - np.sum([0.05] * 19))], 1, 20, 8),
        ("tut2_mnist_3p", Mnist, "mnist", 60000, 10000, 10, (28, 28, 1), 3, [0.001, 0.699, 0.3], 1, 3, 8),
    ]
    out = []
    for (tag, cls, name, ntr, nte, ncls, shape, P, amounts, prop, M, G) in configs:
        ds = make_ds(cls, name, ntr, nte, ncls, shape)
        sc = mplc.scenario.Scenario(P, amounts, dataset=ds, dataset_proportion=prop, minibatch_count=M,
                                    gradient_updates_per_pass_count=G, epoch_count=1,
                                    experiment_path=__import__("pathlib").Path("/tmp/mplc_golden_exp"))
        sc.instantiate_scenario_partners()
        sc.split_data(is_logging_enabled=False)
        sc.compute_batch_sizes()
        rec = {"tag": tag, "dataset": name, "n_train_orig": ntr, "n_test": nte, "partners_count": P,
               "amounts": amounts, "dataset_proportion": prop, "minibatch_count": M,
               "gradient_updates_per_pass_count": G,
               "x_train_global": ds.x_train.ravel().tolist(), "x_val_global": ds.x_val.ravel().tolist(),
               "partners": [{"x_train": p.x_train.ravel().tolist(), "batch_size": int(p.batch_size)}
                            for p in sc.partners_list]}
        out.append(rec)
        print(tag, [len(p["x_train"]) for p in rec["partners"]], [p["batch_size"] for p in rec["partners"]],
              len(rec["x_val_global"]), flush=True)
    return out


# --------------------------------------------------------------------------------------------------
# (d) FedAvg with the Titanic LogisticRegression model on synthetic Titanic-shaped data
# --------------------------------------------------------------------------------------------------
def gen_fedavg_lr(mplc):
    from sklearn.datasets import make_classification
    from mplc.dataset import Dataset, Titanic

    X, y = make_classification(n_samples=887, n_features=27, n_informative=8, random_state=0)
    X = X.astype("float32")
    y = y.astype("float32")
    x_tr, x_te, y_tr, y_te = Titanic.train_test_split_global(X, y)

    class SynthTitanic(Dataset):
        train_test_split_local = staticmethod(Titanic.train_test_split_local)
        train_val_split_local = staticmethod(Titanic.train_val_split_local)

        def __init__(self):
            super().__init__("titanic", (27,), 2, x_tr.copy(), y_tr.copy(), x_te.copy(), y_te.copy())

        def generate_new_model(self):
            clf = Titanic.LogisticRegression()
            clf.classes_ = np.array([0, 1])
            clf.metrics_names = ["log_loss", "Accuracy"]
            return clf

    out = {"data": {"X": X.tolist(), "y": y.tolist()}, "cases": []}
    for P, amounts, E, M in ((3, [0.2, 0.5, 0.3], 3, 1), (5, [0.2] * 5, 2, 1), (10, [0.1] * 10, 3, 1)):
        ds = SynthTitanic()
        sc = mplc.scenario.Scenario(P, amounts, dataset=ds, epoch_count=E, minibatch_count=M,
                                    experiment_path=__import__("pathlib").Path("/tmp/mplc_golden_exp"))
        sc.instantiate_scenario_partners()
        sc.split_data(is_logging_enabled=False)
        sc.compute_batch_sizes()
        sc.save_folder = __import__("pathlib").Path("/tmp/mplc_golden_exp/save")
        os.makedirs(sc.save_folder, exist_ok=True)
        contrib = mplc.contributivity.Contributivity(scenario=sc)
        coalitions = [c for c in combination_order(P) if len(c) >= 2]
        if P == 10:
            rng = np.random.default_rng(5)
            pick = rng.choice(len(coalitions), size=40, replace=False)
            coalitions = [coalitions[i] for i in sorted(pick)] + [tuple(range(10))]
        vals = {}
        np.random.seed(0)
        t0 = time.time()
        for c in coalitions:
            vals[",".join(map(str, c))] = float(contrib.not_twice_characteristic(np.array(c)))
        dt = time.time() - t0
        out["cases"].append({"partners_count": P, "amounts": amounts, "epoch_count": E, "minibatch_count": M,
                             "x_val": ds.x_val.tolist(), "y_val": ds.y_val.tolist(),
                             "partners": [{"x_train": p.x_train.tolist(), "y_train": p.y_train.tolist(),
                                           "batch_size": int(p.batch_size)} for p in sc.partners_list],
                             "values": vals, "ref_seconds": dt,
                             "evals_per_sec": len(coalitions) / dt})
        print(f"fedavg-lr P={P}: {len(coalitions)} coalitions in {dt:.1f}s", flush=True)
    return out


# --------------------------------------------------------------------------------------------------
# (d2) learning history of the Titanic-LR FedAvg grand coalition (same data as gen_fedavg_lr)
# --------------------------------------------------------------------------------------------------
def gen_lr_history(mplc):
    """mplc/mpl_utils.py:11-27 History.history of one FedAvg fit (is_early_stopping True, as Contributivity
    builds it) of the grand coalition, per case of fedavg_lr.json (partition identical: same data, seed 42)."""
    from sklearn.datasets import make_classification
    from mplc.dataset import Dataset, Titanic

    X, y = make_classification(n_samples=887, n_features=27, n_informative=8, random_state=0)
    X = X.astype("float32")
    y = y.astype("float32")
    x_tr, x_te, y_tr, y_te = Titanic.train_test_split_global(X, y)

    class SynthTitanic(Dataset):
        train_test_split_local = staticmethod(Titanic.train_test_split_local)
        train_val_split_local = staticmethod(Titanic.train_val_split_local)

        def __init__(self):
            super().__init__("titanic", (27,), 2, x_tr.copy(), y_tr.copy(), x_te.copy(), y_te.copy())

        def generate_new_model(self):
            clf = Titanic.LogisticRegression()
            clf.classes_ = np.array([0, 1])
            clf.metrics_names = ["log_loss", "Accuracy"]
            return clf

    out = []
    for P, amounts, E, M in ((3, [0.2, 0.5, 0.3], 3, 1), (5, [0.2] * 5, 2, 1), (10, [0.1] * 10, 3, 1)):
        ds = SynthTitanic()
        sc = mplc.scenario.Scenario(P, amounts, dataset=ds, epoch_count=E, minibatch_count=M,
                                    experiment_path=__import__("pathlib").Path("/tmp/mplc_golden_exp"))
        sc.instantiate_scenario_partners()
        sc.split_data(is_logging_enabled=False)
        sc.compute_batch_sizes()
        sc.save_folder = __import__("pathlib").Path("/tmp/mplc_golden_exp/save")
        os.makedirs(sc.save_folder, exist_ok=True)
        np.random.seed(0)
        mpl = sc.multi_partner_learning_approach(sc, partners_list=np.array(sc.partners_list),
                                                 is_early_stopping=True, is_save_data=False)
        mpl.fit()
        hist = {str(k): {m: np.asarray(v, dtype=float).tolist() for m, v in d.items()}
                for k, d in mpl.history.history.items()}
        out.append({"partners_count": P, "epoch_count": E, "minibatch_count": M, "score": float(mpl.history.score),
                    "history": hist})
        print(f"lr history P={P}", flush=True)
    return out


# --------------------------------------------------------------------------------------------------
# (e) Federated step-by-step scores on synthetic learning histories
# --------------------------------------------------------------------------------------------------
def gen_sbs(mplc):
    """mplc/contributivity.py:1015-1115 on seeded History.history dicts (partners' val_accuracy per
    (epoch, minibatch), NaN where unlogged; the collective model's val_accuracy, 0 where unlogged)."""
    out = []
    for case, (P, E, M, stop, holes) in enumerate(((3, 3, 4, None, 0), (4, 5, 6, 3, 3), (2, 2, 10, None, 2),
                                                    (5, 1, 7, None, 0), (3, 4, 5, 2, 0))):
        rng = np.random.default_rng(500 + case)
        coll = np.zeros((E, M))
        parts = [np.full((E, M), np.nan) for _ in range(P)]
        done = E if stop is None else stop
        coll[:done] = rng.uniform(0.1, 0.95, size=(done, M))
        for p in range(P):
            parts[p][:done] = rng.uniform(0.05, 0.95, size=(done, M))
        for _ in range(holes):  # partners with no fit logged in a round
            parts[int(rng.integers(P))][int(rng.integers(done)), int(rng.integers(M))] = np.nan
        hist = {i: {"val_accuracy": parts[i]} for i in range(P)}
        hist["mpl_model"] = {"val_accuracy": coll}
        mpl = types.SimpleNamespace(history=types.SimpleNamespace(history=hist), partners_count=P,
                                    epoch_count=E, minibatch_count=M)
        partners = [types.SimpleNamespace(id=i) for i in range(P)]
        scenario = types.SimpleNamespace(partners_list=partners, mpl=mpl,
                                         multi_partner_learning_approach=mplc.multi_partner_learning.FederatedAverageLearning)
        res = {"P": P, "E": E, "M": M, "collective": coll.tolist(), "partners": [x.tolist() for x in parts]}
        for method in ("Federated SBS linear", "Federated SBS quadratic", "Federated SBS constant"):
            contrib = mplc.contributivity.Contributivity(scenario=scenario)
            with np.errstate(all="ignore"):
                contrib.compute_contributivity(method)
            res[method] = {"name": contrib.name,
                           "scores": [float(x) for x in np.atleast_1d(contrib.contributivity_scores)],
                           "normalized": [float(x) for x in np.atleast_1d(contrib.normalized_scores)],
                           "std": [float(x) for x in np.atleast_1d(contrib.scores_std)]}
        out.append(res)
        print(f"sbs case {case}: P={P} E={E} M={M}", flush=True)
    return out


def main():
    only = set(sys.argv[1:])
    mplc = import_reference()
    jobs = {"shapley_value": gen_shapley, "estimators": gen_estimators, "splits": gen_splits,
            "fedavg_lr": gen_fedavg_lr, "sbs": gen_sbs, "lr_history": gen_lr_history}
    for name, fn in jobs.items():
        if only and name not in only:
            continue
        data = fn(mplc)
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump({"generator": "tests/golden/make_golden.py", "reference": "mshuaic/distributed-learning-"
                       "contributivity @ /root/reference", "data": data}, f)
        print("wrote", name, flush=True)


if __name__ == "__main__":
    main()
