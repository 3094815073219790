"""Contributivity measurement - drop-in for mplc/contributivity.py (reference lines cited per method).

The public surface is the reference's: ``Contributivity(scenario, name="")``,
``compute_contributivity(method_to_compute, sv_accuracy=0.01, alpha=0.95, truncation=0.05, update=50)``,
``not_twice_characteristic(subset)`` and the result fields (name, contributivity_scores, scores_std,
normalized_scores, computation_time_sec, first_charac_fct_calls_count, charac_fct_values,
increments_values).  Estimators consume the global numpy RNG in exactly the reference's order, so on
a fixed v(S) table every method reproduces the reference bit for bit (tests/test_contributivity.py
against tests/golden/estimators.json).

What changes is where v(S) comes from.  When the scenario's learning approach is engine-backed (it
exposes ``evaluate_coalitions``), the estimators first PLAN the coalitions they are about to need and
have them trained as one batch on the MI355X (exact Shapley: all 2^n - 1; Independent: the n
singletons; TMCS/ITMCS: the truncation frontier of a wave of speculatively drawn permutations; SMCS /
WR_SMC / IS: one sampling iteration ahead).  Those values land in a per-scenario coalition cache;
``not_twice_characteristic`` then runs the reference's memo logic unchanged on top of it, so the memo,
the increments and ``first_charac_fct_calls_count`` are exactly what the sequential reference records.
v(S) is a deterministic function of (S, seed) in the engine, so sharing the cache across methods changes
no result (the reference retrains per method, mplc/scenario.py:872-876, with unseeded TF).

Exact Shapley aggregation runs on device (mplc.shapley, csrc/shapley.hip).
"""
import datetime
import logging
from itertools import combinations
from math import factorial
from timeit import default_timer as timer

import numpy as np
from scipy.stats import norm

from . import multi_partner_learning, constants
from .coalitions import tuple_to_mask

logger = logging.getLogger("mplc")


# ------------------------------------------------------------------------------------------------
# Kriging surrogate used by AIS (reference mplc/contributivity.py:22-61)
# ------------------------------------------------------------------------------------------------
class KrigingModel:
    """Universal kriging with polynomial trend in sum(x) of degree `degre` (mplc/contributivity.py:22-61)."""

    def __init__(self, degre, covariance_func):
        self.degre = degre
        self.cov_f = covariance_func
        self.X = np.array([[]])
        self.Y = np.array([[]])
        self.beta = np.array([[]])
        self.H = np.array([[]])
        self.K = np.array([[]])
        self.invK = np.array([[]])

    def fit(self, X, Y):
        self.X, self.Y = X, Y
        m = len(X)
        gram = np.zeros((m, m))
        trend = np.zeros((m, self.degre + 1))
        for a, xa in enumerate(X):
            for b, xb in enumerate(X):
                gram[a, b] = self.cov_f(xa, xb)
            for d in range(self.degre + 1):
                trend[a, d] = np.sum(xa) ** d
        self.H = trend
        self.K = np.linalg.inv(gram)
        self.invK = np.linalg.inv(gram)
        ht_ik_h = trend.transpose().dot(self.invK).dot(trend)
        self.beta = np.linalg.inv(ht_ik_h).dot(trend.transpose()).dot(self.invK).dot(self.Y)

    def predict(self, x):
        g = np.array([np.sum(x) ** d for d in range(self.degre + 1)])
        c = np.array([[self.cov_f(self.X[a], x)] for a in range(len(self.X))])
        return g.transpose().dot(self.beta) + c.transpose().dot(self.invK).dot(self.Y - self.H.dot(self.beta))


def _first_index_above(ratios, u):
    """Index of the first entry with ratio > u in a non-decreasing cumulative array (the inverse-CDF
    scans of mplc/contributivity.py:413-422, 785-792), or None if none exceeds u."""
    i = int(np.searchsorted(ratios, u, side="right"))
    return i if i < len(ratios) else None


class Contributivity:
    """Per-method contributivity state (mplc/contributivity.py:64-75)."""

    def __init__(self, scenario, name=""):
        self.name = name
        self.scenario = scenario
        nb_partners = len(self.scenario.partners_list)
        self.contributivity_scores = np.zeros(nb_partners)
        self.scores_std = np.zeros(nb_partners)
        self.normalized_scores = np.zeros(nb_partners)
        self.computation_time_sec = 0.0
        self.first_charac_fct_calls_count = 0
        self.charac_fct_values = {(): 0}
        self.increments_values = [{} for _ in self.scenario.partners_list]
        self._start = None

    def __str__(self):
        txt = "\n" + self.name + "\n"
        txt += "Computation time: " + str(datetime.timedelta(seconds=self.computation_time_sec)) + "\n"
        txt += "Number of characteristic function computed: " + str(self.first_charac_fct_calls_count) + "\n"
        txt += f"Contributivity scores: {np.round(self.contributivity_scores, 3)}\n"
        txt += f"Std of the contributivity scores: {np.round(self.scores_std, 3)}\n"
        txt += f"Normalized contributivity scores: {np.round(self.normalized_scores, 3)}\n"
        return txt

    # --------------------------------------------------------------------------------------------
    # v(S): engine cache + batched planning
    # --------------------------------------------------------------------------------------------
    @property
    def _n(self):
        return len(self.scenario.partners_list)

    def _batched_evaluator(self):
        approach = getattr(self.scenario, "multi_partner_learning_approach", None)
        return getattr(approach, "evaluate_coalitions", None)

    def _cache(self):
        cache = getattr(self.scenario, "coalition_values", None)
        if cache is None:
            cache = {}
            try:
                self.scenario.coalition_values = cache
            except AttributeError:
                pass
        return cache

    def prefetch(self, subsets):
        """Batch-evaluate the not-yet-known coalitions among `subsets` on the engine (no effect on the memo
        or the call count; those follow the reference's sequential semantics in not_twice_characteristic)."""
        evaluate = self._batched_evaluator()
        if evaluate is None:
            return
        cache = self._cache()
        todo, seen = [], set()
        for s in subsets:
            key = tuple(sorted(int(i) for i in s))
            if len(key) == 0 or key in cache or key in self.charac_fct_values or key in seen:
                continue
            seen.add(key)
            todo.append(key)
        if todo:
            values = evaluate(self.scenario, todo)
            for k, v in zip(todo, values):
                cache[k] = float(v)

    def _world_size(self):
        from .parallel import world
        return world()[1]

    def _lookahead(self, per_iteration):
        """Sampling iterations to plan ahead so that one planned batch holds about `mc_plan_coalitions`
        (default 512) coalitions per rank - several hundred replicas per GPU launch (SMCS batches
        of <= 2N coalitions left the GPU idle).  Speculation never changes a result: v(S) is a deterministic
        function of (S, seed), planning restores the RNG state, and draws that the real loop does not make
        only cost compute."""
        target = int(getattr(self.scenario, "mc_plan_coalitions", 512)) * self._world_size()
        return max(1, target // max(1, per_iteration))

    def _known(self, key):
        return key in self.charac_fct_values or key in self._cache()

    def _coalition_value(self, key):
        cache = self._cache()
        if key in cache:
            return cache[key]
        if self._batched_evaluator() is not None:
            self.prefetch([key])
            return cache[key]
        # plain approach class: the reference's per-coalition construction (mplc/contributivity.py:100-114)
        partners = np.array([self.scenario.partners_list[i] for i in key])
        if len(partners) > 1:
            mpl = self.scenario.multi_partner_learning_approach(self.scenario, partners_list=partners,
                                                                is_early_stopping=True, is_save_data=False)
        else:
            mpl = multi_partner_learning.SinglePartnerLearning(self.scenario, partner=partners[0],
                                                               is_early_stopping=True, is_save_data=False)
        mpl.fit()
        return mpl.history.score

    def not_twice_characteristic(self, subset):
        """Memoised v(S) plus the increment bookkeeping of mplc/contributivity.py:92-136."""
        return self._not_twice_key(tuple(sorted(int(i) for i in subset)))

    def _not_twice_key(self, key):
        """not_twice_characteristic for a key already in normal form (a sorted tuple of ints)."""
        values = self.charac_fct_values
        if key not in values:
            self.first_charac_fct_calls_count += 1
            v = values[key] = self._coalition_value(key)
            inc = self.increments_values
            # the reference's loop over i in 0..n-1 (same order, same keys and values): a member's key without it
            # is key minus one slot; a non-member's key with it is key with i inserted at its sorted position
            pos = 0  # members of key below i
            for i in range(self._n):
                if pos < len(key) and key[pos] == i:
                    without = key[:pos] + key[pos + 1:]
                    if without in values:
                        inc[i][without] = v - values[without]
                    pos += 1
                else:
                    with_i = key[:pos] + (i,) + key[pos:]
                    if with_i in values:
                        inc[i][key] = values[with_i] - v
        return values[key]

    # --------------------------------------------------------------------------------------------
    # result helpers
    # --------------------------------------------------------------------------------------------
    def _begin(self):
        self._start = timer()

    def _finish(self, name, scores, std):
        self.name = name
        self.contributivity_scores = scores
        self.scores_std = std
        self.normalized_scores = self.contributivity_scores / np.sum(self.contributivity_scores)
        self.computation_time_sec = timer() - self._start

    def _single_partner(self, name, v_all):
        self._finish(name, np.array([v_all]), np.array([0]))

    def _sizes(self):
        return [len(p.y_train) for p in self.scenario.partners_list]

    # --------------------------------------------------------------------------------------------
    # Exact Shapley (mplc/contributivity.py:140-171) and independent scores (:174-192)
    # --------------------------------------------------------------------------------------------
    def compute_SV(self):
        from .shapley import shapley_value
        self._begin()
        logger.info("# Launching computation of Shapley Value of all partners")
        n = self._n
        coalitions = [c for r in range(1, n + 1) for c in combinations(range(n), r)]  # sorted int tuples
        self.prefetch(coalitions)
        char_values = [self._not_twice_key(c) for c in coalitions]
        # every rank holds the same (all-reduced) values here, so the sum may be range-sharded across them
        sv = shapley_value(n, char_values, sharded=True)
        self.name = "Shapley"
        self.contributivity_scores = np.array(sv)
        self.scores_std = np.zeros(len(sv))
        self.normalized_scores = sv / np.sum(sv)
        self.computation_time_sec = timer() - self._start

    def compute_independent_scores(self):
        self._begin()
        logger.info("# Launching computation of perf. scores of models trained independently on each partner")
        n = self._n
        self.prefetch([(i,) for i in range(n)])
        scores = [self.not_twice_characteristic(np.array([i])) for i in range(n)]
        self.name = "Independent scores raw"
        self.contributivity_scores = np.array(scores)
        self.scores_std = np.zeros(len(scores))
        self.normalized_scores = scores / np.sum(scores)
        self.computation_time_sec = timer() - self._start

    # --------------------------------------------------------------------------------------------
    # Truncated Monte-Carlo (mplc/contributivity.py:195-253) and interpolated TMC (:257-322)
    # --------------------------------------------------------------------------------------------
    def _device_table(self):
        """The device v(S) table (mplc.mc.VTable) holding every value known to this method so far."""
        table = getattr(self, "_vtable", None)
        if table is None:
            from .mc import VTable
            table = self._vtable = VTable(self._n)
        known = dict(self._cache())
        known.update(self.charac_fct_values)
        table.update(known)
        return table

    def _frontier_plan(self, n, v_all, truncation):
        """plan(perms, stop) -> keys for one frontier step of a permutation wave (mplc.mc.plan_frontier): the
        required first unknown prefixes plus the speculative deeper prefixes whose expected waste stays within one
        batch's fixed cost (`mc_plan_overhead`, default 8 replica-trainings per rank), at most `mc_plan_replicas`
        (default 4096) replicas per rank, so that the tail of a wave does not run as many tiny lockstep batches
        (config #4's TMCS batches averaged 92 replicas).  mc_plan_replicas = 0 turns speculation off."""
        from .mc import plan_frontier, size_predictor
        ws = self._world_size()
        target = int(getattr(self.scenario, "mc_plan_replicas", 4096)) * ws
        # a batch's fixed cost in replica-trainings; per rank the replicas are 1/ws of the batch
        overhead = float(getattr(self.scenario, "mc_plan_overhead", 8.0)) * ws
        cache = self._cache()
        known = self.charac_fct_values

        def value(key):
            return known[key] if key in known else cache.get(key)

        def plan(perms, stop):
            pred = size_predictor(((k, v) for d in (cache, known) for k, v in d.items()), n, v_all)
            keys, required = plan_frontier(perms, stop, value, pred, v_all, truncation, target, overhead)
            st = self.__dict__.setdefault("plan_stats", {"frontier_steps": 0, "required": 0, "speculative": 0})
            st["frontier_steps"] += 1
            st["required"] += required
            st["speculative"] += len(keys) - required
            return keys
        return plan, value

    def _prefetch_permutation_wave(self, n, v_all, truncation, wave, interpolate=False, sizes=None):
        """Draw the next `wave` permutations WITHOUT consuming the global RNG, walk each one's prefixes up
        to its truncation point, and batch-evaluate the uncached prefixes the walks stop on (plus speculative
        deeper ones, _frontier_plan) at once; repeat until every walk is complete.  These are the coalitions
        the sequential loop will ask for on those permutations.  With the MI355X engine the walks and their
        truncation tests run on device (mplc.mc.wave_frontier, csrc/mc_shapley.hip); a plain evaluator (CPU test
        harness) is walked here in Python."""
        if self._batched_evaluator() is None:
            return
        state = np.random.get_state()
        perms = np.array([np.random.permutation(n) for _ in range(wave)])
        np.random.set_state(state)
        plan, value = self._frontier_plan(n, v_all, truncation)
        approach = getattr(self.scenario, "multi_partner_learning_approach", None)
        if getattr(approach, "device_planning", False) and n <= 24:
            from .mc import wave_frontier

            def evaluate(keys):
                self.prefetch(keys)
                cache = self._cache()
                return [cache[k] if k in cache else self.charac_fct_values[k] for k in keys]
            wave_frontier(self._device_table(), perms, v_all, truncation, interpolate, sizes, evaluate, plan=plan)
            return
        while True:
            stop = np.full(wave, n)
            for w in range(wave):
                char = 0.0
                for j in range(n):
                    if abs(v_all - char) < truncation:
                        break  # truncated: no further coalition on this permutation
                    v = value(tuple(sorted(int(i) for i in perms[w, :j + 1])))
                    if v is None:
                        stop[w] = j
                        break
                    char = v
            if np.all(stop >= n):
                return
            self.prefetch(plan(perms, stop))

    def _truncated_loop(self, n, v_all, sv_accuracy, alpha, truncation, interpolate):
        rows = np.zeros((128, n))
        t = 0
        q = norm.ppf((1 - alpha) / 2, loc=0, scale=1)
        v_max = 0
        wave = 0
        sizes = self._sizes()
        while t < 100 or t < q ** 2 * v_max / sv_accuracy ** 2:
            if t >= wave:
                # waves grow with the world size so that every rank's frontier batches stay as large as one
                # GPU's (mc_wave_scale overrides); more permutations per wave only adds speculation
                scale = int(getattr(self.scenario, "mc_wave_scale", 0) or self._world_size())
                span = (100 if t < 100 else 50) * scale
                if t >= 100 and getattr(self.scenario, "mc_wave_adaptive", True):
                    # past the first 100 walks the stopping rule itself estimates how many walks are still to
                    # come; drawing half of them at once (at most 8 waves) merges the small tails of consecutive
                    # waves into one frontier.  Walks the loop then does not make are speculation only.
                    remaining = q ** 2 * v_max / sv_accuracy ** 2 - t
                    span = max(span, min(int(0.5 * remaining), 8 * span))
                self._prefetch_permutation_wave(n, v_all, truncation, span, interpolate, sizes)
                wave = t + span
            t += 1
            if t > rows.shape[0]:
                rows = np.vstack((rows, np.zeros_like(rows)))
            rows[t - 1] = 0.0
            perm = np.random.permutation(n)
            chars = np.zeros(n + 1)
            chars[-1] = v_all
            slope = None
            for j in range(n):
                if abs(v_all - chars[j]) < truncation:
                    if not interpolate:
                        chars[j + 1] = chars[j]
                    else:
                        if slope is None:
                            # reference quirk kept: sizes of partners j..n-1 in INDEX order, not permutation
                            # order (mplc/contributivity.py:297-306)
                            rest = 0
                            for i in range(j, n):
                                rest += sizes[i]
                            slope = (v_all - chars[j]) / rest
                        chars[j + 1] = chars[j] + slope * sizes[j]
                else:
                    chars[j + 1] = self.not_twice_characteristic(perm[: j + 1])
                rows[t - 1][perm[j]] = chars[j + 1] - chars[j]
            v_max = np.max(np.var(rows[:t], axis=0))
        contributions = rows[:t]
        self.mc_walks = t  # permutations the estimator consumed (the waves may have drawn more)
        return np.mean(contributions, axis=0), np.std(contributions, axis=0) / np.sqrt(t - 1)

    def truncated_MC(self, sv_accuracy=0.01, alpha=0.9, truncation=0.05):
        self._begin()
        n = self._n
        v_all = self.not_twice_characteristic(np.arange(n))
        if n == 1:
            return self._single_partner("TMC Shapley", v_all)
        sv, std = self._truncated_loop(n, v_all, sv_accuracy, alpha, truncation, interpolate=False)
        self._finish("TMC Shapley", sv, std)

    def interpol_TMC(self, sv_accuracy=0.01, alpha=0.9, truncation=0.05):
        self._begin()
        n = self._n
        v_all = self.not_twice_characteristic(np.arange(n))
        if n == 1:
            return self._single_partner("ITMCS", v_all)
        sv, std = self._truncated_loop(n, v_all, sv_accuracy, alpha, truncation, interpolate=True)
        self._finish("ITMCS", sv, std)

    # --------------------------------------------------------------------------------------------
    # Importance sampling (mplc/contributivity.py:326-439 linear, :443-569 regression)
    # --------------------------------------------------------------------------------------------
    def _prob(self, n, size):
        return factorial(n - 1 - size) * factorial(size) / factorial(n)

    def _importance_tables(self, n, approx_for):
        """Per player k: the combination-ordered subsets of the others and the running cumSum / renorm
        ratios of the reference's inverse-CDF scan (same sequential sums, mplc/contributivity.py:380-393)."""
        tables = []
        renorms = []
        for k in range(n):
            others = [i for i in range(n) if i != k]
            subsets, cums = [], []
            acc = 0
            for length in range(len(others) + 1):
                for sub in combinations(others, length):
                    acc += self._prob(n, len(sub)) * np.abs(approx_for(sub, k))
                    subsets.append(sub)
                    cums.append(acc)
            renorms.append(acc)
            tables.append((subsets, np.asarray(cums, dtype=np.float64) / acc if acc != 0 else np.full(len(cums), np.nan)))
        return tables, renorms

    def _importance_loop(self, n, sv_accuracy, alpha, tables, renorms, approx_for):
        q = -norm.ppf((1 - alpha) / 2, loc=0, scale=1)
        rows = np.zeros((128, n))
        t = 0
        v_max = 0
        S = None
        planned_until = 0
        while t < 100 or t < 4 * q ** 2 * v_max / sv_accuracy ** 2:
            t += 1
            if t > rows.shape[0]:
                rows = np.vstack((rows, np.zeros_like(rows)))
            rows[t - 1] = 0.0
            # the sampling tables are fixed for the whole loop, so the draws of the next iterations are known
            # exactly: plan several iterations on a copy of the RNG state, batch the coalitions they need
            if self._batched_evaluator() is not None and t > planned_until:
                K = self._lookahead(2 * n)
                self.prefetch(self._plan_importance(n, tables, K, S))
                planned_until = t + K - 1
            for k in range(n):
                u = np.random.uniform(0, 1, 1)[0]
                idx = _first_index_above(tables[k][1], u)
                if idx is not None:
                    S = np.array(tables[k][0][idx])
                if S is None:
                    raise UnboundLocalError("local variable 'S' referenced before assignment")
                SUk = np.append(S, k)
                increment = self.not_twice_characteristic(SUk) - self.not_twice_characteristic(S)
                rows[t - 1][k] = increment * renorms[k] / np.abs(approx_for(tuple(int(i) for i in S), k))
            v_max = np.max(np.var(rows[:t], axis=0))
        contributions = rows[:t]
        self.mc_walks = t  # permutations the estimator consumed (the waves may have drawn more)
        return np.mean(contributions, axis=0), np.std(contributions, axis=0) / np.sqrt(t - 1)

    @staticmethod
    def _plan_importance(n, tables, iterations, S):
        """Coalitions the importance-sampling loop will ask for in its next `iterations` iterations (one
        uniform per player per iteration, mplc/contributivity.py:405-431), drawn from a saved RNG state."""
        state = np.random.get_state()
        plan = []
        cur = None if S is None else tuple(int(i) for i in S)
        for _ in range(iterations):
            for k in range(n):
                idx = _first_index_above(tables[k][1], np.random.uniform(0, 1, 1)[0])
                if idx is not None:
                    cur = tables[k][0][idx]
                if cur is None:
                    break
                plan += [tuple(sorted(cur + (k,))), cur]
        np.random.set_state(state)
        return plan

    def IS_lin(self, sv_accuracy=0.01, alpha=0.95):
        self._begin()
        n = self._n
        v_all = self.not_twice_characteristic(np.arange(n))
        if n == 1:
            return self._single_partner("IS_lin Shapley", v_all)
        self.prefetch([tuple(i for i in range(n) if i != k) for k in range(n)] + [(k,) for k in range(n)])
        last_inc, first_inc = [], []
        for k in range(n):
            last_inc.append(v_all - self.not_twice_characteristic(np.delete(np.arange(n), k)))
            first_inc.append(self.not_twice_characteristic(np.array([k])) - 0)
        sizes = self._sizes()
        size_all = 0
        for s in sizes:
            size_all += s
        memo = {}

        def approx_for(sub, k):
            # depends on sum of sizes only (mplc/contributivity.py:369-377)
            size_S = 0
            for i in sub:
                size_S += sizes[i]
            key = (size_S, k)
            if key not in memo:
                beta = size_S / size_all
                memo[key] = (1 - beta) * first_inc[k] + beta * last_inc[k]
            return memo[key]

        tables, renorms = self._importance_tables(n, approx_for)
        sv, std = self._importance_loop(n, sv_accuracy, alpha, tables, renorms, approx_for)
        self._finish("IS_lin Shapley", sv, std)

    def IS_reg(self, sv_accuracy=0.01, alpha=0.95):
        from sklearn.linear_model import LinearRegression
        self._begin()
        n = self._n
        if n < 4:
            self.compute_SV()
            self.name = "IS_reg Shapley values"
            return
        # seed increments along 2 + n rotated permutations (mplc/contributivity.py:462-472)
        perm = np.random.permutation(n)
        walks = [perm, np.flip(perm)]
        p = walks[-1]
        for _ in range(n):
            p = np.append(p[-1], p[:-1])
            walks.append(p)
        self.prefetch([tuple(sorted(int(i) for i in w[: j + 1])) for w in walks for j in range(n)])
        for w in walks:
            for j in range(n):
                self.not_twice_characteristic(w[: j + 1])
        sizes = self._sizes()

        def features(sub):
            size_S = 0
            for i in sub:
                size_S += sizes[i]
            return [size_S, size_S ** 2]

        models = []
        for k in range(n):
            X = [features(sub) for sub in self.increments_values[k]]
            y = list(self.increments_values[k].values())
            models.append(LinearRegression().fit(X, y))
        memo = {}

        def approx_for(sub, k):
            f = features(sub)
            key = (f[0], k)
            if key not in memo:
                memo[key] = models[k].predict([f])[0]
            return memo[key]

        tables, renorms = self._importance_tables(n, approx_for)
        sv, std = self._importance_loop(n, sv_accuracy, alpha, tables, renorms, approx_for)
        self._finish("IS_reg Shapley", sv, std)

    # --------------------------------------------------------------------------------------------
    # Adaptive importance sampling with Kriging (mplc/contributivity.py:573-723)
    # --------------------------------------------------------------------------------------------
    def AIS_Kriging(self, sv_accuracy=0.01, alpha=0.95, update=50):
        self._begin()
        n = self._n
        full = np.arange(n)
        seeds = [tuple(range(n))]
        for k1 in range(n):
            for k2 in range(n):
                seeds += [(k1,), tuple(np.delete(full, [k1]))]
                if k1 != k2:
                    seeds += [tuple(sorted((k1, k2))), tuple(np.delete(full, [k1, k2]))]
        self.prefetch(seeds)
        self.not_twice_characteristic(full)
        for k1 in range(n):
            for k2 in range(n):
                self.not_twice_characteristic(np.array([k1]))
                self.not_twice_characteristic(np.delete(full, [k1]))
                if k1 != k2:
                    self.not_twice_characteristic(np.array([k1, k2]))
                    self.not_twice_characteristic(np.delete(full, [k1, k2]))
        sizes = self._sizes()

        def coordinate(sub, k):
            c = np.zeros(n)
            for i in sub:
                c[i] = sizes[i]
            return np.delete(c, k)

        phi = np.zeros(n)
        for k in range(n):
            phi[k] = np.median(coordinate(np.delete(full, k), k))

        # Reference closure quirk (mplc/contributivity.py:618-624): each covk reads phi[k] through the
        # late-bound loop variable k of AIS_Kriging's own scope, i.e. the k of whatever loop is running
        # when the covariance is evaluated: n - 1 while models are fitted, the current player while the
        # renormalisation and sampling loops predict.  `live_k` reproduces that binding.
        live_k = [n - 1]

        def cov(x1, x2):
            return np.exp(-np.sqrt(np.sum((x1 - x2) ** 2)) ** 2 / phi[live_k[0]] ** 2)

        generations = []
        gen_tables = []

        def refit():
            models = []
            for k in range(n):
                X = [coordinate(sub, k) for sub in self.increments_values[k]]
                Y = [v for v in self.increments_values[k].values()]
                m = KrigingModel(2, cov)
                m.fit(X, Y)
                models.append(m)
            generations.append(models)

        q = -norm.ppf((1 - alpha) / 2, loc=0, scale=1)
        t = 0
        v_max = 0
        contributions = None
        S = None
        j = 0
        planned_until = 0
        while t < 100 or t < 4 * q ** 2 * v_max / sv_accuracy ** 2:
            if t == 0:
                contributions = np.array([np.zeros(n)])
            else:
                contributions = np.vstack((contributions, np.zeros(n)))
            if t % update == 0:
                j = t // update
                live_k[0] = n - 1
                refit()
                memo = {}

                def approx_for(sub, k, _models=generations[j], _memo=memo):
                    key = (tuple(sub), k)
                    if key not in _memo:
                        live_k[0] = k
                        _memo[key] = _models[k].predict(coordinate(sub, k))[0]
                    return _memo[key]

                tables, renorms = self._importance_tables(n, approx_for)
                gen_tables.append((tables, renorms, approx_for))
            tables, renorms, approx_for = gen_tables[j]
            if self._batched_evaluator() is not None and t >= planned_until:
                # exact up to the next refit (the tables of this generation are fixed until then)
                K = min(self._lookahead(2 * n), update - t % update)
                self.prefetch(self._plan_importance(n, tables, K, S))
                planned_until = t + K
            for k in range(n):
                u = np.random.uniform(0, 1, 1)[0]
                idx = _first_index_above(tables[k][1], u)
                if idx is not None:
                    S = np.array(tables[k][0][idx])
                if S is None:
                    raise UnboundLocalError("local variable 'S' referenced before assignment")
                SUk = np.append(S, k)
                increment = self.not_twice_characteristic(SUk) - self.not_twice_characteristic(S)
                # reference indexing kept: row t - 1 (the last row at t = 0) (mplc/contributivity.py:709)
                contributions[t - 1][k] = increment * renorms[k] / np.abs(approx_for(tuple(int(i) for i in S), k))
            v_max = np.max(np.var(contributions, axis=0))
            t += 1
        self._finish("AIS Shapley", np.mean(contributions, axis=0),
                     np.std(contributions, axis=0) / np.sqrt(t - 1))

    # --------------------------------------------------------------------------------------------
    # Stratified MC (mplc/contributivity.py:727-819) and without-replacement SMC (:823-938)
    # --------------------------------------------------------------------------------------------
    def _stratum_cdf(self, N, strata):
        """cumSum after each combination of one stratum, added sequentially (mplc/contributivity.py:786-792)."""
        cache = getattr(self, "_cdf_cache", None)
        if cache is None:
            cache = self._cdf_cache = {}
        key = (N, strata)
        if key not in cache:
            step = factorial(N - 1 - strata) * factorial(strata) / factorial(N - 1)
            count = factorial(N - 1) // (factorial(N - 1 - strata) * factorial(strata))
            vals = np.empty(count)
            acc = 0
            for i in range(count):
                acc += step
                vals[i] = acc
            cache[key] = vals
        return cache[key]

    @staticmethod
    def _unrank_combination(items, size, rank):
        """The rank-th combination (lexicographic, as itertools.combinations) of `size` elements of items."""
        out = []
        m = len(items)
        start = 0
        for slot in range(size):
            for i in range(start, m):
                block = _binom(m - i - 1, size - slot - 1)
                if rank < block:
                    out.append(items[i])
                    start = i + 1
                    break
                rank -= block
        return tuple(out)

    def _stratified_pick(self, N, k, strata, u):
        cdf = self._stratum_cdf(N, strata)
        idx = _first_index_above(cdf, u)
        if idx is None:
            return None
        others = [i for i in range(N) if i != k]
        return self._unrank_combination(others, strata, idx)

    def Stratified_MC(self, sv_accuracy=0.01, alpha=0.95):
        self._begin()
        N = self._n
        v_all = self.not_twice_characteristic(np.arange(N))
        if N == 1:
            return self._single_partner("Stratified MC Shapley", v_all)
        gamma, beta = 0.2, 0.0075
        t = 0
        sigma2 = np.zeros((N, N))
        mu = np.zeros((N, N))
        v_max = 0
        keep_going = [[True] * N for _ in range(N)]
        samples = [[[] for _ in range(N)] for _ in range(N)]
        S = None
        var = np.zeros(N)
        planned_until = 0

        def exploration(t):
            return 1 + 1 / (1 + np.exp(gamma / beta)) - 1 / (1 + np.exp(-(t - gamma * N) / (beta * N)))

        def allocation(k, e):
            if np.sum(sigma2[k]) == 0:
                return np.repeat(1 / N, N)
            return np.repeat(1 / N, N) * (1 - e) + sigma2[k] / np.sum(sigma2[k]) * e

        def plan(t0, iterations):
            """Draws of iterations t0, t0+1, ... from a saved RNG state with sigma2 as it stands.  Every draw
            consumes one uniform (np.random.choice with p) plus one (the subset), whatever the values, so
            the stream stays aligned; within iteration t0 the plan is exact (player k's allocation only
            depends on sigma2[k] from earlier iterations), later ones speculate that sigma2 does not move
            the stratum draw (after the first ~gamma*N iterations the exploration weight e is ~1e-12)."""
            state = np.random.get_state()
            out = []
            cur = S
            for tt in range(t0, t0 + iterations):
                e_t = exploration(tt)
                for k in range(N):
                    st = np.random.choice(np.arange(N), 1, p=allocation(k, e_t))[0]
                    sub = self._stratified_pick(N, k, st, np.random.uniform(0, 1, 1)[0])
                    if sub is not None:
                        cur = sub
                    if cur is not None:
                        cur = tuple(int(i) for i in cur)
                        out += [tuple(sorted(cur + (k,))), cur]
            np.random.set_state(state)
            return out

        while np.any(keep_going) or (1 - alpha) < v_max / (sv_accuracy ** 2):
            t += 1
            e = exploration(t)

            def alloc(k):
                return allocation(k, e)

            if self._batched_evaluator() is not None:
                exact = plan(t, 1)
                if t > planned_until or not all(self._known(c) for c in exact):
                    # speculate only once the allocation has settled (e ~ 0): before that, each iteration
                    # is planned exactly on its own
                    K = self._lookahead(2 * N) if t > gamma * N + 8 else 1
                    self.prefetch(exact + (plan(t + 1, K - 1) if K > 1 else []))
                    planned_until = t + K - 1
            for k in range(N):
                strata = np.random.choice(np.arange(N), 1, p=alloc(k))[0]
                u = np.random.uniform(0, 1, 1)[0]
                sub = self._stratified_pick(N, k, strata, u)
                if sub is not None:
                    S = np.array(sub, dtype=int)
                if S is None:
                    raise UnboundLocalError("local variable 'S' referenced before assignment")
                SUk = np.append(S, k)
                increment = self.not_twice_characteristic(SUk) - self.not_twice_characteristic(S)
                samples[k][strata].append(increment)
                sigma2[k, strata] = np.var(samples[k][strata])
                mu[k, strata] = np.mean(samples[k][strata])
            shap = np.mean(mu, axis=1)
            var = np.zeros(N)
            for k in range(N):
                for strata in range(N):
                    cnt = len(samples[k][strata])
                    if cnt == 0:
                        var[k] = np.inf
                    else:
                        var[k] += sigma2[k, strata] ** 2 / cnt  # sigma2 squared: reference quirk (:809)
                    if cnt > 20:
                        keep_going[k][strata] = False
                var[k] /= N ** 2
            v_max = np.max(var)
        self.sampling_iterations = t  # the loop's iterations to its stopping rule (bench report)
        self._finish("Stratified MC Shapley", shap, np.sqrt(var))

    @staticmethod
    def _plan_wr_smc(N, iterations, keep_going, sigma2, drawn, pending):
        """Draws of the next `iterations` WR_SMC iterations (mplc/contributivity.py:858-900) from a saved RNG
        state.  The without-replacement bookkeeping is simulated exactly (pops from the pending lists, draw
        counts, the keep_going flags they switch off); once every stratum of a player is done the allocation
        follows sigma2, taken as it stands (speculation).  Pending lists are not copied (2^(N-1) entries per
        player at N=20): simulated pops are an overlay of removed positions."""
        state = np.random.get_state()
        out = []
        counts = [[len(drawn[k][s]) for s in range(N)] for k in range(N)]
        keep = [list(row) for row in keep_going]
        removed = {}
        full = [[len(pending[k][s]) + len(drawn[k][s]) for s in range(N)] for k in range(N)]
        for _ in range(iterations):
            for k in range(N):
                if np.any(keep[k]):
                    p = np.array(keep[k]) / np.sum(keep[k])
                elif np.sum(sigma2[k]) == 0:
                    continue
                else:
                    p = sigma2[k] / np.sum(sigma2[k])
                st = np.random.choice(np.arange(N), 1, p=p)[0]
                gone = removed.setdefault((k, st), [])
                L = len(pending[k][st]) - len(gone)
                if L <= 0:  # speculation ran into an exhausted stratum: stop planning here
                    np.random.set_state(state)
                    return out
                pick = np.random.choice(L, 1, p=np.repeat(1 / L, L))[0]
                # position `pick` of the list after the simulated pops -> position in the real list
                i = int(pick)
                for g in sorted(gone):
                    if g <= i:
                        i += 1
                gone.append(i)
                sub = tuple(int(v) for v in pending[k][st][i])
                out += [tuple(sorted(sub + (k,))), sub]
                counts[k][st] += 1
            for k in range(N):
                for s in range(N):
                    if counts[k][s] > 20 or counts[k][s] == full[k][s]:
                        keep[k][s] = False
        np.random.set_state(state)
        return out

    def without_replacment_SMC(self, sv_accuracy=0.01, alpha=0.95):
        self._begin()
        N = self._n
        v_all = self.not_twice_characteristic(np.arange(N))
        if N == 1:
            return self._single_partner("WR_SMC Shapley", v_all)
        t = 0
        sigma2 = np.zeros((N, N))
        mu = np.zeros((N, N))
        v_max = 0
        keep_going = [[True] * N for _ in range(N)]
        drawn = [[dict() for _ in range(N)] for _ in range(N)]
        pending = []
        for k in range(N):
            others = [i for i in range(N) if i != k]
            pending.append([list(combinations(others, strata)) for strata in range(N)])
        var = np.zeros(N)
        planned_until = 0
        while np.any(keep_going) or (1 - alpha) < v_max / (sv_accuracy ** 2):
            t += 1

            def alloc(k):
                if np.any(keep_going[k]):
                    return np.array(keep_going[k]) / np.sum(keep_going[k])
                if np.sum(sigma2[k]) == 0:
                    return None
                return sigma2[k] / np.sum(sigma2[k])

            if self._batched_evaluator() is not None:
                exact = self._plan_wr_smc(N, 1, keep_going, sigma2, drawn, pending)
                if t > planned_until or not all(self._known(c) for c in exact):
                    K = self._lookahead(2 * N)
                    self.prefetch(self._plan_wr_smc(N, K, keep_going, sigma2, drawn, pending))
                    planned_until = t + K - 1
            for k in range(N):
                p = alloc(k)
                if p is None:
                    continue
                strata = np.random.choice(np.arange(N), 1, p=p)[0]
                L = len(pending[k][strata])
                pick = np.random.choice(L, 1, p=np.repeat(1 / L, L))[0]
                sub = pending[k][strata].pop(pick)
                S = np.array(list(sub), dtype=int)
                SUk = np.append(S, k)
                increment = self.not_twice_characteristic(SUk) - self.not_twice_characteristic(S)
                drawn[k][strata][sub] = increment
                L = len(drawn[k][strata])
                mu[k, strata] = (mu[k, strata] * (L - 1) + increment) / L
                sigma2[k, strata] = 0
                for v in drawn[k][strata].values():
                    sigma2[k, strata] += (v - mu[k, strata]) ** 2
                if L > 1:
                    sigma2[k, strata] /= L - 1
                else:
                    sigma2[k, strata] = 0
                sigma2[k, strata] *= 1 / L - factorial(N - 1 - strata) * factorial(strata) / factorial(N - 1)
            shap = np.mean(mu, axis=1)
            var = np.zeros(N)
            for k in range(N):
                for strata in range(N):
                    cnt = len(drawn[k][strata])
                    if cnt == 0:
                        var[k] = np.inf
                    else:
                        var[k] += sigma2[k, strata] ** 2 / cnt
                    if cnt > 20:
                        keep_going[k][strata] = False
                    if len(drawn[k][strata]) == factorial(N - 1) / (factorial(N - 1 - strata) * factorial(strata)):
                        keep_going[k][strata] = False
                var[k] /= N ** 2
            v_max = np.max(var)
        self.sampling_iterations = t  # the loop's iterations to its stopping rule (bench report)
        self._finish("WR_SMC Shapley", shap, np.sqrt(var))

    # --------------------------------------------------------------------------------------------
    # Federated step-by-step scores (mplc/contributivity.py:1015-1115): post-processing of the recorded
    # history of the scenario's main learning run (scenario.mpl, Scenario.run); no coalition evaluations
    # --------------------------------------------------------------------------------------------
    def compute_relative_perf_matrix(self):
        """Per kept round (the first and last 10 % of the E*M rounds are skipped), each partner's
        val_accuracy after its fit divided by the round-start collective model's val_accuracy
        (mplc/contributivity.py:1079-1115).  Shape [kept rounds, partners]."""
        mpl = getattr(self.scenario, "mpl", None)
        hist = getattr(getattr(mpl, "history", None), "history", None)
        if not hist or "mpl_model" not in hist:
            raise RuntimeError("the Federated SBS methods read the learning history of the scenario's main "
                               "multi-partner run: call Scenario.run() (or fit a learner with record_history=True)")
        collective = np.asarray(hist["mpl_model"]["val_accuracy"])
        # [partners, E, M] -> [E, M, partners] as axis swaps (a strided view: the memory layout, and with it
        # the summation order of the score dot products below, is the reference's)
        per_partner = np.swapaxes(np.swapaxes([v["val_accuracy"] for k, v in hist.items() if k != "mpl_model"],
                                              0, 2), 0, 1)
        E, M = mpl.epoch_count, mpl.minibatch_count
        first = int(np.round(E * M * 0.1))
        last = int(np.round(E * M * (1 - 0.1)))
        with np.errstate(divide="ignore", invalid="ignore"):
            rel = np.divide(np.reshape(per_partner, (E * M, mpl.partners_count)),
                            np.reshape(collective, (E * M))[:, None])
        return rel[first:last, :]

    def _sbs(self, name, scores):
        self.name = name
        self.contributivity_scores = scores
        self.normalized_scores = self.contributivity_scores / np.sum(self.contributivity_scores)

    def federated_SBS_linear(self):
        start = timer()
        rel = self.compute_relative_perf_matrix()
        self._sbs("Federated step by step linear scores", np.arange(rel.shape[0]).dot(np.nan_to_num(rel)))
        self.computation_time_sec = timer() - start

    def federated_SBS_quadratic(self):
        start = timer()
        rel = self.compute_relative_perf_matrix()
        self._sbs("Federated step by step quadratic scores",
                  np.square(np.arange(rel.shape[0])).dot(np.nan_to_num(rel)))
        self.computation_time_sec = timer() - start

    def federated_SBS_constant(self):
        start = timer()
        rel = self.compute_relative_perf_matrix()
        with np.errstate(invalid="ignore"):
            self._sbs("Federated step by step constant scores", np.nanmean(rel, axis=0))
        self.computation_time_sec = timer() - start

    # --------------------------------------------------------------------------------------------
    # Dispatcher (mplc/contributivity.py:1134-1198)
    # --------------------------------------------------------------------------------------------
    OUT_OF_SCOPE = ("PVRL", "LFlip")
    SBS = {"Federated SBS linear": "federated_SBS_linear", "Federated SBS quadratic": "federated_SBS_quadratic",
           "Federated SBS constant": "federated_SBS_constant"}

    def compute_contributivity(self, method_to_compute, sv_accuracy=0.01, alpha=0.95, truncation=0.05,
                               update=50):
        dispatch = {
            "Shapley values": lambda: self.compute_SV(),
            "Independent scores": lambda: self.compute_independent_scores(),
            "TMCS": lambda: self.truncated_MC(sv_accuracy=sv_accuracy, alpha=alpha, truncation=truncation),
            "ITMCS": lambda: self.interpol_TMC(sv_accuracy=sv_accuracy, alpha=alpha, truncation=truncation),
            "IS_lin_S": lambda: self.IS_lin(sv_accuracy=sv_accuracy, alpha=alpha),
            "IS_reg_S": lambda: self.IS_reg(sv_accuracy=sv_accuracy, alpha=alpha),
            "AIS_Kriging_S": lambda: self.AIS_Kriging(sv_accuracy=sv_accuracy, alpha=alpha, update=update),
            "SMCS": lambda: self.Stratified_MC(sv_accuracy=sv_accuracy, alpha=alpha),
            "WR_SMC": lambda: self.without_replacment_SMC(sv_accuracy=sv_accuracy, alpha=alpha),
        }
        if method_to_compute in dispatch:
            dispatch[method_to_compute]()
        elif method_to_compute in self.SBS:
            approach = getattr(self.scenario, "multi_partner_learning_approach", None)
            if approach is not multi_partner_learning.FederatedAverageLearning:
                logger.warning(f"{method_to_compute}: step by step contributivity methods are only suited for "
                               "federated averaging learning approach")
            getattr(self, self.SBS[method_to_compute])()
        elif method_to_compute in self.OUT_OF_SCOPE:
            raise NotImplementedError(
                f"'{method_to_compute}' trains its own modified learner (label-flip / partner-selection policy) "
                "instead of evaluating coalitions; it is outside this engine's scope (DESIGN.md)")
        else:
            logger.warning("Unrecognized name of method, statement ignored!")


def _binom(a, b):
    if b < 0 or b > a:
        return 0
    return factorial(a) // (factorial(b) * factorial(a - b))


__all__ = ["Contributivity", "KrigingModel", "constants"]

# keep the reference's module-level names importable
from .shapley import shapley_value  # noqa: E402,F401


def power_set(List):
    """mplc/contributivity.py:1205-1207."""
    return [list(j) for i in range(len(List)) for j in combinations(List, i + 1)]


def coalition_mask(subset):
    return tuple_to_mask(subset)
