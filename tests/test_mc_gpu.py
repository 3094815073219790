"""GPU: Monte-Carlo Shapley permutation walks (csrc/mc_shapley.hip) against the reference.

- truncated_mc_table on each reference golden TMCS / ITMCS case (tests/golden/estimators.json: the
  reference's own outputs with np.random.seed on fixed tables) must reproduce scores and std BIT FOR BIT:
  device rows follow the reference's fp64 operation order, the stopping rule runs in numpy as the reference.
- the Contributivity estimators planned through the device walk (device_planning approach) must leave the
  memo, call count, scores and RNG stream of the sequential reference unchanged.
- walk rows on random tables equal a Python restatement of the reference loop exactly; the fixed-budget
  moments equal numpy's over the same rows (1e-12)."""
import numpy as np
import pytest

from test_contributivity import CASES, parse_table, run_case, same

pytestmark = pytest.mark.gpu

MC_CASES = [c for c in CASES if c["method"] in ("TMCS", "ITMCS") and not c["error"]]


def bitmask_table(case):
    n = case["n"]
    V = np.full(1 << n, np.nan)
    V[0] = 0.0
    for k, v in parse_table(case).items():
        V[sum(1 << i for i in k)] = v
    return V


def reference_rows(V, n, perms, v_all, trunc, interpolate, sizes):
    """mplc/contributivity.py:230-244 / :289-314 restated in Python floats."""
    rows = np.zeros((len(perms), n))
    for k, perm in enumerate(perms):
        char = [0.0] * (n + 1)
        char[-1] = v_all
        first, a, mask = True, 0.0, 0
        for j in range(n):
            mask |= 1 << int(perm[j])
            if abs(v_all - char[j]) < trunc:
                if not interpolate:
                    char[j + 1] = char[j]
                else:
                    if first:
                        a = (v_all - char[j]) / sum(sizes[j:])
                        first = False
                    char[j + 1] = char[j] + a * sizes[j]
            else:
                char[j + 1] = V[mask]
            rows[k][perm[j]] = char[j + 1] - char[j]
    return rows


@pytest.mark.parametrize("case", MC_CASES, ids=lambda c: f"{c['method']}-n{c['n']}-s{c['seed']}")
def test_truncated_mc_table_matches_reference_goldens(case):
    from mplc.mc import VTable, truncated_mc_table
    table = VTable.from_array(bitmask_table(case))
    np.random.seed(case["seed"])
    sv, std, t = truncated_mc_table(table, sv_accuracy=0.01, alpha=0.95, truncation=0.05,
                                    interpolate=case["method"] == "ITMCS",
                                    sizes=[float(s) for s in case["sizes"]])
    assert same(sv, case["scores"]) and same(std, case["std"])
    assert float(np.random.uniform()) == case["rng_next_uniform"]


@pytest.mark.parametrize("case", MC_CASES, ids=lambda c: f"planned-{c['method']}-n{c['n']}-s{c['seed']}")
def test_device_planned_estimator_changes_nothing(case, monkeypatch):
    import mplc.multi_partner_learning as mpl_mod

    real = mpl_mod.MultiPartnerLearning.device_planning
    assert real is True
    calls = []
    c, calls, err, nxt = run_case(case, monkeypatch, batched=True, device_planning=True)
    assert err is None, err
    assert same(np.atleast_1d(c.contributivity_scores), case["scores"])
    assert same(np.atleast_1d(c.scores_std), case["std"])
    assert c.first_charac_fct_calls_count == case["calls_count"]
    assert [list(k) for k in c.charac_fct_values.keys()] == case["memo_keys"]
    assert nxt == case["rng_next_uniform"]
    assert len(calls) == len(set(calls))
    assert getattr(c, "_vtable", None) is not None  # the device walk planned the waves


@pytest.mark.parametrize("interpolate", [False, True])
@pytest.mark.parametrize("n", [5, 13, 20])
def test_walk_rows_exact_on_random_tables(n, interpolate):
    from mplc.mc import VTable, tmc_walk
    rng = np.random.default_rng(n)
    s = rng.uniform(100, 1000, n)
    masks = np.arange(1 << n)
    acc = np.zeros(1 << n)
    for i in range(n):
        acc += ((masks >> i) & 1) * s[i]
    V = 1 - np.exp(-acc / (s.sum() / 3)) + 1e-3 * rng.uniform(-1, 1, 1 << n)
    V[0] = 0.0
    sizes = [float(int(x)) for x in rng.integers(50, 500, n)]
    perms = np.array([rng.permutation(n) for _ in range(300)])
    v_all = V[-1]
    trunc = 0.05
    rows, status, _ = tmc_walk(VTable.from_array(V), perms, v_all, trunc, interpolate, sizes)
    assert np.all(status == n)
    ref = reference_rows(V, n, perms, v_all, trunc, interpolate, sizes)
    assert np.array_equal(rows, ref)


def test_walk_reports_unknown_frontier_and_wave_frontier_fills_it():
    from mplc.mc import VTable, mask_to_key, tmc_walk, wave_frontier
    n = 8
    rng = np.random.default_rng(3)
    full = rng.uniform(0.1, 0.9, 1 << n)
    full[0] = 0.0
    table = VTable(n)
    table.update({(): 0.0, tuple(range(n)): float(full[-1])})
    perms = np.array([rng.permutation(n) for _ in range(50)])
    _, status, need = tmc_walk(table, perms, full[-1], 0.0, False, None)
    assert np.all(status == 0)  # truncation 0: every walk needs its first singleton
    assert all(mask_to_key(m) == (int(p[0]),) for m, p in zip(need, perms))
    asked = []

    def evaluate(keys):
        asked.extend(keys)
        return [full[sum(1 << i for i in k)] for k in keys]
    rows = wave_frontier(table, perms, full[-1], 0.0, False, None, evaluate)
    assert len(asked) == len(set(asked))
    assert np.array_equal(rows, reference_rows(full, n, perms, full[-1], 0.0, False, None))


def test_moments_match_numpy_over_the_same_walks():
    from mplc.mc import VTable, tmc_moments, tmc_walk
    n = 16
    rng = np.random.default_rng(7)
    V = rng.uniform(0, 1, 1 << n)
    V[0] = 0.0
    table = VTable.from_array(V)
    perms = np.array([rng.permutation(n) for _ in range(5000)])
    rows, _, _ = tmc_walk(table, perms, V[-1], 0.05)
    mean, std, k = tmc_moments(table, len(perms), truncation=0.05, perms=perms)
    assert k == len(perms)
    np.testing.assert_allclose(mean, rows.mean(axis=0), rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(std, rows.std(axis=0), rtol=1e-9, atol=1e-12)
    # device-drawn permutations: a valid estimator (sum of the mean = v(N) for untruncated walks)
    mean2, _, k2 = tmc_moments(table, 20000, truncation=0.0, seed=11)
    assert k2 == 20000 and abs(mean2.sum() - V[-1]) < 1e-9
