"""CPU: pin the Shapley oracle against the reference's own outputs (tests/golden/shapley_value.json)."""
import itertools
import json
import os

import numpy as np
import pytest

from oracle import shapley as osh
from mplc.coalitions import (combination_list_to_bitmask, combination_order_masks, mask_to_tuple, tuple_to_mask,
                             all_coalitions)

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "shapley_value.json")


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)["data"]


def test_reference_order_restatement_is_bit_exact(golden):
    assert len(golden) >= 20
    for case in golden:
        n = case["n"]
        out = osh.shapley_reference_order(n, case["v_combination_order"])
        assert np.array_equal(out, np.array(case["shapley"])), f"n={n}"


def test_pure_python_restatement_small_n(golden):
    for case in golden:
        if case["n"] <= 6:
            assert osh.reference_shapley_value(case["n"], case["v_combination_order"]) == case["shapley"]


def test_bitmask_long_double_oracle(golden):
    for case in golden:
        n = case["n"]
        V = combination_list_to_bitmask(n, case["v_combination_order"])
        ref = np.array(case["shapley"])
        out = osh.shapley_bitmask_ld(n, V)
        assert np.max(np.abs(out - ref)) <= 1e-13 * np.max(np.abs(ref)), f"n={n}"


def test_combination_order_matches_itertools():
    for n in (1, 2, 5, 12, 13, 14):
        masks = combination_order_masks(n)
        expect = [tuple_to_mask(c) for r in range(1, n + 1) for c in itertools.combinations(range(n), r)]
        assert masks.tolist() == expect
        assert [mask_to_tuple(m) for m in masks[:50]] == all_coalitions(n)[:50]


def test_efficiency_property_large_n():
    # sum_i SV_i = v(N) - v(empty) (efficiency) on the section 8(d) synthetic table
    n = 20
    V = osh.synthetic_table(n)
    sv = osh.shapley_bitmask_ld(n, V)
    assert abs(sv.sum() - V[-1]) < 1e-13
    sv64 = osh.shapley_bitmask_f64_omp(n, V, threads=4)
    assert np.max(np.abs(sv64 - sv)) < 1e-11 * np.max(np.abs(sv))


def test_ranking_fixtures_consistent():
    """tests/golden/ranking_10p*.json (scripts/ranking_fixture.py, two summation orders of the CNN oracle): the stored
    Shapley values are the reference-order restatement of the stored v(S) table, and both passes describe the same
    scenario (tests/test_ranking_gpu.py derives its tie bands from their difference)."""
    import itertools
    import json
    import os
    import numpy as np
    from oracle import shapley as oshap
    golden = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    recs = [json.load(open(os.path.join(golden, f))) for f in ("ranking_10p.json", "ranking_10p_t2.json")]
    assert recs[0]["data_crc32"] == recs[1]["data_crc32"] and recs[0]["scenario"] == recs[1]["scenario"]
    assert [r["threads_per_worker"] for r in recs] == [1, 2]
    n = len(recs[0]["shapley"])
    coals = [c for k in range(1, n + 1) for c in itertools.combinations(range(n), k)]
    for r in recs:
        v = [r["values_bitmask"][sum(1 << p for p in c)] for c in coals]
        assert [float(x) for x in oshap.shapley_reference_order(n, v)] == r["shapley"]
        assert abs(sum(r["shapley"]) - r["values_bitmask"][(1 << n) - 1]) < 1e-12
