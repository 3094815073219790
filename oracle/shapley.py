"""ORACLE (test infrastructure only) - Python side of the exact-Shapley CPU restatements.

  reference_shapley_value(n, v_comb)  pure-Python restatement of mplc/contributivity.py:1210-1253
                                      (small n only: O(n 4^n) like the reference, list.index and all)
  shapley_reference_order(n, v_comb)  C restatement, same fp64 operation order, O(n 2^n)
  shapley_bitmask_ld(n, V)            long-double single pass over a bitmask table (any n <= 34)
  shapley_bitmask_f64_omp(n, V, thr)  fp64 OpenMP single pass (host CPU baseline)
"""
import bisect
import ctypes
import os
import subprocess
from itertools import combinations
from math import factorial

import numpy as np

_DIR = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_DIR, "liboracle.so")
_lib = None


def build():
    r = subprocess.run(["make", "-s", "-C", _DIR], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"oracle build failed:\n{r.stdout}\n{r.stderr}")
    return _LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        h = ctypes.CDLL(_LIB)
        dp = ctypes.POINTER(ctypes.c_double)
        h.oracle_shapley_reference_order.argtypes = [ctypes.c_int, dp, dp]
        h.oracle_shapley_bitmask_ld.argtypes = [ctypes.c_int, dp, dp]
        h.oracle_shapley_bitmask_f64_omp.argtypes = [ctypes.c_int, dp, dp, ctypes.c_int]
        _lib = h
    return _lib


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def reference_shapley_value(n, v_comb):
    """Line-by-line restatement of mplc/contributivity.py:1218-1253 (power_set :1205-1207)."""
    N = [list(j) for i in range(n) for j in combinations(list(range(n)), i + 1)]
    out = []
    for i in range(n):
        shapley = 0
        for j in N:
            if i not in j:
                cmod = len(j)
                Cui = j[:]
                bisect.insort_left(Cui, i)
                l_ = N.index(j)
                k = N.index(Cui)
                temp = float(float(v_comb[k]) - float(v_comb[l_])) * float(
                    factorial(cmod) * factorial(n - cmod - 1)) / float(factorial(n))
                shapley += temp
        k = N.index([i])
        shapley += float(v_comb[k]) * float(factorial(0) * factorial(n - 1)) / float(factorial(n))
        out.append(shapley)
    return out


def shapley_reference_order(n, v_comb):
    v = np.ascontiguousarray(v_comb, dtype=np.float64)
    out = np.zeros(n)
    if lib().oracle_shapley_reference_order(n, _dp(v), _dp(out)) != 0:
        raise ValueError("unsupported n")
    return out


def shapley_bitmask_ld(n, V):
    V = np.ascontiguousarray(V, dtype=np.float64)
    assert V.shape == (1 << n,)
    out = np.zeros(n)
    if lib().oracle_shapley_bitmask_ld(n, _dp(V), _dp(out)) != 0:
        raise ValueError("unsupported n")
    return out


def shapley_bitmask_f64_omp(n, V, threads=0):
    V = np.ascontiguousarray(V, dtype=np.float64)
    out = np.zeros(n)
    if lib().oracle_shapley_bitmask_f64_omp(n, _dp(V), _dp(out), int(threads)) != 0:
        raise ValueError("unsupported n")
    return out


def synthetic_table(n, seed_s=0, seed_u=1):
    """SURVEY.md section 8(d) synthetic table: s_i ~ U[100,1000] (default_rng(0)),
    V[mask] = 1 - exp(-sum_{i in mask} s_i / (sum s / 4)) + 1e-3 u(mask), u ~ U[-1,1) (default_rng(1)), V[0] = 0."""
    s = np.random.default_rng(seed_s).uniform(100, 1000, size=n)
    V = np.zeros(1 << n, dtype=np.float64)
    # subset sums by doubling
    for i in range(n):
        V[1 << i: 1 << (i + 1)] = V[0: 1 << i] + s[i]
    V = 1.0 - np.exp(-V / (s.sum() / 4.0))
    V += 1e-3 * np.random.default_rng(seed_u).uniform(-1, 1, size=1 << n)
    V[0] = 0.0
    return V
