"""Coalition encodings.

The reference names coalitions by sorted index tuples (memo key ``tuple(np.sort(subset))``,
mplc/contributivity.py:94-96) and orders the exact-Shapley table by ``itertools.combinations`` size by
size (mplc/contributivity.py:149-151, 1205-1207).  The engine uses bitmasks (bit i <=> partner i).
Lexicographic order of equal-size sorted tuples is DESCENDING order of the bit-reversed mask, so the
combination order of all 2^n - 1 non-empty coalitions is a sort by (popcount asc, reversed mask desc).
"""
import itertools

import numpy as np


def tuple_to_mask(subset):
    m = 0
    for i in subset:
        m |= 1 << int(i)
    return m


def mask_to_tuple(mask):
    out = []
    i = 0
    m = int(mask)
    while m:
        if m & 1:
            out.append(i)
        m >>= 1
        i += 1
    return tuple(out)


def popcount(masks):
    masks = np.asarray(masks, dtype=np.uint64)
    c = np.zeros(masks.shape, dtype=np.int64)
    m = masks.copy()
    while np.any(m):
        c += (m & np.uint64(1)).astype(np.int64)
        m >>= np.uint64(1)
    return c


def _bit_reverse(masks, n):
    masks = np.asarray(masks, dtype=np.uint64)
    r = np.zeros_like(masks)
    for i in range(n):
        r |= ((masks >> np.uint64(i)) & np.uint64(1)) << np.uint64(n - 1 - i)
    return r


def combination_order_masks(n):
    """Masks of all non-empty coalitions in the reference's combination order (int64 array, length 2^n - 1)."""
    if n < 1:
        raise ValueError("n must be >= 1")
    if n <= 12:
        return np.array([tuple_to_mask(c) for r in range(1, n + 1) for c in itertools.combinations(range(n), r)],
                        dtype=np.int64)
    masks = np.arange(1, 1 << n, dtype=np.uint64)
    pc = popcount(masks)
    rev = _bit_reverse(masks, n)
    order = np.lexsort((-rev.astype(np.int64), pc))  # primary popcount asc, secondary reversed desc
    return masks[order].astype(np.int64)


def combination_list_to_bitmask(n, char_func_list):
    """Reference combination-ordered v list (length 2^n - 1) -> bitmask-ordered float64 table (length 2^n, V[0]=0)."""
    v = np.asarray(char_func_list, dtype=np.float64)
    if v.shape != ((1 << n) - 1,):
        raise ValueError(f"expected {(1 << n) - 1} characteristic values for {n} partners, got {v.shape}")
    table = np.zeros(1 << n, dtype=np.float64)
    table[combination_order_masks(n)] = v
    return table


def all_coalitions(n, min_size=1):
    """All coalitions (sorted tuples) in combination order, of size >= min_size."""
    return [c for r in range(max(1, min_size), n + 1) for c in itertools.combinations(range(n), r)]
