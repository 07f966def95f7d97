"""Tie-invariant comparison of L1 searches against the reference's (test-only).

The reference ranks with numpy's default argsort (models/models_ea.py:26,
utils/eval_utils.py:78,85), which leaves the order among exactly equal distances unspecified;
the engine (and oracle/l1.py) order ties by index.  What does not depend on the tie order:
  get_neg   the distance of the j-th negative of every query (the sorted distance profile of
            positions 1..k), and the set of negatives strictly between the first position's
            distance (the dropped entry's class) and the k-th's;
  get_hits  each Hits@k lies between the value with every tied candidate ranked after the true
            match and the value with every tied candidate ranked before it.
"""
import numpy as np


def cityblock(A, B):
    A = np.asarray(A, np.float32).astype(np.float64)
    B = np.asarray(B, np.float32).astype(np.float64)
    out = np.zeros((A.shape[0], B.shape[0]))
    for d in range(A.shape[1]):
        out += np.abs(A[:, d:d + 1] - B[None, :, d])
    return out


def check_neg(vec, ILL, got, want, k):
    """Raises AssertionError unless ``got`` and ``want`` (t*k negatives) agree up to tie order.
    Returns the number of queries whose lists differ (tie order only)."""
    S = cityblock(vec[np.asarray(ILL)], vec)
    got, want = np.asarray(got).reshape(-1, k), np.asarray(want).reshape(-1, k)
    differ = 0
    for i in range(len(ILL)):
        dg, dw = S[i, got[i]], S[i, want[i]]
        assert np.array_equal(dg, dw), (i, dg, dw)
        # strictly between the dropped first entry's class (the query's own distance 0, which
        # a duplicate row shares: which of them is dropped is tie order too) and the k-th
        kth, d0 = dw[-1], S[i].min()
        sg, sw = (dg < kth) & (dg > d0), (dw < kth) & (dw > d0)
        assert set(got[i][sg]) == set(want[i][sw]), i
        differ += int(not np.array_equal(got[i], want[i]))
    return differ


def hits_bounds(vec, pairs, top_k=(1, 10, 50, 100)):
    """(optimistic, pessimistic) Hits@k dicts over every tie order."""
    pairs = np.asarray(pairs)
    S = cityblock(vec[pairs[:, 0]], vec[pairs[:, 1]])
    n = len(pairs)
    d = np.diag(S)
    lo_l = (S < d[:, None]).sum(1)                  # rank with the match first among its ties
    hi_l = (S <= d[:, None]).sum(1) - 1             # ... last
    lo_r = (S < d[None, :]).sum(0)
    hi_r = (S <= d[None, :]).sum(0) - 1
    opt, pes = {}, {}
    for side, lo, hi in (("l", lo_l, hi_l), ("r", lo_r, hi_r)):
        for k in top_k:
            opt["Hits@%d_%s" % (k, side)] = int((lo < k).sum()) / n * 100
            pes["Hits@%d_%s" % (k, side)] = int((hi < k).sum()) / n * 100
    return opt, pes


def check_hits(vec, pairs, got, keys, vals):
    """Raises unless the reference's metrics (keys, vals) and ``got`` both lie inside the tie
    bounds; returns {metric: (got, reference)} where they differ."""
    opt, pes = hits_bounds(vec, pairs)
    diff = {}
    for kk, v in zip(keys, vals):
        kk = str(kk)
        assert pes[kk] - 1e-9 <= v <= opt[kk] + 1e-9, (kk, v, pes[kk], opt[kk])
        assert pes[kk] - 1e-9 <= got[kk] <= opt[kk] + 1e-9, (kk, got[kk], pes[kk], opt[kk])
        if abs(got[kk] - v) > 1e-9:
            diff[kk] = (got[kk], float(v))
    return diff
