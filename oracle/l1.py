"""Restatement of the reference's L1 searches (§8f #1) — TEST INFRASTRUCTURE ONLY.

  cityblock   scipy.spatial.distance.cdist(.., 'cityblock'): fp64 sum over d of |u_d - v_d|,
              written out as a plain loop over d (same order, same terms)
  get_neg     models/models_ea.py:19-30     argsort of each row, entries [1, k+1)
  hits        utils/eval_utils.py:71-98     position of i in the argsort of row i / column i
  mutual      models/models_ea.py:143-167   argmin both ways, intersection, bsz best by score
  eval_at_1   utils/eval_utils.py:161-167   argmin of row i == i

Orderings use a stable sort (ties by index); numpy's default argsort leaves tie order
unspecified, so fixtures are built from tie-free inputs.
"""
import numpy as np


def cityblock(A, B):
    A = np.asarray(A, np.float32).astype(np.float64)
    B = np.asarray(B, np.float32).astype(np.float64)
    out = np.zeros((A.shape[0], B.shape[0]))
    for d in range(A.shape[1]):
        out += np.abs(A[:, d:d + 1] - B[None, :, d])
    return out


def get_neg(ILL, vec, k):
    S = cityblock(vec[np.asarray(ILL)], vec)
    return np.argsort(S, axis=1, kind="stable")[:, 1:k + 1].reshape(-1)


def hit_ranks(vec, pairs):
    pairs = np.asarray(pairs)
    S = cityblock(vec[pairs[:, 0]], vec[pairs[:, 1]])
    n = len(pairs)
    lr = np.array([np.where(np.argsort(S[i], kind="stable") == i)[0][0] for i in range(n)])
    rl = np.array([np.where(np.argsort(S[:, i], kind="stable") == i)[0][0] for i in range(n)])
    return lr, rl


def get_hits(vec, pairs, top_k=(1, 10, 50, 100)):
    lr, rl = hit_ranks(vec, pairs)
    n = len(pairs)
    m = {}
    for k in top_k:
        m["Hits@{}_l".format(k)] = int((lr < k).sum()) / n * 100
    for k in top_k:
        m["Hits@{}_r".format(k)] = int((rl < k).sum()) / n * 100
    return m


def mutual_pairs(vec, index1, index2, bsz):
    S = cityblock(vec[np.asarray(index1)], vec[np.asarray(index2)])
    l2r, r2l = S.argmin(1), S.argmin(0)
    vals = S.min(1)
    pairs = [(i, v) for i, v in enumerate(l2r) if r2l[v] == i]
    scores = np.array([vals[i] for i, _ in pairs])
    order = np.argsort(scores, kind="stable")[:bsz]
    return np.array(pairs, dtype=np.int64).reshape(-1, 2)[order]


def eval_at_1(vec, pairs):
    pairs = np.asarray(pairs)
    S = cityblock(vec[pairs[:, 0]], vec[pairs[:, 1]])
    return float((S.argmin(1) == np.arange(len(pairs))).mean() * 100)
