"""Synthetic two-KG inputs and the vectorised adjacency contract (§8a a1).

``kg_pair_triples`` is the generator every SURVEY/BASELINE number was measured on: per KG of n
entities and t triples (numpy PCG64, seed 0): a ring (i, r, (i+1) mod n) so every entity has a
self loop, then t-n uniform (head, relation, tail) triples; KG2 ids are offset by n, so the
adjacency is block-diagonal across the two KGs (like DBP15K, no cross-KG edges).

``adjacency_coo`` restates utils/data_utils.py:296-336 (get_matrix + get_sparse_tensor) with
numpy instead of a Python dict loop:
  * deg_i = 1 + #(non-self-loop triples touching i)        (multi-edges counted, :297-305)
  * one entry per distinct (h, t) and (t, h), h != t       (dict de-duplication, :307-318)
  * a self loop for every entity that appears in a triple   (:319-320)
  * A_ij = 1/sqrt(deg_i)/sqrt(deg_j) in float64, stored fp32  (:334, :55)
With ``reference_order=True`` the entries come out in the dict's insertion order (bit-identical
to the reference COO, checked in tests/test_adjacency.py); otherwise sorted by (row, col).
"""
import numpy as np


def kg_pair_triples(n, t, n_rel=1000, seed=0):
    """[2t, 3] int64 triples (head, relation, tail) of the synthetic two-KG pair."""
    rng = np.random.default_rng(seed)
    out = []
    for k in range(2):
        ring_r = rng.integers(0, n_rel, n)
        h = rng.integers(0, n, t - n)
        r = rng.integers(0, n_rel, t - n)
        tl = rng.integers(0, n, t - n)
        ring = np.stack([np.arange(n), ring_r, (np.arange(n) + 1) % n], 1)
        rnd = np.stack([h, r, tl], 1)
        out.append(np.concatenate([ring, rnd]) + np.array([k * n, 0, k * n]))
    return np.concatenate(out).astype(np.int64)


def adjacency_coo(triples, n_ent, reference_order=True):
    """(row int64[E], col int64[E], val float32[E]) of the normalised adjacency."""
    tr = np.asarray(triples, dtype=np.int64)
    h, t = tr[:, 0], tr[:, 2]
    ns = h != t
    deg = np.zeros(n_ent, dtype=np.int64)
    appear = np.zeros(n_ent, dtype=bool)
    appear[h] = True
    appear[t] = True
    deg += appear
    deg += np.bincount(h[ns], minlength=n_ent) + np.bincount(t[ns], minlength=n_ent)

    hs, ts = h[ns], t[ns]
    # candidate keys in dict-insertion order: (h,t), (t,h) per non-self triple
    cand = np.empty(2 * hs.size, dtype=np.int64)
    cand[0::2] = hs * n_ent + ts
    cand[1::2] = ts * n_ent + hs
    if reference_order:
        uniq, first = np.unique(cand, return_index=True)
        keys = uniq[np.argsort(first, kind="stable")]
        seq = np.empty(2 * h.size, dtype=np.int64)
        seq[0::2] = h
        seq[1::2] = t
        ents, efirst = np.unique(seq, return_index=True)
        ents = ents[np.argsort(efirst, kind="stable")]
    else:
        keys = np.unique(cand)
        ents = np.nonzero(appear)[0]
    row = np.concatenate([keys // n_ent, ents])
    col = np.concatenate([keys % n_ent, ents])
    if not reference_order:
        order = np.argsort(row * n_ent + col, kind="stable")
        row, col = row[order], col[order]
    d = deg.astype(np.float64)
    val = ((1.0 / np.sqrt(d[row])) / np.sqrt(d[col])).astype(np.float32)
    return row, col, val


def features(n_nodes, dim=300, seed=1):
    """X ~ N(0,1) [n, dim], L2-row-normalised fp32 (get_features, utils/data_utils.py:358)."""
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n_nodes, dim), dtype=np.float32)
    x /= np.maximum(np.linalg.norm(x, axis=1, keepdims=True), 1e-12)
    return x


# configs of BASELINE.json (n entities per KG, t triples per KG, relations)
CONFIGS = {
    "cfg1": dict(n=1000, t=2500, n_rel=1000),
    "dbp15k": dict(n=15000, t=50000, n_rel=1000),
    "cfg4": dict(n=1000000, t=10000000, n_rel=3000),
    "cfg5": dict(n=2000000, t=20000000, n_rel=3000),
}
