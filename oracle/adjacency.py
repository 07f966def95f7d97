"""Adjacency contract restated with explicit loops (small inputs only).

Follows utils/data_utils.py:296-336 (get_matrix / get_sparse_tensor): entity degree = 1 + the
number of non-self-loop triples touching it (multi-edges counted); one entry per distinct ordered
pair in either direction of a non-self-loop triple, in first-insertion order; a self loop per
entity seen in any triple, in first-appearance order; value 1/sqrt(deg_r)/sqrt(deg_c) in fp64,
stored as fp32.
"""
import math

import numpy as np


def adjacency_loops(triples):
    degree = {}
    for h, _, t in triples:
        for v in (h, t):
            if v not in degree:
                degree[v] = 1
        if h != t:
            degree[h] += 1
            degree[t] += 1
    seen = {}
    for h, _, t in triples:
        if h == t:
            continue
        seen.setdefault((h, t), None)
        seen.setdefault((t, h), None)
    for v in degree:
        seen[(v, v)] = None
    rows = np.array([k[0] for k in seen], dtype=np.int64)
    cols = np.array([k[1] for k in seen], dtype=np.int64)
    vals = np.array([1.0 / math.sqrt(degree[r]) / math.sqrt(degree[c]) for r, c in seen],
                    dtype=np.float64).astype(np.float32)
    return rows, cols, vals
