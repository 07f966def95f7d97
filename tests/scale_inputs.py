"""Deterministic inputs of the BASELINE configs, regenerated from seeds on any machine.

Test infrastructure (tests/golden/gen_golden.py and the -m gpu scale tests share it): the
fixtures under tests/golden/ hold only seeds' outputs, the inputs are rebuilt here bit-for-bit
on the GPU box (numpy PCG64 streams and IEEE elementwise float64 arithmetic only, no BLAS and no
reductions whose order could depend on the machine).

  dbp15k_graph()        the DBP15K-scale pair of SURVEY.md §8d (2 x 15k entities, 2 x 50k triples)
  features(N)           X ~ N(0,1), L2-row-normalised fp32 (gnnea.synth.features)
  upstream(N, D, seed)  the fixed cotangent R of sum(out * R)
  sample_rows(N, k)     sorted row sample the fixtures store outputs for
  ea_pairs / negatives  train pairs (i, i+n) and seeded negatives for EAModel.get_loss
  sinkhorn_cost(B)      M = cdist(X, Y) / max M over 16 dims, fp32 (the reference builds M with
                        torch.cdist over batch embeddings, models/models_ea.py:213-218; a 16-dim
                        elementwise restatement keeps it reproducible to the bit without BLAS)
"""
import numpy as np
import torch

from gnnea import synth

DBP = synth.CONFIGS["dbp15k"]


def dbp15k_graph():
    """(triples, N, row, col, val): reference entry order (utils/data_utils.py:296-336)."""
    n, t = DBP["n"], DBP["t"]
    tr = synth.kg_pair_triples(n, t, DBP["n_rel"], seed=0)
    r, c, v = synth.adjacency_coo(tr, 2 * n, reference_order=True)
    return tr, 2 * n, r, c, v


def features(N, seed=1):
    return synth.features(N, 300, seed=seed)


def upstream(N, D=300, seed=7):
    return np.random.default_rng(seed).standard_normal((N, D), dtype=np.float32)


def sample_rows(N, k=1024, seed=99):
    return np.sort(np.random.default_rng(seed).choice(N, k, replace=False))


def ea_pairs(n, t=4500, seed=21):
    """t train pairs (left entity i of KG1, right entity i + n of KG2), int64 [t, 2]."""
    perm = np.random.default_rng(seed).permutation(n)[:t]
    return np.stack([perm, perm + n], 1).astype(np.int64)


def negatives(N, t, k, seed):
    """[t*k] int64 negative entities (stand-ins for get_neg's L1 nearest neighbours)."""
    return np.random.default_rng(seed).integers(0, N, t * k).astype(np.int64)


def sinkhorn_cost(B, seed=5, dims=16, block=1024):
    """[B, B] fp32 cost normalised to max 1, bit-reproducible: float64 elementwise ops only."""
    rng = np.random.default_rng(seed)
    X = torch.from_numpy(0.05 * rng.standard_normal((B, dims)))
    Y = torch.from_numpy(0.05 * rng.standard_normal((B, dims)))
    M = torch.empty(B, B, dtype=torch.float64)
    for i0 in range(0, B, block):
        xb = X[i0:i0 + block]
        acc = torch.zeros(xb.shape[0], B, dtype=torch.float64)
        for k in range(dims):
            d = xb[:, k:k + 1] - Y[:, k].unsqueeze(0)
            acc.add_(d.mul(d))  # separate multiply and add: no fused contraction
        M[i0:i0 + block] = acc.sqrt_()
    M32 = M.float()
    return M32 / M32.max()
