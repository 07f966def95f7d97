"""Alignment metrics on the device (drop-in for the reference utils/eval_utils.py, §8f #1).

get_hits (utils/eval_utils.py:71-98) builds the full fp64 cityblock matrix with scipy on the host
and argsorts every row and column.  Here the rank of the true match is counted directly on the
device (gnnea_l1_rank_f32: #closer candidates + #equal candidates of lower index), which is the
position of i in a stable argsort of the same fp64 distances; only the counts come back.
Node-classification helpers (acc_f1, nc_metrics, ...) are not on the alignment path and are out
of scope.
"""

import numpy as np
import torch

from gnnea import _lib, l1


def format_metrics(metrics, split):
    """utils/eval_utils.py:7-9"""
    return " ".join("{}_{}: {:.4f}".format(split, name, val) for name, val in metrics.items())


def _on_device(vec):
    vec = vec.detach()
    if not vec.is_cuda:
        # the reference hands CPU tensors here (models/models_ea.py:63-64): upload, then search
        # on the device; without a HIP device require_device raises (there is no CPU path)
        if torch.cuda.is_available():
            vec = vec.to("cuda")
        _lib.require_device(vec)
    return vec


def _pair_index(test_pair, device):
    p = torch.as_tensor(np.asarray(test_pair, dtype=np.int64).reshape(-1, 2), device=device)
    return p[:, 0], p[:, 1]


def _metrics(rank_lr, rank_rl, top_k, n):
    tk = torch.as_tensor(list(top_k), dtype=torch.int64, device=rank_lr.device)
    lr = (rank_lr.long()[None, :] < tk[:, None]).sum(1).tolist()
    rl = (rank_rl.long()[None, :] < tk[:, None]).sum(1).tolist()
    metrics = {}
    for k, c in zip(top_k, lr):
        metrics["Hits@{}_l".format(k)] = c / n * 100
    for k, c in zip(top_k, rl):
        metrics["Hits@{}_r".format(k)] = c / n * 100
    return metrics


def _sharded(vec, adj):
    from gnnea.dist_graph import DistAdj
    return isinstance(adj, DistAdj) and adj.part.world > 1 and vec.shape[0] == adj.part.n_rows


def get_hits(vec, test_pair, top_k=(1, 10, 50, 100), adj=None):
    """utils/eval_utils.py:71-98: Hits@k of the aligned pairs under the L1 distance, both ways.
    ``adj``: the DistAdj of a row-sharded ``vec`` (this rank's rows; every rank calls this):
    the ranks are counted over per-rank candidate blocks and summed (gnnea.dist_search)."""
    if _sharded(vec, adj):
        from gnnea import dist_search
        return dist_search.get_hits(vec, adj.part, test_pair, top_k)
    vec = _on_device(vec)
    li, ri = _pair_index(test_pair, vec.device)
    rank_lr, rank_rl = l1.hits_ranks(vec[li], vec[ri])
    return _metrics(rank_lr, rank_rl, top_k, len(test_pair))


def eval_gw_matching_matrix(T, test_pair, index1_R, index2_R, top_k=(1, 10, 50, 100)):
    """utils/eval_utils.py:133-158: ranks under an ascending argsort of the plan entries
    T[L, R] (the reference's order, kept as is), ties to the lower index."""
    T = _on_device(T)
    L = torch.as_tensor([index1_R[l] for l, r in test_pair], dtype=torch.int64, device=T.device)
    R = torch.as_tensor([index2_R[r] for l, r in test_pair], dtype=torch.int64, device=T.device)
    sim = T[L][:, R]
    n = sim.shape[0]
    ar = torch.arange(n, device=T.device)
    diag = sim[ar, ar]
    lower = ar[None, :] < ar[:, None]  # [i, j]: j < i
    rank_lr = (sim < diag[:, None]).sum(1) + ((sim == diag[:, None]) & lower).sum(1)
    rank_rl = (sim < diag[None, :]).sum(0) + ((sim == diag[None, :]) & lower.t()).sum(0)
    return _metrics(rank_lr, rank_rl, top_k, len(test_pair))


def eval_at_1(outputs, data, adj=None):
    """utils/eval_utils.py:161-167: % of test entities whose L1-nearest right entity is the match
    (argmin of exact fp64 distances, first index on ties).  ``adj``: as get_hits."""
    if _sharded(outputs, adj):
        from gnnea import dist_search
        return dist_search.eval_at_1(outputs, adj.part, data["test"])
    outputs = _on_device(outputs)
    li, ri = _pair_index(data["test"], outputs.device)
    idx, _ = l1.nearest(outputs[li], outputs[ri])
    cnt = (idx == torch.arange(len(li), device=outputs.device)).float()
    return torch.sum(cnt) / len(cnt) * 100
