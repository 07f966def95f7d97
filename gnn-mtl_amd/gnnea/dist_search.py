"""§8f #1 across GPUs: hard-negative mining and Hits@k over a row-sharded output, without
gathering the embedding to every rank.

The reference mines k negatives per ILL entity every 50 epochs from the full output
(run/train_ea.py:60-62 -> models/models_ea.py:19-30: cdist cityblock + argsort()[1:k+1]) and
ranks the aligned pairs with get_hits (utils/eval_utils.py:71-98).  After a row-sharded encode /
decode (gnnea.dist_graph.DistAdj) rank r holds the global rows [r·rows, (r+1)·rows) of the
output.  Instead of DistAdj.gather_rows (every rank receives 2n x D values, 2.4 GB at cfg-4):

  queries   every rank contributes the query rows it owns (zero rows elsewhere) to ONE all-reduce
            sum: the t query rows on every rank (t·D·4 bytes; a sum with one non-zero term per
            element is exact);
  get_neg   each rank runs the L1 top-(k+1) of every query over its own rows (gnnea.l1.topk:
            fp64 distances equal to scipy's, ordered by (distance, index)); the W per-rank lists
            of (distance, global index) are all-gathered (W·t·(k+1)·16 bytes) and merged by
            (distance, index) — the global top-(k+1) is contained in the union of the per-rank
            top-(k+1) lists, and the ordering is the single-GPU one, so the result is index-exact;
  get_hits  both sides' pair rows by the query all-reduce, the candidate positions split evenly
            over the ranks: each rank counts, per query, the candidates of its block that come
            before the true match in the stable order (gnnea_l1_rank_range_f32), and one
            all-reduce of the integer counts gives every rank the single-GPU ranks;
  eval_at_1 the nearest right entity (top-1 over each rank's block of the right rows, merged).

Every rank must call these (they run collectives); results are replicated.  The engine is the
HIP library; the CPU tests substitute an exact fp64 double (tests/test_dist_search.py).
"""
import numpy as np
import torch
import torch.distributed as dist

from . import l1

INT64_MAX = np.iinfo(np.int64).max


class HipSearchEngine:
    """The product's local search: libgnnea L1 kernels (device tensors)."""

    def topk(self, Q, X, K):
        """(global-order-free) local indices [nq, K] and fp64 distances of the K nearest rows of
        X, ordered by (distance, index)."""
        return l1.topk(Q, X, K, 0, want_dist=True)

    def pairs(self, A, B):
        return l1.pairs(A, B)

    def ranks(self, Q, X, diag, x_off):
        return l1.ranks_range(Q, X, diag, x_off)


def _gloo_dev(t):
    return dist.get_backend() == "gloo" and t.device.type != "cpu"


def _all_reduce(t):
    if _gloo_dev(t):
        h = t.cpu()
        dist.all_reduce(h)
        t.copy_(h)
    else:
        dist.all_reduce(t)
    return t


def _all_gather(t):
    """[W, *t.shape]: every rank's t in rank order."""
    W = dist.get_world_size()
    if dist.get_backend() == "gloo":  # (host-staged for device tensors)
        h = t.cpu().contiguous()
        parts = [torch.empty_like(h) for _ in range(W)]
        dist.all_gather(parts, h)
        return torch.stack(parts).to(t.device)
    out = torch.empty((W,) + tuple(t.shape), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t.contiguous())
    return out


def _ids(ids, device):
    return torch.as_tensor(np.asarray(ids, dtype=np.int64).reshape(-1), device=device)


def gather_query_rows(out_loc, part, ids):
    """[len(ids), D] fp32: the rows ``ids`` (global entity ids) of the sharded output on every
    rank, by one all-reduce of zero-filled rows (each element has exactly one non-zero term)."""
    dev = out_loc.device
    ids = _ids(ids, dev)
    rows = out_loc.shape[0]
    g0 = part.global_row0
    if ids.numel() and (int(ids.min()) < 0 or int(ids.max()) >= part.world * rows):
        raise IndexError("gnnea.dist_search: entity id out of range")
    Q = torch.zeros((ids.numel(), out_loc.shape[1]), dtype=torch.float32, device=dev)
    own = (ids >= g0) & (ids < g0 + rows)
    sel = own.nonzero().reshape(-1)
    if sel.numel():
        Q[sel] = out_loc.detach()[ids[sel] - g0].float()
    return _all_reduce(Q)


def topk_blocks(Q, X, x_off, K, engine=None):
    """The K nearest of a candidate list split over the ranks (this rank holds candidates
    [x_off, x_off + len(X))): global candidate indices [nq, K] in (distance, index) order,
    replicated on every rank, and their fp64 distances."""
    engine = engine or HipSearchEngine()
    nq, dev = Q.shape[0], Q.device
    Kl = min(K, X.shape[0])
    if Kl > 0 and nq:
        idx, dst = engine.topk(Q, X, Kl)
        idx = idx.to(torch.int64) + int(x_off)
        dst = dst.to(torch.float64)
    else:
        idx = torch.empty((nq, 0), dtype=torch.int64, device=dev)
        dst = torch.empty((nq, 0), dtype=torch.float64, device=dev)
    if Kl < K:  # too few candidates here: pad with entries that sort last
        idx = torch.cat([idx, torch.full((nq, K - Kl), INT64_MAX, dtype=torch.int64,
                                         device=dev)], 1)
        dst = torch.cat([dst, torch.full((nq, K - Kl), float("inf"), dtype=torch.float64,
                                         device=dev)], 1)
    ai = _all_gather(idx).permute(1, 0, 2).reshape(nq, -1)
    ad = _all_gather(dst).permute(1, 0, 2).reshape(nq, -1)
    # merge: by index, then stably by distance = (distance, index) order
    o = torch.sort(ai, dim=1, stable=True).indices
    ai, ad = ai.gather(1, o), ad.gather(1, o)
    o = torch.sort(ad, dim=1, stable=True).indices
    return ai.gather(1, o)[:, :K], ad.gather(1, o)[:, :K]


def get_neg(ILL, out_loc, part, k, engine=None):
    """models/models_ea.py:19-30 on a row-sharded output: the k L1-nearest entities of every ILL
    entity, nearest first, the first of the (distance, index) order (the entity itself) dropped;
    flattened t*k int64 numpy, as the single-GPU get_neg returns."""
    Q = gather_query_rows(out_loc, part, ILL)
    idx, _ = topk_blocks(Q, out_loc.detach(), part.global_row0, k + 1, engine)
    if bool((idx[:, 1:] == INT64_MAX).any()):
        raise ValueError("gnnea.dist_search.get_neg: k + 1 > entities")
    return idx[:, 1:].reshape(-1).cpu().numpy()


def _block(n, rank, world):
    return n * rank // world, n * (rank + 1) // world


def hits_ranks(out_loc, part, test_pair, engine=None):
    """(rank_lr, rank_rl) int64 of the aligned pairs (utils/eval_utils.py:71-98 argsort
    positions, ties by index), candidate positions split over the ranks, counts all-reduced."""
    engine = engine or HipSearchEngine()
    pr = np.asarray(test_pair, dtype=np.int64).reshape(-1, 2)
    L = gather_query_rows(out_loc, part, pr[:, 0])
    R = gather_query_rows(out_loc, part, pr[:, 1])
    diag = engine.pairs(L, R)
    j0, j1 = _block(len(pr), part.rank, part.world)
    lr = engine.ranks(L, R[j0:j1], diag, j0).to(torch.int64)
    rl = engine.ranks(R, L[j0:j1], diag, j0).to(torch.int64)
    both = _all_reduce(torch.stack([lr, rl]))
    return both[0], both[1]


def get_hits(out_loc, part, test_pair, top_k=(1, 10, 50, 100), engine=None):
    """utils/eval_utils.py:71-98 on a row-sharded output: Hits@k both ways (percent)."""
    lr, rl = hits_ranks(out_loc, part, test_pair, engine)
    n = len(np.asarray(test_pair).reshape(-1, 2))
    metrics = {}
    for k in top_k:
        metrics["Hits@{}_l".format(k)] = int((lr < k).sum()) / n * 100
    for k in top_k:
        metrics["Hits@{}_r".format(k)] = int((rl < k).sum()) / n * 100
    return metrics


def eval_at_1(out_loc, part, test_pair, engine=None):
    """utils/eval_utils.py:161-167 on a row-sharded output: % of test entities whose L1-nearest
    right entity (first index on ties) is the match."""
    pr = np.asarray(test_pair, dtype=np.int64).reshape(-1, 2)
    L = gather_query_rows(out_loc, part, pr[:, 0])
    R = gather_query_rows(out_loc, part, pr[:, 1])
    j0, j1 = _block(len(pr), part.rank, part.world)
    idx, _ = topk_blocks(L, R[j0:j1], j0, 1, engine)
    hit = (idx[:, 0] == torch.arange(len(pr), device=idx.device)).double()
    return hit.sum() / len(pr) * 100
