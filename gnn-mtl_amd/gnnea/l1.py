"""Host driver of the L1 (cityblock) distance kernels (§8f #1, csrc/l1.hip).

Replaces the scipy ``cdist(.., metric='cityblock')`` + ``argsort`` searches of
BaseModel.get_neg (models/models_ea.py:19-30), get_hits (utils/eval_utils.py:71-98) and
UEAModel.generate_pairs (models/models_ea.py:143-167).  Distances are fp64 sums of exact terms in
scipy's order, so they equal scipy's bit for bit; orderings break distance ties by the lower index.
"""
import torch

from . import _lib
from ._lib import check, ptr, stream_of

KEY_BUDGET = 1 << 31  # bytes of fp32 distance keys per top-k chunk


def _rows(t):
    _lib.require_device(t)
    if t.dim() != 2:
        raise ValueError("gnnea.l1: expected a 2-D [rows, dim] tensor")
    t = t.detach()
    if t.dtype != torch.float32:
        t = t.float()
    if t.stride(1) != 1:
        t = t.contiguous()
    return t


def pairs(A, B):
    """fp64 L1(A[i], B[i]) for every i (the diagonal of cdist(A, B))."""
    A, B = _rows(A), _rows(B)
    if A.shape != B.shape:
        raise ValueError("gnnea.l1.pairs: shape mismatch %s vs %s" % (A.shape, B.shape))
    n, D = A.shape
    out = torch.empty(n, dtype=torch.float64, device=A.device)
    with _lib.on_device(A.device):
        check(_lib.lib().gnnea_l1_pairs_f32(ptr(A), A.stride(0), ptr(B), B.stride(0), n, D,
                                            ptr(out), stream_of(A.device)))
    return out


def keys(Q, X):
    """[nq, nx] fp32 keys (the fp32 rounding of every L1 distance)."""
    Q, X = _rows(Q), _rows(X)
    nq, D = Q.shape
    nx = X.shape[0]
    if X.shape[1] != D:
        raise ValueError("gnnea.l1.keys: dim mismatch")
    out = torch.empty((nq, nx), dtype=torch.float32, device=Q.device)
    with _lib.on_device(Q.device):
        check(_lib.lib().gnnea_l1_keys_f32(ptr(Q), Q.stride(0), nq, ptr(X), X.stride(0), nx, D,
                                           ptr(out), nx, stream_of(Q.device)))
    return out


def ranks(Q, X, diag):
    """int32 rank of X[q] in the stable distance order of row q (get_hits' rank_index)."""
    Q, X = _rows(Q), _rows(X)
    nq, D = Q.shape
    if nq > X.shape[0] or X.shape[1] != D:
        raise ValueError("gnnea.l1.ranks: need nq <= nx and equal dims")
    diag = diag.to(device=Q.device, dtype=torch.float64).contiguous()
    out = torch.empty(nq, dtype=torch.int32, device=Q.device)
    with _lib.on_device(Q.device):
        check(_lib.lib().gnnea_l1_rank_f32(ptr(Q), Q.stride(0), nq, ptr(X), X.stride(0),
                                           X.shape[0], D, ptr(diag), ptr(out),
                                           stream_of(Q.device)))
    return out


def ranks_range(Q, X, diag, x_off):
    """int32 count, per row q of Q, of the candidates X = [x_off, x_off + len(X)) of a larger
    candidate list that come before candidate q in the stable distance order of row q (the
    row-sharded get_hits sums these over the ranks)."""
    Q = _rows(Q)
    nq, D = Q.shape
    X = _rows(X) if X.shape[0] else X
    if X.shape[0] and X.shape[1] != D:
        raise ValueError("gnnea.l1.ranks_range: dim mismatch")
    diag = diag.to(device=Q.device, dtype=torch.float64).contiguous()
    out = torch.empty(nq, dtype=torch.int32, device=Q.device)
    with _lib.on_device(Q.device):
        check(_lib.lib().gnnea_l1_rank_range_f32(
            ptr(Q), Q.stride(0), nq, ptr(X) if X.shape[0] else None,
            X.stride(0) if X.shape[0] else D, X.shape[0], D, ptr(diag), int(x_off), ptr(out),
            stream_of(Q.device)))
    return out


def hits_ranks(L, R):
    """(rank_lr, rank_rl) of the aligned pairs (L[i], R[i]) in both search directions."""
    diag = pairs(L, R)
    return ranks(L, R, diag), ranks(R, L, diag)


def topk(Q, X, K, skip=0, want_dist=False):
    """The K nearest rows of X (L1) to each row of Q, ordered by (distance, index); columns
    [skip, K) are returned (get_neg: K = k+1, skip = 1 drops the entity itself)."""
    Q, X = _rows(Q), _rows(X)
    nq, D = Q.shape
    nx = X.shape[0]
    if X.shape[1] != D:
        raise ValueError("gnnea.l1.topk: dim mismatch")
    if not 0 <= skip <= K <= nx:
        raise ValueError("gnnea.l1.topk: need 0 <= skip <= K <= rows of X (K=%d, nx=%d)"
                         % (K, nx))
    dev = Q.device
    w = K - skip
    idx = torch.empty((nq, w), dtype=torch.int64, device=dev)
    dist = torch.empty((nq, w), dtype=torch.float64, device=dev) if want_dist else None
    overflow = torch.zeros(1, dtype=torch.int32, device=dev)
    L = _lib.lib()
    chunk = max(1, min(nq, KEY_BUDGET // max(1, 4 * nx)))
    kbuf = torch.empty((min(chunk, nq), nx), dtype=torch.float32, device=dev)
    st = stream_of(dev)
    with _lib.on_device(dev):
        for q0 in range(0, nq, chunk):
            n = min(chunk, nq - q0)
            Qc = Q[q0:q0 + n]
            check(L.gnnea_l1_keys_f32(ptr(Qc), Q.stride(0), n, ptr(X), X.stride(0), nx, D,
                                      ptr(kbuf), nx, st))
            check(L.gnnea_topk_rows_f32(ptr(kbuf), nx, n, nx, K, ptr(Qc), Q.stride(0), ptr(X),
                                        X.stride(0), D, skip, ptr(idx[q0:q0 + n]),
                                        ptr(dist[q0:q0 + n]) if dist is not None else None, w,
                                        ptr(overflow), st))
    topk.last_overflow = overflow
    return (idx, dist) if want_dist else idx


topk.last_overflow = None


def nearest(Q, X):
    """(argmin index, min distance) of every row of Q over the rows of X; first index on ties
    (np.argmin / np.min of cdist)."""
    idx, dist = topk(Q, X, 1, 0, want_dist=True)
    return idx[:, 0], dist[:, 0]
