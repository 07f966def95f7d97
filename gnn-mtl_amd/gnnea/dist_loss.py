"""Column-sharded EA margin loss over a row-sharded embedding (models/models_ea.py:103-123).

After a row-sharded encode / decode (gnnea.dist_graph.DistAdj) every rank holds its own rows of
the output, ``out_loc`` [rows, D].  The reference loss

    A_i   = |x_left_i - x_right_i|_1,   B_s,ij = |x_nl_s[ik+j] - x_nr_s[ik+j]|_1    (s = 1, 2)
    loss  = (sum relu(A_i + 1 - B_1,ij) + sum relu(A_i + 1 - B_2,ij)) / (2 t k)

reads arbitrary rows of both KGs.  Gathering every row to every rank (DistAdj.gather_rows) moves
2n x D values per rank per step (2.4 GB at cfg-4) and then evaluates the same loss on all ranks.
L1 distances are sums over columns, so here instead:

  1. one all-to-all turns the row shards into column blocks: rank r receives every row of both
     KGs for its columns [c0_r, c1_r) (dist.feature_slices; (W-1)/W of out_loc leaves each rank,
     300 MB at cfg-4 / 8 GPUs);
  2. each rank sums |x_a - x_b| over its columns for all M = 2tk + t terms (gnnea_l1_terms_f32,
     fp64, every term exact) and ONE all-reduce of the M partials gives the distances on every
     rank (9 MB at t = 4500, k = 125);
  3. hinge, loss and the integer multipliers m (the margin kernel's: -[h > 0] per negative, the
     number of active terms per pair) are computed identically everywhere;
  4. backward: the gradient of the rank's column block for every row, sum_j c m_j
     (e_a - e_b) sgn(x_a - x_b) (gnnea_margin_bwd_f32 over the column block), then the reverse
     all-to-all returns each rank its own rows.
The loss is replicated; d loss / d out_loc is this rank's rows, and the parameter gradients are
summed by allreduce_grads as with the gathered loss.  Distances are fp64 sums of exact fp64
terms (the reference's are fp32 sums): hinge decisions agree with the gathered loss except on
ties within fp32 rounding.
"""
import torch
import torch.distributed as dist

from . import _lib
from .dist import feature_slices


def column_blocks(D, world):
    """The column block [c0, c1) of every rank (multiples of 4 wide, the last one possibly not)."""
    return feature_slices(D, world)


def _p2p(sends, recvs):
    """Point-to-point exchange: ``sends`` / ``recvs`` map global peer rank -> tensor.  Under gloo
    device tensors are staged through host memory (the one-device rehearsal and the CPU tests)."""
    gloo = dist.get_backend() == "gloo"
    ops, staged = [], []
    for p, t in sends.items():  # (an empty block moves nothing; both ends agree on its size)
        if t.numel():
            ops.append(dist.P2POp(dist.isend, t.detach().cpu() if gloo and t.is_cuda else t, p))
    for p, t in recvs.items():
        if not t.numel():
            continue
        if gloo and t.is_cuda:
            h = torch.empty(t.shape, dtype=t.dtype)
            staged.append((t, h))
            t = h
        ops.append(dist.P2POp(dist.irecv, t, p))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    for t, h in staged:
        t.copy_(h)


def to_columns(out_loc, part):
    """[rows, D] row shard -> [2n, w] every row of both KGs (global order), this rank's columns."""
    W, me = part.world, part.rank
    D = out_loc.shape[1]
    blocks = column_blocks(D, W)
    c0, c1 = blocks[me]
    rows = out_loc.shape[0]
    X = torch.empty((W * rows, c1 - c0), dtype=out_loc.dtype, device=out_loc.device)
    X[me * rows:(me + 1) * rows].copy_(out_loc[:, c0:c1])
    sends = {p: out_loc[:, blocks[p][0]:blocks[p][1]].contiguous() for p in range(W) if p != me}
    recvs = {p: X[p * rows:(p + 1) * rows] for p in range(W) if p != me}
    _p2p(sends, recvs)
    return X


def from_columns(dX, part, D):
    """Inverse of to_columns for a gradient: [2n, w] (this rank's columns of every row) ->
    [rows, D] (every column of this rank's rows)."""
    W, me = part.world, part.rank
    blocks = column_blocks(D, W)
    rows = dX.shape[0] // W
    out = torch.empty((rows, D), dtype=dX.dtype, device=dX.device)
    c0, c1 = blocks[me]
    out[:, c0:c1].copy_(dX[me * rows:(me + 1) * rows])
    sends = {p: dX[p * rows:(p + 1) * rows].contiguous() for p in range(W) if p != me}
    recvs = {p: torch.empty((rows, blocks[p][1] - blocks[p][0]), dtype=dX.dtype,
                            device=dX.device) for p in range(W) if p != me}
    _p2p(sends, recvs)
    for p, t in recvs.items():
        out[:, blocks[p][0]:blocks[p][1]].copy_(t)
    return out


def _allreduce_sum(t):
    if dist.get_backend() == "gloo" and t.is_cuda:
        h = t.cpu()
        dist.all_reduce(h)
        t.copy_(h)
    else:
        dist.all_reduce(t)
    return t


class HipLossEngine:
    """The product's local compute of the sharded loss: libgnnea kernels (device tensors)."""

    def l1_terms(self, X, a, b):
        """fp64 [n] partial distances sum_{c in X's columns} |X[a_j, c] - X[b_j, c]|."""
        _lib.require_device(X, a, b)
        X = X if X.stride(1) == 1 else X.contiguous()
        out = torch.empty(a.numel(), dtype=torch.float64, device=X.device)
        with _lib.on_device(X.device):
            _lib.check(_lib.lib().gnnea_l1_terms_f32(
                _lib.ptr(X), X.stride(0), X.shape[1], a.numel(), _lib.ptr(a), _lib.ptr(b),
                _lib.ptr(out), _lib.stream_of(X.device)))
        return out

    def margin_grad(self, X, idx, m, t, k, g):
        """d loss / d X for the multipliers m (gnnea_margin_bwd_f32: exact integer sums of the
        sign vectors per row, no atomics), scaled by g / (2tk)."""
        from .margin import grad_from_multipliers
        return grad_from_multipliers(X, idx, m, t, k, g)


class ShardedMarginFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, out_loc, part, engine, left, right, nl1, nr1, nl2, nr2, t, k):
        X = to_columns(out_loc.detach(), part)
        a = torch.cat([nl1, nl2, left])  # term order of the margin kernels: negatives, pairs
        b = torch.cat([nr1, nr2, right])
        d = engine.l1_terms(X, a, b) if X.shape[1] else \
            torch.zeros(a.numel(), dtype=torch.float64, device=X.device)
        d = _allreduce_sum(d)
        tk = t * k
        A = d[2 * tk:]
        Ar = A.repeat_interleave(k)
        h1 = torch.relu(Ar + 1.0 - d[:tk])
        h2 = torch.relu(Ar + 1.0 - d[tk:2 * tk])
        loss = (h1.sum() + h2.sum()) / (2.0 * tk)
        act1, act2 = (h1 > 0).to(torch.float64), (h2 > 0).to(torch.float64)
        n_pair = (act1 + act2).view(t, k).sum(1)
        m = torch.cat([-act1, -act2, n_pair]).to(torch.float32)
        ctx.save_for_backward(X, left, right, nl1, nr1, nl2, nr2, m)
        ctx.part, ctx.engine, ctx.tk, ctx.D = part, engine, (t, k), out_loc.shape[1]
        return loss.to(out_loc.dtype)

    @staticmethod
    def backward(ctx, g):
        X, left, right, nl1, nr1, nl2, nr2, m = ctx.saved_tensors
        t, k = ctx.tk
        dX = ctx.engine.margin_grad(X, (left, right, nl1, nr1, nl2, nr2), m, t, k, g) \
            if X.shape[1] else torch.zeros_like(X)
        return (from_columns(dX, ctx.part, ctx.D),) + (None,) * 10


def sharded_margin_loss(out_loc, dadj, left, right, neg_left, neg_right, neg2_left, neg2_right,
                        t, k, engine=None):
    """EAModel.get_loss over a row-sharded output (the rank's rows of a DistAdj encode /
    decode); index arrays hold global entity ids (numpy or tensors).  Every rank must call it
    (two collectives forward, one backward); returns the replicated loss."""
    from .margin import _idx_cached
    if neg_right is None or neg2_left is None:
        raise ValueError("gnnea.dist_loss: negatives are not set (call get_neg first)")
    if t <= 0 or k <= 0:
        raise ValueError("gnnea.dist_loss: need t > 0 pairs and k > 0 negatives")
    part = dadj.part
    n_all = part.world * out_loc.shape[0]
    idx = [_idx_cached(x, out_loc.device, n_all)
           for x in (left, right, neg_left, neg_right, neg2_left, neg2_right)]
    if idx[0].numel() != t or any(x.numel() != t * k for x in idx[2:]):
        raise ValueError("gnnea.dist_loss: index arrays must have t and t*k entries")
    out = out_loc.float() if out_loc.dtype == torch.bfloat16 else out_loc
    return ShardedMarginFn.apply(out, part, engine or HipLossEngine(), *idx, t, k)
