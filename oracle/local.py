"""fp64 oracle of the graph layers on a SAMPLE of rows, computed over their neighbourhoods only
— TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

At the BASELINE sizes (2 x 1M and 2 x 2M entities) a whole-graph fp64 CPU evaluation is out of
reach; a layer's output row i, however, depends only on the input rows of its neighbourhood
N(i) (and on x_i itself for the HighWay gate / residual), and the input gradient of row j only on
the outputs of the rows that aggregate j.  So for a row sample the oracle evaluates:

  outputs   rows S:   inputs U = S ∪ N(S)                              exact for every i in S
  dx        rows T:   outputs S1 = T ∪ dep(T), inputs U1 = S1 ∪ N(S1)  exact for every j in T
            (dep(T) = rows i with A_ij != 0 for some j in T, from the transpose, so no symmetry
             is assumed), loss = sum(out_S1 * R_S1), autograd in fp64.

Layers (same formulas as oracle/gnn.py):
  gcn       layers/layers.py:30-39       act(A · (x W^T + b))
  highway   layers/layers.py:59-77       g*act(A·(xW^T+b)) + (1-g)*x,  g = sigmoid(x Kg + bg)
  gat       layers/att_layers.py:29-61, 82-91   per-head edge softmax of exp(-LReLU(z)), concat

ReLU is a branch: where the fp64 pre-activation is within rounding of 0 (|pre| <= tau·max|pre|)
the fp32 path under test may legitimately take the other side, and the derivative differs by the
full upstream value there.  The oracle therefore takes relu's branch from fp64 everywhere except
in that band, where it follows the sign of the tested output (``gpu_rows``); every other
operation is the oracle's own.
"""
import numpy as np
import scipy.sparse as sp
import torch

TAU = 1e-5
# elements whose relu branch was taken from the tested output (|pre| inside the rounding band),
# and all relu elements evaluated: reported by the BASELINE-size tests
BAND = {"band": 0, "total": 0}


def reset_band():
    BAND["band"] = BAND["total"] = 0


class LocalGraph:
    """Row / column neighbourhoods of a COO adjacency (duplicates summed, like coalesce())."""

    def __init__(self, row, col, val, n):
        self.n = int(n)
        self.A = sp.csr_matrix((np.asarray(val, np.float64), (np.asarray(row, np.int64),
                                                              np.asarray(col, np.int64))),
                               shape=(self.n, self.n))
        self.A.sum_duplicates()
        self.A.sort_indices()
        self.AT = self.A.T.tocsr()
        self.AT.sort_indices()

    def in_nbrs(self, rows):
        return np.unique(self.A[np.asarray(rows)].indices)

    def dependents(self, rows):
        return np.unique(self.AT[np.asarray(rows)].indices)

    def sub(self, out_rows, in_rows):
        """Local COO (row positions in out_rows, column positions in in_rows, values)."""
        blk = self.A[np.asarray(out_rows)].tocoo()
        pos = np.searchsorted(in_rows, blk.col)
        assert np.all(in_rows[pos] == blk.col), "in_rows must cover the neighbourhood"
        return (torch.from_numpy(blk.row.astype(np.int64)), torch.from_numpy(pos.astype(np.int64)),
                torch.from_numpy(blk.data.astype(np.float64)))


def _agg(r, c, v, n_out, h):
    out = torch.zeros((n_out, h.shape[1]), dtype=h.dtype)
    return out.index_add(0, r, h[c] * v.unsqueeze(1))


def _relu_hybrid(pre, gpu_rows, tau=TAU):
    """relu(pre) with the branch inside the rounding band taken from the tested output."""
    with torch.no_grad():
        band = pre.abs() <= tau * pre.abs().max().clamp_min(1e-300)
        mask = pre > 0
        if gpu_rows is not None:
            mask = torch.where(band, torch.as_tensor(gpu_rows).double() > 0, mask)
            BAND["band"] += int(band.sum())
            BAND["total"] += band.numel()
    return pre * mask.to(pre.dtype)


def _act(pre, act, gpu_rows, tau=TAU):
    if act == "relu":
        return _relu_hybrid(pre, gpu_rows, tau)
    if act == "identity":
        return pre
    raise ValueError(act)


def layer_rows(kind, g, x_U, U, S, params, act="relu", gpu_rows=None, alpha=0.2, tau=TAU):
    """Outputs of rows S (sorted, ⊆ U) from the input rows U (sorted) in fp64."""
    r, c, v = g.sub(S, U)
    nS = len(S)
    sp_ = torch.from_numpy(np.searchsorted(U, S))
    if kind == "gcn":
        W, b = params
        return _act(_agg(r, c, v, nS, x_U @ W.t() + b), act, gpu_rows, tau)
    if kind == "highway":
        W, b, Kg, bg = params
        s = _act(_agg(r, c, v, nS, x_U @ W.t() + b), act, gpu_rows, tau)
        xs = x_U[sp_]
        gate = torch.sigmoid(xs @ Kg + (bg if bg is not None else 0.0))
        return gate * s + (1.0 - gate) * xs
    if kind == "gat":
        Ws, As = params  # [H, in, d], [H, 1, 2d]
        outs = []
        d = Ws.shape[2]
        for h_ in range(Ws.shape[0]):
            hU = x_U @ Ws[h_]
            z = hU[sp_][r] @ As[h_, 0, :d] + hU[c] @ As[h_, 0, d:]
            e = torch.exp(-torch.nn.functional.leaky_relu(z, alpha))
            den = torch.zeros(nS, dtype=hU.dtype).index_add(0, r, e)
            num = torch.zeros((nS, d), dtype=hU.dtype).index_add(0, r, e.unsqueeze(1) * hU[c])
            gr = None if gpu_rows is None else np.asarray(gpu_rows)[:, h_ * d:(h_ + 1) * d]
            outs.append(_act(num / den.unsqueeze(1), act, gr, tau))
        return torch.cat(outs, dim=1)
    raise ValueError(kind)


def _t64(a):
    return torch.as_tensor(np.asarray(a)).double()


def sampled_outputs(kind, g, x, S, params, act="relu", gpu_out=None, alpha=0.2, tau=TAU):
    """fp64 outputs of rows S; ``gpu_out(rows)`` returns the tested rows of act(pre) (relu's
    branch band, ``tau`` relative to max|pre|: ~1e-5 for fp32 paths, ~1e-2 for bf16 storage)."""
    S = np.unique(S)
    U = np.union1d(S, g.in_nbrs(S))
    ps = [None if p is None else _t64(p) for p in params]
    with torch.no_grad():
        return S, layer_rows(kind, g, _t64(x[U]), U, S, ps, act,
                             None if gpu_out is None else gpu_out(S), alpha, tau)


def sampled_input_grads(kind, g, x, R, T, params, act="relu", gpu_out=None, alpha=0.2,
                        tau=TAU):
    """fp64 d sum(out * R) / d x on rows T (and d/d params restricted to these outputs is NOT
    the full gradient: only dx is exact here)."""
    T = np.unique(T)
    S1 = np.union1d(T, g.dependents(T))
    U1 = np.union1d(S1, g.in_nbrs(S1))
    ps = [None if p is None else _t64(p) for p in params]
    xU = _t64(x[U1]).requires_grad_(True)
    out = layer_rows(kind, g, xU, U1, S1, ps, act,
                     None if gpu_out is None else gpu_out(S1), alpha, tau)
    (out * _t64(R[S1])[:, :out.shape[1]]).sum().backward()
    return T, xU.grad[torch.from_numpy(np.searchsorted(U1, T))]
