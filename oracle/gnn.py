"""fp64 torch-CPU restatement of the GNN layers on the hot path.

  gcn_layer      layers/layers.py:30-39   act(A · (x W^T + b))
  highway_layer  layers/layers.py:59-77   g*act(A·(xW^T+b)) + (1-g)*x,  g = sigmoid(x Kg + bg)
  gat_layer      layers/att_layers.py:29-61, 82-91   per-head edge softmax, heads concatenated
  linear         layers/layers.py:92-96
Aggregation is a scatter-add over the COO entries (duplicates summed, like torch.spmm's
coalesce); GAT uses the coalesced (sorted, de-duplicated) edge set like adj.coalesce().
Gradients come from torch autograd on these fp64 graphs.
"""
import numpy as np
import torch


def _t(a):
    return torch.as_tensor(np.asarray(a)).double()


def coo_aggregate(row, col, val, n_rows, h):
    row = torch.as_tensor(row).long()
    col = torch.as_tensor(col).long()
    out = torch.zeros((n_rows, h.shape[1]), dtype=h.dtype)
    return out.index_add_(0, row, h[col] * _t(val).unsqueeze(1))


def linear(x, W, b, act=lambda v: v):
    return act(x @ W.t() + (b if b is not None else 0.0))


def gcn_layer(x, W, b, row, col, val, act=torch.relu):
    return act(coo_aggregate(row, col, val, x.shape[0], x @ W.t() + b))


def highway_layer(x, W, b, Kg, row, col, val, act=torch.relu, bg=None):
    s = act(coo_aggregate(row, col, val, x.shape[0], x @ W.t() + b))
    g = torch.sigmoid(x @ Kg + (bg if bg is not None else 0.0))
    return g * s + (1.0 - g) * x


def coalesced_edges(row, col, n):
    key = np.unique(np.asarray(row, dtype=np.int64) * n + np.asarray(col, dtype=np.int64))
    return torch.as_tensor(key // n), torch.as_tensor(key % n)


def gat_layer(x, Ws, As, row, col, alpha=0.2, act=torch.relu, concat=True):
    """Ws: [H, in, d], As: [H, 1, 2d]."""
    n = x.shape[0]
    r, c = coalesced_edges(row, col, n)
    outs = []
    for W, a in zip(Ws, As):
        h = x @ W
        d = h.shape[1]
        z = h[r] @ a[0, :d] + h[c] @ a[0, d:]
        e = torch.exp(-torch.nn.functional.leaky_relu(z, alpha))
        den = torch.zeros(n, dtype=h.dtype).index_add_(0, r, e)
        num = torch.zeros((n, d), dtype=h.dtype).index_add_(0, r, e.unsqueeze(1) * h[c])
        outs.append(act(num / den.unsqueeze(1)))
    if concat:
        return torch.cat(outs, dim=1)
    return torch.stack(outs, dim=2).mean(dim=2)


def layer_with_grads(fn, x, params, R):
    """(out, dx, [dparams]) of sum(fn(x, *params) * R) in fp64."""
    x = _t(x).requires_grad_(True)
    ps = [_t(p).requires_grad_(True) for p in params]
    out = fn(x, *ps)
    (out * _t(R)[:, :out.shape[1]]).sum().backward()
    return out.detach(), x.grad, [p.grad for p in ps]
