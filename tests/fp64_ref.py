"""Whole-graph fp64 torch references ON THE DEVICE for the BASELINE-size tests (test-only).

The CPU oracle (oracle/local.py) checks sampled rows; the weight gradients are sums over every
row of the graph, so they are checked against this fp64 restatement evaluated with plain torch
ops (index_add aggregation in edge chunks, vendor fp64 GEMMs) on the same device.  Formulas:
  GraphConvolution          layers/layers.py:30-39
  HighWayGraphConvolution   layers/layers.py:59-77
  EAModel.get_loss          models/models_ea.py:103-123
ReLU's branch inside the rounding band of 0 follows the tested output (see oracle/local.py).
"""
import torch

CHUNK = 1 << 22
TAU = 1e-5


def agg(r, c, v, n_out, h):
    """sum_e v_e * h[c_e] into row r_e, fp64, edge chunks (no E x D temporary)."""
    out = torch.zeros((n_out, h.shape[1]), dtype=h.dtype, device=h.device)
    for e0 in range(0, r.numel(), CHUNK):
        sl = slice(e0, e0 + CHUNK)
        out.index_add_(0, r[sl], h[c[sl]] * v[sl].unsqueeze(1))
    return out


class Agg(torch.autograd.Function):
    """A·h with backward Aᵀ·g (differentiable chunked aggregation)."""

    @staticmethod
    def forward(ctx, h, r, c, v, n_out):
        ctx.graph = (r, c, v, h.shape[0])
        return agg(r, c, v, n_out, h)

    @staticmethod
    def backward(ctx, g):
        r, c, v, n_in = ctx.graph
        return agg(c, r, v, n_in, g), None, None, None, None


def relu_mask(pre, tested=None):
    """relu'(pre) as a 0/1 fp64 tensor; inside |pre| <= TAU*max|pre| the tested output's sign."""
    band = pre.abs() <= TAU * pre.abs().max().clamp_min(1e-300)
    m = pre > 0
    if tested is not None:
        m = torch.where(band, tested > 0, m)
    return m.to(pre.dtype)


def gcn_grads(r, c, v, x, W, b, R, tested_out):
    """(dW, db) of sum(relu(A(xWᵀ+b)) * R) in fp64."""
    N = x.shape[0]
    pre = agg(r, c, v, N, x @ W.t() + b)
    G = R * relu_mask(pre, tested_out)
    del pre
    P = agg(c, r, v, N, G)
    return P.t() @ x, P.sum(0)


def highway_grads(r, c, v, x, W, b, Kg, R, tested_S):
    """(dW, db) of sum(out * R), out = g*relu(A(xWᵀ+b)) + (1-g)x, g = sigmoid(x Kg)."""
    N = x.shape[0]
    pre = agg(r, c, v, N, x @ W.t() + b)
    m = relu_mask(pre, tested_S)
    del pre
    g = torch.sigmoid(x @ Kg)
    P = agg(c, r, v, N, R * g * m)
    return P.t() @ x, P.sum(0)


def highway_layer(h, W, b, Kg, r, c, v, relu):
    s = Agg.apply(h @ W.t() + b, r, c, v, h.shape[0])
    if relu:
        s = torch.relu(s)
    g = torch.sigmoid(h @ Kg)
    return g * s + (1.0 - g) * h


def margin_loss(out, left, right, neg_left, neg_right, neg2_left, neg2_right, t, k):
    """EAModel.get_loss (models/models_ea.py:103-123)."""
    A = (out[left] - out[right]).abs().sum(1)
    D = A + 1.0
    B1 = (out[neg_left] - out[neg_right]).abs().sum(1)
    L1 = torch.relu(-B1.reshape(t, k) + D.reshape(t, 1))
    B2 = (out[neg2_left] - out[neg2_right]).abs().sum(1)
    L2 = torch.relu(-B2.reshape(t, k) + D.reshape(t, 1))
    return (L1.sum() + L2.sum()) / (2.0 * t * k)
