"""Fused entity-alignment margin loss (§8f #2, csrc/margin.hip).

Drop-in body of EAModel.get_loss / UEAModel.get_loss (models/models_ea.py:103-123, 169-183):
  loss = (sum relu(A + 1 - B1) + sum relu(A + 1 - B2)) / (2 t k)
with A, B the L1 distances of the gathered pair / negative-pair rows.  The forward never
materialises the (t*k) x D gathers; the backward scatters sign vectors into d(outputs).
"""
import numpy as np
import torch

from . import _lib
from ._lib import check, ptr, stream_of


def _idx(a, device, n_rows):
    """int64 device copy; host arrays are range-checked before upload (a bad row index would
    fault the gather kernels), device tensors with one min/max reduction."""
    if torch.is_tensor(a) and a.is_cuda:
        t = a.to(device=device, dtype=torch.int64).contiguous()
        if t.numel():
            lo, hi = torch.aminmax(t)
            if int(lo) < 0 or int(hi) >= n_rows:
                raise IndexError("gnnea.margin: row index out of range [0, %d)" % n_rows)
        return t
    arr = np.asarray(a.cpu() if torch.is_tensor(a) else a).astype(np.int64).reshape(-1)
    if arr.size and (arr.min() < 0 or arr.max() >= n_rows):
        raise IndexError("gnnea.margin: row index out of range [0, %d)" % n_rows)
    return torch.from_numpy(arr).to(device)


class MarginLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, outputs, left, right, nl1, nr1, nl2, nr2, t, k):
        _lib.require_device(outputs)
        out = outputs if outputs.stride(-1) == 1 else outputs.contiguous()
        if out.dtype != torch.float32:
            raise TypeError("gnnea.margin: outputs must be fp32")
        N, D = out.shape
        dev = out.device
        A = torch.empty(t, dtype=torch.float32, device=dev)
        h = torch.empty(2 * t * k, dtype=torch.float32, device=dev)
        with torch.cuda.device(dev):
            check(_lib.lib().gnnea_margin_fwd_f32(
                ptr(out), out.stride(0), D, t, k, ptr(left), ptr(right), ptr(nl1), ptr(nr1),
                ptr(nl2), ptr(nr2), ptr(A), ptr(h), stream_of(dev)))
        ctx.save_for_backward(out, left, right, nl1, nr1, nl2, nr2, h)
        ctx.tk = (t, k)
        return torch.sum(h) / (2.0 * t * k)

    @staticmethod
    def backward(ctx, g):
        out, left, right, nl1, nr1, nl2, nr2, h = ctx.saved_tensors
        t, k = ctx.tk
        N, D = out.shape
        grad = torch.zeros((N, D), dtype=torch.float32, device=out.device)
        g = g.reshape(1).to(torch.float32).contiguous()
        with torch.cuda.device(out.device):
            check(_lib.lib().gnnea_margin_bwd_f32(
                ptr(out), out.stride(0), D, t, k, ptr(left), ptr(right), ptr(nl1), ptr(nr1),
                ptr(nl2), ptr(nr2), ptr(h), ptr(g), 1.0 / (2.0 * t * k), ptr(grad), D,
                stream_of(out.device)))
        return grad, None, None, None, None, None, None, None, None


def margin_loss(outputs, left, right, neg_left, neg_right, neg2_left, neg2_right, t, k,
                checked=False):
    """Index arrays may be numpy (int or the reference's float64 np.ones products) or tensors;
    checked=True passes already range-checked int64 device tensors through untouched."""
    if neg_right is None or neg2_left is None:
        raise ValueError("gnnea.margin: negatives are not set (call get_neg first)")
    arrays = (left, right, neg_left, neg_right, neg2_left, neg2_right)
    if checked:
        idx = list(arrays)
    else:
        idx = [_idx(a, outputs.device, outputs.shape[0]) for a in arrays]
    if idx[0].numel() != t or any(a.numel() != t * k for a in idx[2:]):
        raise ValueError("gnnea.margin: index arrays must have t and t*k entries")
    return MarginLossFn.apply(outputs, *idx, t, k)
