"""Fused entity-alignment margin loss (§8f #2, csrc/margin.hip).

Drop-in body of EAModel.get_loss / UEAModel.get_loss (models/models_ea.py:103-123, 169-183):
  loss = (sum relu(A + 1 - B1) + sum relu(A + 1 - B2)) / (2 t k)
with A, B the L1 distances of the gathered pair / negative-pair rows.  The forward never
materialises the (t*k) x D gathers; the backward gathers, per output row, the integer-weighted
sign vectors of the terms that touch it (no atomics: deterministic).
"""
import numpy as np
import torch

from . import _lib
from ._lib import check, ptr, stream_of
from .graph import DeviceCSR


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


_DEV_IDX = {}


def _idx_cached(a, device, n_rows):
    """_idx with the device copy of a host index array cached per array: the reference hands the
    same numpy objects every epoch (data[split][:, 0] views of one array, negatives reassigned
    every 50 epochs, models/models_ea.py:89-91 / run/train_ea.py:61-62), so the copy, the range
    check and the incidence build behind it happen once per negative set, not once per step.
    Keyed by (data pointer, shape, strides, dtype) with the owning array held alive; like the
    CSR cache per adjacency object, an array modified IN PLACE is not noticed (the reference
    never does that)."""
    if not isinstance(a, np.ndarray):
        return _idx(a, device, n_rows)
    owner = a.base if a.base is not None else a
    key = (a.__array_interface__["data"][0], a.shape, a.strides, a.dtype.str, str(device),
           n_rows)
    hit = _DEV_IDX.get(key)
    if hit is not None and hit[0] is owner:
        return hit[1]
    t = _idx(a, device, n_rows)
    if len(_DEV_IDX) >= 48:
        _DEV_IDX.clear()
    _DEV_IDX[key] = (owner, t)
    return t


CHUNK = 256  # incidence entries per backward work item
CODES = True  # sign-code backward for float4 rows (tests flip it to compare with the row gather)


class Incidence:
    """Row -> term-end incidence of the six index tensors and the backward work items."""

    def __init__(self, idx, n_rows):
        left, right, nl1, nr1, nl2, nr2 = idx
        rows = torch.cat([nl1, nl2, left, nr1, nr2, right])
        if rows.numel() >= 2 ** 31:
            raise ValueError("gnnea.margin: too many terms for an int32 incidence")
        dev = rows.device
        cols = torch.arange(rows.numel(), dtype=torch.int64, device=dev)
        self.csr = DeviceCSR.from_coo(rows, cols, None, n_rows, max(1, rows.numel()))
        rp = self.csr.rowptr.long()
        deg = rp[1:] - rp[:-1]
        nch = (deg + CHUNK - 1) // CHUNK
        r = torch.repeat_interleave(torch.arange(n_rows, device=dev), nch)
        first = torch.cumsum(nch, 0) - nch
        c = torch.arange(r.numel(), device=dev) - first[r]
        beg = rp[r] + c * CHUNK
        end = torch.minimum(rp[r + 1], beg + CHUNK)
        multi = nch[r] > 1
        slot = torch.where(multi, torch.cumsum(multi.long(), 0) - 1, torch.full_like(r, -1))
        self.items = torch.stack([r, beg, end, slot], 1).to(torch.int32).contiguous()
        lr = torch.nonzero(nch > 1).flatten()
        self.long_rows = lr.to(torch.int32).contiguous()
        self.long_ptr = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev),
                                   torch.cumsum(nch[lr], 0)]).to(torch.int32).contiguous()
        self.n_slots = int(multi.sum())  # one setup sync per negative set


_INCIDENCE = {}


def incidence(idx, n_rows):
    """Incidence + work items of the six index tensors, cached per tuple of device buffers (data
    pointer, size; the entry holds the tensors alive so a pointer cannot be reused by other
    indices): the negatives change every 50 epochs, the loss runs every one.  Keyed by buffer,
    not by Python object: autograd hands the backward fresh wrappers of its saved tensors."""
    key = tuple((a.data_ptr(), a.numel(), a.dtype) for a in idx) + (n_rows,)
    hit = _INCIDENCE.get(key)
    if hit is not None:
        return hit[1]
    inc = Incidence(idx, n_rows)
    if len(_INCIDENCE) > 8:
        _INCIDENCE.clear()
    _INCIDENCE[key] = (tuple(idx), inc)
    return inc


class MarginLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, outputs, left, right, nl1, nr1, nl2, nr2, t, k):
        _lib.require_device(outputs)
        out = outputs if outputs.stride(-1) == 1 else outputs.contiguous()
        if out.dtype not in (torch.float32, torch.bfloat16):
            raise TypeError("gnnea.margin: outputs must be fp32 or bf16")
        N, D = out.shape
        dev = out.device
        M = 2 * t * k + t
        A = torch.empty(t, dtype=torch.float32, device=dev)
        h = torch.empty(2 * t * k, dtype=torch.float32, device=dev)
        m = torch.empty(M, dtype=torch.float32, device=dev)
        # float4 rows: the forward also stores 2-bit sign codes per column (D/4 bytes per term,
        # 90 MB at t=4500, k=125, D=300) so the backward reads them instead of both rows
        bf = out.dtype == torch.bfloat16
        use_codes = bf or (CODES and D % 4 == 0 and out.stride(0) % 4 == 0 and
                           out.data_ptr() % 16 == 0)
        with _lib.on_device(dev):
            if use_codes:
                sb = D // 4
                codes = torch.empty(M * sb, dtype=torch.uint8, device=dev)
                fn = _lib.lib().gnnea_margin_fwd_code_bf16 if bf else \
                    _lib.lib().gnnea_margin_fwd_code_f32
                check(fn(
                    ptr(out), out.stride(0), D, t, k, ptr(left), ptr(right), ptr(nl1), ptr(nr1),
                    ptr(nl2), ptr(nr2), ptr(A), ptr(h), ptr(m), ptr(codes), sb, stream_of(dev)))
            else:
                codes = None
                check(_lib.lib().gnnea_margin_fwd_f32(
                    ptr(out), out.stride(0), D, t, k, ptr(left), ptr(right), ptr(nl1), ptr(nr1),
                    ptr(nl2), ptr(nr2), ptr(A), ptr(h), ptr(m), stream_of(dev)))
        ctx.save_for_backward(out, left, right, nl1, nr1, nl2, nr2, m, codes)
        ctx.tk = (t, k)
        return torch.sum(h) / (2.0 * t * k)

    @staticmethod
    def backward(ctx, g):
        out, left, right, nl1, nr1, nl2, nr2, m, codes = ctx.saved_tensors
        t, k = ctx.tk
        N, D = out.shape
        inc = incidence((left, right, nl1, nr1, nl2, nr2), N)
        # (bf16 rows: the gradient in bf16, each value rounded once from the fp32 sum)
        grad = torch.zeros((N, D), dtype=out.dtype, device=out.device)
        scratch = torch.empty((max(inc.n_slots, 1), D), dtype=torch.float32, device=out.device)
        g = g.reshape(1).to(torch.float32).contiguous()
        with _lib.on_device(out.device):
            if codes is not None:
                fn = _lib.lib().gnnea_margin_bwd_code_bf16 if out.dtype == torch.bfloat16 else \
                    _lib.lib().gnnea_margin_bwd_code_f32
                check(fn(
                    D, t, k, ptr(m), ptr(codes), D // 4, ptr(inc.csr.col), ptr(inc.items),
                    inc.items.shape[0], ptr(inc.long_rows), ptr(inc.long_ptr),
                    inc.long_rows.numel(), ptr(scratch), ptr(g), 1.0 / (2.0 * t * k), ptr(grad),
                    D, stream_of(out.device)))
                return grad, None, None, None, None, None, None, None, None
            check(_lib.lib().gnnea_margin_bwd_f32(
                ptr(out), out.stride(0), D, t, k, ptr(left), ptr(right), ptr(nl1), ptr(nr1),
                ptr(nl2), ptr(nr2), ptr(m), ptr(inc.csr.col), ptr(inc.items),
                inc.items.shape[0], ptr(inc.long_rows), ptr(inc.long_ptr),
                inc.long_rows.numel(), ptr(scratch), ptr(g), 1.0 / (2.0 * t * k), ptr(grad), D,
                stream_of(out.device)))
        return grad, None, None, None, None, None, None, None, None


def grad_from_multipliers(X, idx, m, t, k, g):
    """d loss / d X of the margin loss for given term multipliers m [2tk + t] (the forward's
    format: negatives of side 1, of side 2, then the pairs), scaled by g / (2tk): the row-gather
    backward kernel (any D; X may be a column block of the embedding, the column-sharded loss of
    gnnea.dist_loss)."""
    left, right, nl1, nr1, nl2, nr2 = idx
    X = X if X.stride(1) == 1 else X.contiguous()
    N, D = X.shape
    inc = incidence(tuple(idx), N)
    grad = torch.zeros((N, D), dtype=torch.float32, device=X.device)
    scratch = torch.empty((max(inc.n_slots, 1), D), dtype=torch.float32, device=X.device)
    g = g.reshape(1).to(device=X.device, dtype=torch.float32).contiguous()
    m = m.to(torch.float32).contiguous()
    with _lib.on_device(X.device):
        check(_lib.lib().gnnea_margin_bwd_f32(
            ptr(X), X.stride(0), D, t, k, ptr(left), ptr(right), ptr(nl1), ptr(nr1), ptr(nl2),
            ptr(nr2), ptr(m), ptr(inc.csr.col), ptr(inc.items), inc.items.shape[0],
            ptr(inc.long_rows), ptr(inc.long_ptr), inc.long_rows.numel(), ptr(scratch), ptr(g),
            1.0 / (2.0 * t * k), ptr(grad), D, stream_of(X.device)))
    return grad


def margin_loss(outputs, left, right, neg_left, neg_right, neg2_left, neg2_right, t, k,
                checked=False):
    """Index arrays may be numpy (int or the reference's float64 np.ones products) or tensors;
    checked=True passes already range-checked int64 device tensors through untouched."""
    if neg_right is None or neg2_left is None:
        raise ValueError("gnnea.margin: negatives are not set (call get_neg first)")
    if t <= 0 or k <= 0:
        raise ValueError("gnnea.margin: need t > 0 pairs and k > 0 negatives")
    arrays = (left, right, neg_left, neg_right, neg2_left, neg2_right)
    if checked:
        idx = list(arrays)
    else:
        idx = [_idx_cached(a, outputs.device, outputs.shape[0]) for a in arrays]
    if idx[0].numel() != t or any(a.numel() != t * k for a in idx[2:]):
        raise ValueError("gnnea.margin: index arrays must have t and t*k entries")
    if outputs.dtype == torch.bfloat16:
        # bf16 models (cfg-5): the sign-code kernels read the bf16 rows and write a bf16
        # gradient (the same values as the fp32 kernels on outputs.float() and a cast back);
        # rows they cannot take (D or the row stride not a multiple of 4, unaligned) go through
        # that copy
        o = outputs if outputs.stride(-1) == 1 else outputs.contiguous()
        D = o.shape[1]
        if not (D % 4 == 0 and o.stride(0) % 4 == 0 and o.data_ptr() % 8 == 0):
            outputs = outputs.float()
    return MarginLossFn.apply(outputs, *idx, t, k)
