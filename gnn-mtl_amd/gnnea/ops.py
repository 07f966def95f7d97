"""Functional HIP ops and their autograd wrappers (the only callers of the C-ABI).

Every function here launches libgnnea kernels on the tensor's current stream; none has a CPU
path (``_lib.require_device``).  Reference call sites each op replaces are cited per function.
"""
import ctypes
import os
import weakref

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import check, ptr, stream_of
from .graph import DeviceCSR, csr_of

ACT_CODES = {}


def _register_acts():
    ACT_CODES[F.relu] = _lib.GNNEA_ACT_RELU
    ACT_CODES[torch.relu] = _lib.GNNEA_ACT_RELU
    ACT_CODES[F.elu] = _lib.GNNEA_ACT_ELU
    ACT_CODES[F.leaky_relu] = _lib.GNNEA_ACT_LEAKY_RELU
    ACT_CODES[torch.sigmoid] = _lib.GNNEA_ACT_SIGMOID
    ACT_CODES[F.sigmoid] = _lib.GNNEA_ACT_SIGMOID
    ACT_CODES[torch.tanh] = _lib.GNNEA_ACT_TANH
    ACT_CODES[F.tanh] = _lib.GNNEA_ACT_TANH


_register_acts()


def act_code(act):
    """Fusable activation code for a reference ``act`` callable, or None (apply in torch)."""
    try:
        return ACT_CODES.get(act)
    except TypeError:
        return None


def _f32c(t):
    if t.dtype != torch.float32:
        raise TypeError("gnnea: fp32 tensors required (got %s)" % t.dtype)
    return t if t.is_contiguous() else t.contiguous()


FEATURE_DTYPES = (torch.float32, torch.bfloat16)


def _rows(t, dtype=None):
    """Row-major matrix with unit column stride; a column block of a wider row-major buffer
    (row stride > width) is passed through as is (the kernels take a leading dimension)."""
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    if t.dtype not in FEATURE_DTYPES:
        raise TypeError("gnnea: fp32 or bf16 features required (got %s)" % t.dtype)
    if t.dim() == 2 and t.stride(1) == 1 and (t.shape[0] <= 1 or t.stride(0) >= t.shape[1]):
        return t
    return t.contiguous()


def _featc(t, dtype=None):
    """Contiguous feature matrix in fp32 or bf16 storage (converted to ``dtype`` when given)."""
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    if t.dtype not in FEATURE_DTYPES:
        raise TypeError("gnnea: fp32 or bf16 features required (got %s)" % t.dtype)
    return t if t.is_contiguous() else t.contiguous()


# ------------------------------------------------------------------------------------------ #
# dense projection (MFMA)                                                                     #
# ------------------------------------------------------------------------------------------ #
_WS = {}


def _gemm_ws(device, nbytes):
    key = (device, )
    buf = _WS.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
        _WS[key] = buf
    return buf


_WSQ = {}


def _ws_query(fn, M, N, K):
    """Workspace size of a GEMM shape (a pure function of the shape: cached, it runs per call)."""
    key = (fn.__name__, M, N, K)
    v = _WSQ.get(key)
    if v is None:
        if len(_WSQ) > 256:
            _WSQ.clear()
        v = _WSQ[key] = int(fn(M, N, K))
    return v


_SMALL_OPERAND = 1 << 22
# fp32 products at least this large (M*N*K) run on the bf16 MFMA with three-way split operands
# (gnnea_gemm_x3_f32: fp32-level rounding, 6/16 of the f32 MFMA time); smaller ones on the f32
# MFMA (gnnea_gemm_f32).  GEMM_X3 = False keeps every fp32 product on the f32 MFMA.
GEMM_X3 = True
X3_MIN_MNK = 1 << 26


X3_MIN_M = 4096  # tall A only (DBP15K scale, 30k rows: x3 55 us vs f32 MFMA 75 us, measured)


def _use_x3(M, N, K, x3, trans_a=False, trans_b=False):
    """x3 splits op(B) into bf16 planes once per call: for a small B (the weight) times a tall,
    K-contiguous A.  The weight gradients dW = Aᵀ·B (trans_a, both operands tall, a small M x N
    output) split both operands on the fly instead (gnnea_gemm_x3_f32's trans_a form, B
    untransposed).  The bias column sums (B = the tall gradient) stay on the f32 MFMA."""
    if trans_a:
        if trans_b or M * N > _SMALL_OPERAND:
            return False
        if x3 is not None:
            return bool(x3)
        return GEMM_X3 and K >= X3_MIN_M and M * N * K >= X3_MIN_MNK
    if N * K > _SMALL_OPERAND:
        return False
    if x3 is not None:
        return bool(x3)
    return GEMM_X3 and M >= X3_MIN_M and M * N * K >= X3_MIN_MNK


def _ld(t):
    """Row stride of a row-major matrix; a single row's stride is meaningless (torch reports 1
    for a transposed column vector), its width is the valid leading dimension."""
    return t.stride(0) if t.shape[0] > 1 else max(t.shape[1], 1)


def gemm(a, b, trans_a=False, trans_b=False, bias=None, out=None, beta=0.0, out_dtype=None,
         x3=None, sliced_out=None, act=None):
    """out = op(a) @ op(b) (+ bias) (+ beta*out) on MFMA.

    fp32 operands: gnnea_gemm_f32 (exact-f32 MFMA), or for large products gnnea_gemm_x3_f32
    (three-way bf16 splits, fp32-level rounding; ``x3`` forces either).  A bf16 operand (cfg-5
    storage) switches to gnnea_gemm_bf16 (both operands bf16, fp32 accumulate, out bf16 unless
    an fp32 ``out`` / ``out_dtype`` is given).  ``act`` (a GNNEA_ACT_* code; beta = 0, no
    sliced_out): out = act(op(a) @ op(b) + bias) -- gnnea_gemm_x3_act_f32 / gnnea_gemm_bf16_act,
    relu in the weight-resident kernels' epilogue; after gnnea_gemm_f32 the act runs in place
    (gnnea_act_fwd_f32)."""
    _lib.require_device(a, b)
    if act == _lib.GNNEA_ACT_IDENTITY:
        act = None
    if act is not None and (beta != 0.0 or sliced_out is not None):
        raise ValueError("gnnea.gemm: act needs beta = 0 and no sliced_out")
    bf = a.dtype == torch.bfloat16 or b.dtype == torch.bfloat16
    if bf:
        a = _featc(a, torch.bfloat16)
        b = _featc(b, torch.bfloat16)
        # the bf16 kernel stages K-contiguous operands with one 16-B LDS store per chunk and
        # transposes the others element by element: hand it a small weight pre-transposed
        # (W is <= a few MB; dY.W in the Linear backward, x.W in GAT / HighWay)
        if not trans_b and b.numel() <= _SMALL_OPERAND:
            b, trans_b = b.t().contiguous(), True
        if trans_a and a.numel() <= _SMALL_OPERAND:
            a, trans_a = a.t().contiguous(), False
    else:
        if a.dtype != torch.float32 or b.dtype != torch.float32:
            raise TypeError("gnnea: fp32 tensors required (got %s, %s)" % (a.dtype, b.dtype))
        a = _rows(a)
        b = _rows(b)
    M = a.shape[1] if trans_a else a.shape[0]
    K = a.shape[0] if trans_a else a.shape[1]
    Kb = b.shape[1] if trans_b else b.shape[0]
    N = b.shape[0] if trans_b else b.shape[1]
    if K != Kb:
        raise ValueError("gnnea.gemm: inner dimensions differ (%d vs %d)" % (K, Kb))
    if out is None:
        dt = out_dtype or (torch.bfloat16 if bf else torch.float32)
        out = torch.empty((M, N), dtype=dt, device=a.device)
        beta = 0.0
    if out.dtype not in FEATURE_DTYPES or (not bf and out.dtype != torch.float32):
        raise TypeError("gnnea.gemm: out must be fp32 (or bf16 with bf16 operands)")
    if bias is not None:
        bias = _featc(bias, torch.float32)
    L = _lib.lib()
    x3 = not bf and _use_x3(M, N, K, x3, trans_a, trans_b)
    ws_fn = L.gnnea_gemm_bf16_ws_bytes if bf else (
        (L.gnnea_gemm_x3t_ws_bytes if trans_a else L.gnnea_gemm_x3_ws_bytes) if x3
        else L.gnnea_gemm_ws_bytes)
    ws_bytes = _ws_query(ws_fn, M, N, K)
    ws = _gemm_ws(a.device, ws_bytes) if ws_bytes > 0 else None
    with _lib.on_device(a.device):
        if bf and act is not None:
            cd = _lib.GNNEA_BF16 if out.dtype == torch.bfloat16 else _lib.GNNEA_F32
            check(L.gnnea_gemm_bf16_act(int(trans_a), int(trans_b), M, N, K, ptr(a), _ld(a),
                                        ptr(b), _ld(b), ptr(bias), int(act), ptr(out), _ld(out),
                                        cd, ptr(ws), ws_bytes if ws is not None else 0,
                                        stream_of(a.device)))
        elif act is not None and x3:
            check(L.gnnea_gemm_x3_act_f32(int(trans_a), int(trans_b), M, N, K, ptr(a), _ld(a),
                                          ptr(b), _ld(b), ptr(bias), int(act), ptr(out),
                                          _ld(out), ptr(ws), ws_bytes if ws is not None else 0,
                                          stream_of(a.device)))
        elif bf:
            cd = _lib.GNNEA_BF16 if out.dtype == torch.bfloat16 else _lib.GNNEA_F32
            check(L.gnnea_gemm_bf16(int(trans_a), int(trans_b), M, N, K, ptr(a), _ld(a),
                                    ptr(b), _ld(b), ptr(bias), float(beta), ptr(out),
                                    _ld(out), cd, ptr(ws),
                                    ws_bytes if ws is not None else 0, stream_of(a.device)))
        elif sliced_out is not None and x3 and not trans_a:
            # row-major out AND the slice-major copy from one GEMM epilogue
            check(L.gnnea_gemm_x3_dual_f32(int(trans_a), int(trans_b), M, N, K, ptr(a), _ld(a),
                                           ptr(b), _ld(b), ptr(bias), float(beta), ptr(out),
                                           _ld(out), ptr(sliced_out), sliced_out.stride(0),
                                           ptr(ws), ws_bytes if ws is not None else 0,
                                           stream_of(a.device)))
        else:
            fn = L.gnnea_gemm_x3_f32 if x3 else L.gnnea_gemm_f32
            check(fn(int(trans_a), int(trans_b), M, N, K, ptr(a), _ld(a), ptr(b), _ld(b),
                     ptr(bias), float(beta), ptr(out), _ld(out), ptr(ws),
                     ws_bytes if ws is not None else 0, stream_of(a.device)))
            if act is not None:  # the exact-f32 kernel has no act epilogue
                if not out.is_contiguous():
                    raise ValueError("gnnea.gemm: act needs a contiguous out on this path")
                check(L.gnnea_act_fwd_f32(ptr(out), ptr(out), out.numel(), int(act),
                                          stream_of(a.device)))
            if sliced_out is not None:
                check(L.gnnea_slice_pack_f32(ptr(out), _ld(out), M, N, ptr(sliced_out),
                                             sliced_out.stride(0), stream_of(a.device)))
    return out


def _rows64(t):
    if t.dim() == 2 and t.stride(1) == 1 and (t.shape[0] <= 1 or t.stride(0) >= t.shape[1]):
        return t
    return t.contiguous()


def gemm_f64(a, b, trans_a=False, trans_b=False, alpha=1.0, e=None, beta=0.0, out=None):
    """out = alpha * op(a) @ op(b) + beta * e, fp64 on the f64 matrix cores (gnnea_gemm_f64; the
    GW / FGW products of SinkhornOT/cderivation.py).  ``e`` may be ``out``."""
    _lib.require_device(a, b)
    if a.dtype != torch.float64 or b.dtype != torch.float64:
        raise TypeError("gnnea.gemm_f64: fp64 tensors required (got %s, %s)" % (a.dtype, b.dtype))
    a = _rows64(a)
    b = _rows64(b)
    M = a.shape[1] if trans_a else a.shape[0]
    K = a.shape[0] if trans_a else a.shape[1]
    Kb = b.shape[1] if trans_b else b.shape[0]
    N = b.shape[0] if trans_b else b.shape[1]
    if K != Kb:
        raise ValueError("gnnea.gemm_f64: inner dimensions differ (%d vs %d)" % (K, Kb))
    if out is None:
        out = torch.empty((M, N), dtype=torch.float64, device=a.device)
    if out.shape != (M, N) or out.dtype != torch.float64 or out.stride(1) != 1:
        raise ValueError("gnnea.gemm_f64: out must be a row-major fp64 [M, N] tensor")
    if e is not None:
        if e.shape != (M, N) or e.dtype != torch.float64:
            raise ValueError("gnnea.gemm_f64: e must be fp64 [M, N]")
        e = _rows64(e)
    L = _lib.lib()
    with _lib.on_device(a.device):
        check(L.gnnea_gemm_f64(int(trans_a), int(trans_b), M, N, K, ptr(a), _ld(a), ptr(b),
                               _ld(b), float(alpha), ptr(e), _ld(e) if e is not None else 0,
                               float(beta), ptr(out), _ld(out), stream_of(a.device)))
    return out


class LinearFn(torch.autograd.Function):
    """y = x W^T + b  (nn.Linear.forward at layers/layers.py:32,61,93) on MFMA."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        ctx.bias_dtype = bias.dtype if bias is not None else None
        return gemm(x, weight, trans_b=True, bias=bias)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        bf = x.dtype == torch.bfloat16 or weight.dtype == torch.bfloat16
        dy = _featc(dy, torch.bfloat16 if bf else torch.float32)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = gemm(dy, weight, out_dtype=x.dtype if bf else None)  # [N,out]·[out,in]
        want_w, want_b = ctx.needs_input_grad[1], ctx.has_bias and ctx.needs_input_grad[2]
        if want_w and want_b:  # dW and db from one pass over dY
            r = gemm_ta_db(dy, x, weight.dtype if bf else None)
            if r is not None:
                dw, db = r[0], r[1].to(ctx.bias_dtype)
                want_w = want_b = False
        if want_w:
            dw = gemm(dy, x, trans_a=True, out_dtype=weight.dtype if bf else None)  # [out,N]·[N,in]
        if want_b:
            db = colsum(dy, ctx.bias_dtype)
        return dx, dw, db


class LinearActFn(torch.autograd.Function):
    """y = act(x Wᵀ + b)  (Linear.forward at layers/layers.py:121-122 with dropout inactive; the
    MLPDecoder's relu layers, models/decoders.py:57-63): the act in the GEMM's epilogue, and in
    the backward the act's derivative and the bias gradient in one pass over dY and y."""

    @staticmethod
    def forward(ctx, x, weight, bias, act):
        y = gemm(x, weight, trans_b=True, bias=bias, act=act)
        ctx.save_for_backward(x, weight, y)
        ctx.act = act
        ctx.has_bias = bias is not None
        ctx.bias_dtype = bias.dtype if bias is not None else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, y = ctx.saved_tensors
        bf = x.dtype == torch.bfloat16 or weight.dtype == torch.bfloat16
        dy = _featc(dy, y.dtype)
        want_db = ctx.has_bias and ctx.needs_input_grad[2]
        g, db = act_bwd_colsum(dy, y, ctx.act, want_db)
        g = _featc(g, torch.bfloat16 if bf else torch.float32)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = gemm(g, weight, out_dtype=x.dtype if bf else None)
        if ctx.needs_input_grad[1]:
            dw = gemm(g, x, trans_a=True, out_dtype=weight.dtype if bf else None)
        if db is not None and db.dtype != ctx.bias_dtype:
            db = db.to(ctx.bias_dtype)
        return dx, dw, db, None


# slice-major copies of GEMM outputs written by the GEMM itself (gnnea_gemm_x3_dual_f32), keyed
# by the row-major output's storage: the GAT forward finds the projection's sliced table here
# instead of packing it (a stale entry is ignored: the tensor's version must match)
_SLICED_COPIES = {}


def sliced_copy_of(t, D):
    """The slice-major copy of ``t`` written by its projection GEMM, or None; the entry is
    removed (it is used once, by the layer's forward, and would otherwise keep an H-sized table
    alive through the backward)."""
    e = _SLICED_COPIES.pop(t.data_ptr(), None)
    if e is None:
        return None
    ref, ver, shape, xs = e
    src = ref()
    if src is None or src._version != ver or tuple(src.shape) != tuple(t.shape) or \
            t.shape[1] < D or t.stride(1) != 1:
        return None
    return xs


class MatmulFn(torch.autograd.Function):
    """y = x W  (torch.mm(input, self.W) at layers/att_layers.py:33, torch.spmm(x, kernel_gate)
    at layers/layers.py:69) on MFMA.  ``sliced``: also write y slice-major from the same GEMM
    epilogue when the aggregation that follows uses the sliced table (GAT above the Infinity
    Cache), registered for sliced_copy_of."""

    @staticmethod
    def forward(ctx, x, w, sliced=False):
        ctx.save_for_backward(x, w)
        M, N = x.shape[0], w.shape[1]
        if sliced and x.dtype == torch.float32 and w.dtype == torch.float32 and N % 4 == 0 \
                and use_sliced(M, N, torch.float32):
            xs = sliced_empty(M, N, x.device, torch.float32)
            y = gemm(x, w, sliced_out=xs)
            _SLICED_COPIES.clear()  # one live copy: the layer's projection
            _SLICED_COPIES[y.data_ptr()] = (weakref.ref(y), y._version, tuple(y.shape), xs)
            return y
        return gemm(x, w)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        bf = x.dtype == torch.bfloat16 or w.dtype == torch.bfloat16
        dy = _featc(dy, torch.bfloat16 if bf else torch.float32)
        dx = gemm(dy, w, trans_b=True, out_dtype=x.dtype if bf else None) \
            if ctx.needs_input_grad[0] else None
        dw = gemm(x, dy, trans_a=True, out_dtype=w.dtype if bf else None) \
            if ctx.needs_input_grad[1] else None
        return dx, dw, None


class HeadMeanFn(torch.autograd.Function):
    """y = x.view(-1, heads, dh).mean(dim=1) (the non-concatenated GAT layer, att_layers.py:89-91)
    in one pass each way (gnnea_head_mean_*)."""

    @staticmethod
    def forward(ctx, x, heads, dh):
        x = _rows(x)
        n = x.shape[0]
        y = torch.empty((n, dh), dtype=x.dtype, device=x.device)
        with _lib.on_device(x.device):
            check(_sfn("gnnea_head_mean", x.dtype)(ptr(x), _ld(x), n, heads, dh, ptr(y), _ld(y), 0,
                                                   stream_of(x.device)))
        ctx.meta = (heads, dh, x.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        heads, dh, dt = ctx.meta
        dy = _rows(dy, dt)
        n = dy.shape[0]
        dx = torch.empty((n, heads * dh), dtype=dt, device=dy.device)
        with _lib.on_device(dy.device):
            check(_sfn("gnnea_head_mean", dt)(ptr(dy), _ld(dy), n, heads, dh, ptr(dx), _ld(dx), 1,
                                              stream_of(dy.device)))
        return dx, None, None


def head_mean(x, heads, dh):
    """Mean over the heads of a head-concatenated [N, heads*dh] matrix (fp32 / bf16 on HIP)."""
    _lib.require_device(x)
    if x.dim() != 2 or x.shape[1] != heads * dh:
        raise ValueError("gnnea.head_mean: x must be [N, heads*dh]")
    return HeadMeanFn.apply(x, heads, dh)


def linear(x, weight, bias=None, act=None):
    """x Wᵀ + b, or act(x Wᵀ + b) for a GNNEA_ACT_* code ``act`` (the act fused into the GEMM)."""
    if act is None or act == _lib.GNNEA_ACT_IDENTITY:
        return LinearFn.apply(x, weight, bias)
    return LinearActFn.apply(x, weight, bias, int(act))


def act_bwd_colsum(dy, y, act, want_db=True):
    """(G, db): G = dy * act'(y) (y = the act's output) and db = column sums of G, one pass
    (gnnea_act_bwd_colsum_*; db fp32, None when not wanted -- then gnnea_act_bwd alone)."""
    if not want_db:
        return act_bwd(dy, y, act), None
    y = _rows(y)
    dy = _rows(dy, y.dtype)
    n, D = y.shape
    L = _lib.lib()
    g = torch.empty_like(y)
    db = torch.empty(D, dtype=torch.float32, device=y.device)
    ws_bytes = int(L.gnnea_act_bwd_colsum_ws_bytes(n, D))
    ws = _gemm_ws(y.device, ws_bytes)
    fn = L.gnnea_act_bwd_colsum_bf16 if y.dtype == torch.bfloat16 else \
        L.gnnea_act_bwd_colsum_f32
    with _lib.on_device(y.device):
        check(fn(ptr(dy), _ld(dy), ptr(y), _ld(y), n, D, int(act), ptr(g), _ld(g), ptr(db),
                 ptr(ws), ws_bytes, stream_of(y.device)))
    return g, db


def gemm_ta_db(a, b, out_dtype=None):
    """(aᵀ·b, column sums of a) in one pass over a (gnnea_gemm_x3_ta_db_f32 / gnnea_gemm_bf16_ta_db:
    a layer's dW = dhᵀ·x and db = colsum(dh), db fp32; dW bit-identical to gemm(a, b,
    trans_a=True, out_dtype=out_dtype)), or None where that kernel is not the one gemm would run
    (then: gemm + colsum)."""
    bf = a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16
    if not bf and (a.dtype != torch.float32 or b.dtype != torch.float32):
        return None
    a, b = _rows(a), _rows(b)
    K, M = a.shape
    N = b.shape[1]
    if b.shape[0] != K:
        raise ValueError("gnnea.gemm_ta_db: shape mismatch")
    L = _lib.lib()
    al = 8 if bf else 16
    if bf:
        ok = L.gnnea_gemm_bf16_ta_db_applies(M, N, K, _ld(a), _ld(b))
    else:
        ok = _use_x3(M, N, K, None, trans_a=True) and \
            L.gnnea_gemm_x3_ta_db_applies(M, N, K, _ld(a), _ld(b))
    if not ok or a.data_ptr() % al or b.data_ptr() % al:
        return None
    odt = (out_dtype or torch.bfloat16) if bf else torch.float32
    out = torch.empty((M, N), dtype=odt, device=a.device)
    db = torch.empty(M, dtype=torch.float32, device=a.device)
    ws_bytes = int(L.gnnea_gemm_x3_ta_db_ws_bytes(M, N, K))
    ws = _gemm_ws(a.device, ws_bytes)
    with _lib.on_device(a.device):
        if bf:
            cd = _lib.GNNEA_BF16 if odt == torch.bfloat16 else _lib.GNNEA_F32
            check(L.gnnea_gemm_bf16_ta_db(M, N, K, ptr(a), _ld(a), ptr(b), _ld(b), ptr(out), N, cd,
                                          ptr(db), ptr(ws), ws_bytes, stream_of(a.device)))
        else:
            check(L.gnnea_gemm_x3_ta_db_f32(M, N, K, ptr(a), _ld(a), ptr(b), _ld(b), ptr(out), N,
                                            ptr(db), ptr(ws), ws_bytes, stream_of(a.device)))
    return out, db


def _wgrads(dh, x, need_w, need_b):
    """(dW, db) of a layer h = x Wᵀ + b from dh: one pass when both are wanted (gemm_ta_db)."""
    if need_w and need_b:
        r = gemm_ta_db(dh, x)
        if r is not None:
            return r
    return (gemm(dh, x, trans_a=True) if need_w else None), (colsum(dh) if need_b else None)


def _f32_mask_ok(M, N, K, lda, ldc, *ts):
    return (_use_x3(M, N, K, None) and all(t.data_ptr() % 16 == 0 for t in ts)
            and bool(_lib.lib().gnnea_gemm_f32_mask_applies(M, N, K, lda, ldc)))


def gemm_relu_mask(x, weight, bias):
    """(relu(x Wᵀ + b), sign bits) in one pass (gnnea_gemm_{bf16,f32}_relu_mask: the output
    bit-identical to gemm(..., act=relu), plus 1 bit per element for gemm_dmask), or None where
    the weight-resident kernel that gemm would run does not apply."""
    if x.dtype == torch.float32 and weight.dtype == torch.float32:
        x, weight = _rows(x), _rows(weight)
        M, K = x.shape
        N = weight.shape[0]
        if weight.shape[1] != K:
            raise ValueError("gnnea.gemm_relu_mask: shape mismatch")
        if not _f32_mask_ok(M, N, K, _ld(x), N, x):
            return None
        L = _lib.lib()
        y = torch.empty((M, N), dtype=torch.float32, device=x.device)
        ldm = int(L.gnnea_gemm_f32_mask_ld(N))
        mask = torch.empty((M, ldm), dtype=torch.uint8, device=x.device)
        b = _featc(bias, torch.float32) if bias is not None else None
        ws_bytes = int(L.gnnea_gemm_f32_mask_ws_bytes(N))
        ws = _gemm_ws(x.device, ws_bytes)
        with _lib.on_device(x.device):
            check(L.gnnea_gemm_f32_relu_mask(1, M, N, K, ptr(x), _ld(x), ptr(weight), _ld(weight),
                                             ptr(b), ptr(y), N, ptr(mask), ldm, ptr(ws), ws_bytes,
                                             stream_of(x.device)))
        return y, mask
    if x.dtype != torch.bfloat16 or weight.dtype != torch.bfloat16:
        return None
    x, weight = _rows(x), _rows(weight)
    M, K = x.shape
    N = weight.shape[0]
    if weight.shape[1] != K:
        raise ValueError("gnnea.gemm_relu_mask: shape mismatch")
    L = _lib.lib()
    if not L.gnnea_gemm_bf16_dmask_applies(M, N, K, _ld(x), N, N) or \
            (x.data_ptr() | weight.data_ptr()) % 8:
        return None
    y = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    ldm = int(L.gnnea_gemm_bf16_mask_ld(N))
    mask = torch.empty((M, ldm), dtype=torch.uint8, device=x.device)
    b = _featc(bias, torch.float32) if bias is not None else None
    ws_bytes = int(L.gnnea_gemm_bf16_dmask_ws_bytes(N, K))
    ws = _gemm_ws(x.device, ws_bytes)
    with _lib.on_device(x.device):
        check(L.gnnea_gemm_bf16_relu_mask(1, M, N, K, ptr(x), _ld(x), ptr(weight), _ld(weight),
                                          ptr(b), ptr(y), N, ptr(mask), ldm, ptr(ws), ws_bytes,
                                          stream_of(x.device)))
    return y, mask


def gemm_dmask(g, weight, y, mask=None):
    """bf16(g · weight) * relu'(y) in one pass (gnnea_gemm_bf16_dmask: the product that carries the
    gradient into a relu Linear's output y, masked in its epilogue -- bit-identical to gemm
    followed by act_bwd's G; with ``mask``, gemm_relu_mask's sign bits of y, read instead of y:
    gnnea_gemm_bf16_dmask_bits), or None where that kernel does not apply (then the caller runs
    the two steps).  fp32: from the sign bits only (gnnea_gemm_f32_dmask_bits)."""
    if g.dtype == torch.float32 and weight.dtype == torch.float32 and y.dtype == torch.float32:
        if mask is None:
            return None
        g, weight = _rows(g), _rows(weight)
        M, K = g.shape
        N = weight.shape[1]
        if weight.shape[0] != K or y.shape != (M, N):
            raise ValueError("gnnea.gemm_dmask: shape mismatch")
        if not _f32_mask_ok(M, N, K, _ld(g), N, g, mask):
            return None
        L = _lib.lib()
        out = torch.empty((M, N), dtype=torch.float32, device=g.device)
        ws_bytes = int(L.gnnea_gemm_f32_mask_ws_bytes(N))
        ws = _gemm_ws(g.device, ws_bytes)
        with _lib.on_device(g.device):
            check(L.gnnea_gemm_f32_dmask_bits(0, M, N, K, ptr(g), _ld(g), ptr(weight), _ld(weight),
                                              ptr(mask), mask.stride(0), ptr(out), N, ptr(ws),
                                              ws_bytes, stream_of(g.device)))
        return out
    if g.dtype != torch.bfloat16 or weight.dtype != torch.bfloat16 or y.dtype != torch.bfloat16:
        return None
    g, weight, y = _rows(g), _rows(weight), _rows(y)
    M, K = g.shape
    N = weight.shape[1]
    if weight.shape[0] != K or y.shape != (M, N):
        raise ValueError("gnnea.gemm_dmask: shape mismatch")
    L = _lib.lib()
    out = torch.empty((M, N), dtype=torch.bfloat16, device=g.device)
    if not L.gnnea_gemm_bf16_dmask_applies(M, N, K, _ld(g), _ld(y), _ld(out)) or \
            (g.data_ptr() | y.data_ptr() | weight.data_ptr()) % 8:
        return None
    ws_bytes = int(L.gnnea_gemm_bf16_dmask_ws_bytes(N, K))
    ws = _gemm_ws(g.device, ws_bytes)
    with _lib.on_device(g.device):
        if mask is not None:
            check(L.gnnea_gemm_bf16_dmask_bits(0, M, N, K, ptr(g), _ld(g), ptr(weight),
                                               _ld(weight), ptr(mask), mask.stride(0), ptr(out),
                                               _ld(out), ptr(ws), ws_bytes, stream_of(g.device)))
        else:
            check(L.gnnea_gemm_bf16_dmask(0, M, N, K, ptr(g), _ld(g), ptr(weight), _ld(weight),
                                          ptr(y), _ld(y), ptr(out), _ld(out), ptr(ws), ws_bytes,
                                          stream_of(g.device)))
    return out


class MLPChainFn(torch.autograd.Function):
    """A stack of Linear layers y_{k+1} = act_k(y_k W_kᵀ + b_k), act_k relu or identity, dropout
    inactive (the MLPDecoder, models/decoders.py, each layer as layers/layers.py:121-122) as ONE
    autograd node, so that the backward can fuse across layers: the product carrying the gradient
    into a relu layer's output y_k masks it in its epilogue (gemm_dmask, reading the sign bits
    the forward product wrote with y_k, gemm_relu_mask), which removes the act_bwd pass over
    (dy_k, y_k) of the per-layer LinearActFn; db_k is a column sum of the masked gradient (fp32:
    from the weight-gradient product itself, gemm_ta_db).  Forward and every stored value as
    LinearFn / LinearActFn compute them (same GEMM calls); the bias gradients sum the same values
    in another order."""

    @staticmethod
    def forward(ctx, x, acts, *params):
        ys, masks = [x], []
        for k, act in enumerate(acts):
            w, b = params[2 * k], params[2 * k + 1]
            a = act if act == _lib.GNNEA_ACT_RELU else None
            ym = gemm_relu_mask(ys[-1], w, b) if a is not None and k + 1 < len(acts) and \
                any(ctx.needs_input_grad) else None  # (the sign bits only for a backward)
            ys.append(ym[0] if ym is not None else gemm(ys[-1], w, trans_b=True, bias=b, act=a))
            masks.append(ym[1] if ym is not None else None)
        ctx.acts = tuple(acts)
        ctx.bias_dtypes = [params[2 * k + 1].dtype if params[2 * k + 1] is not None else None
                           for k in range(len(acts))]
        ws = [params[2 * k] for k in range(len(acts))]
        ctx.save_for_backward(*ys[:-1], ys[-1], *ws, *masks)
        return ys[-1]

    @staticmethod
    def backward(ctx, dy):
        nl = len(ctx.acts)
        saved = ctx.saved_tensors
        ys, ws, masks = list(saved[:nl + 1]), list(saved[nl + 1:2 * nl + 1]), saved[2 * nl + 1:]
        need = ctx.needs_input_grad
        grads = [None] * (2 * nl)
        g = None     # the gradient at the current layer's pre-activation (masked), when known
        d = dy       # else the gradient at its output
        dx = None
        for k in range(nl - 1, -1, -1):
            x, w, y, act = ys[k], ws[k], ys[k + 1], ctx.acts[k]
            bf = x.dtype == torch.bfloat16 or w.dtype == torch.bfloat16
            want_db = ctx.bias_dtypes[k] is not None and need[3 + 2 * k]
            db, pend = None, want_db  # (pend: db still to form from g)
            if g is None:
                if act == _lib.GNNEA_ACT_RELU:
                    d = _featc(d, y.dtype)
                    g, db = act_bwd_colsum(d, y, act, want_db)
                    pend = False
                else:
                    g = _featc(d, torch.bfloat16 if bf else torch.float32)
            g = _featc(g, torch.bfloat16 if bf else torch.float32)
            need_w = need[2 + 2 * k]
            if pend and need_w:
                r = gemm_ta_db(g, x, w.dtype if bf else None)
                if r is not None:
                    (grads[2 * k], db), need_w, pend = r, False, False
            if need_w:
                grads[2 * k] = gemm(g, x, trans_a=True, out_dtype=w.dtype if bf else None)
            if pend:
                db = colsum(g, ctx.bias_dtypes[k])
            if db is not None and db.dtype != ctx.bias_dtypes[k]:
                db = db.to(ctx.bias_dtypes[k])
            grads[2 * k + 1] = db
            if k == 0 and not need[0]:
                break
            # the gradient into x = y_{k-1}: masked here when that layer is a relu layer
            gn = None
            if k > 0 and ctx.acts[k - 1] == _lib.GNNEA_ACT_RELU:
                gn = gemm_dmask(g, w, x, masks[k - 1])
            if gn is not None:
                g, d = gn, None
            else:
                d = gemm(g, w, out_dtype=x.dtype if bf else None)
                g = None
            if k == 0:
                dx = d
        return (dx, None, *grads)


def mlp_chain(x, layers):
    """The fused MLPChainFn over an nn.Sequential of layers.layers.Linear, or None when a layer
    is not fusable (an act other than relu / identity, active dropout, no weight) or carries
    forward hooks (they see the per-layer modules' calls, which the chain does not make)."""
    acts, params = [], []
    for m in [layers] + list(layers):
        if m._forward_hooks or m._forward_pre_hooks:
            return None
    for m in layers:
        code = act_code(getattr(m, "act", None))
        lin = getattr(m, "linear", None)
        if code not in (_lib.GNNEA_ACT_RELU, _lib.GNNEA_ACT_IDENTITY) or lin is None or \
                (m.training and m.dropout > 0):
            return None
        acts.append(int(code))
        params += [lin.weight, lin.bias]
    if not acts:
        return None
    return MLPChainFn.apply(x, tuple(acts), *params)


def matmul(x, w, sliced=False):
    return MatmulFn.apply(x, w, sliced)


# ------------------------------------------------------------------------------------------ #
# CSR aggregation                                                                              #
# ------------------------------------------------------------------------------------------ #
INFINITY_CACHE_BYTES = 256 << 20


def _off(t, r0, c0=0):
    """Device pointer of element (r0, c0) of a row-major tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr() + t.element_size() * (r0 * t.stride(0) + c0))


def _off32(t, r0):
    """Device pointer of element r0 of a 1-D 4-byte tensor (CSR rowptr)."""
    return ctypes.c_void_p(t.data_ptr() + 4 * r0)


def _blocks(csr, x):
    """Row blocks to launch one after another: the diagonal blocks when the gathered matrix is
    larger than the Infinity Cache (a single launch keeps all blocks' gathers in flight)."""
    if x.shape[0] * x.shape[1] * x.element_size() <= INFINITY_CACHE_BYTES:
        return [(0, csr.n_rows)]
    return csr.row_blocks()


def spmm(csr, x, act=_lib.GNNEA_ACT_IDENTITY, out=None, beta=0.0, out_dtype=None):
    """out = act(A @ x + beta*out) with the gather-model CSR kernel.

    fp32 x: gnnea_spmm_csr_{,beta_}f32.  bf16 x (cfg-5 storage): gnnea_spmm_csr_bf16 with fp32
    arithmetic and a bf16 (default) or fp32 ``out``.  Other dtypes are computed as fp32."""
    _lib.require_device(x)
    if x.dtype not in FEATURE_DTYPES or x.stride(1) != 1:
        x = x.float().contiguous() if x.dtype not in FEATURE_DTYPES else x.contiguous()
    if x.dim() != 2 or x.shape[0] < csr.n_cols:
        raise ValueError("gnnea.spmm: x must be [%d, D]" % csr.n_cols)
    if out is None:
        out = torch.empty((csr.n_rows, x.shape[1]), dtype=out_dtype or x.dtype, device=x.device)
        beta = 0.0
    if x.dtype == torch.float32 and out.dtype != torch.float32:
        raise TypeError("gnnea.spmm: fp32 x needs an fp32 out")
    if out.dtype not in FEATURE_DTYPES:
        raise TypeError("gnnea.spmm: out must be fp32 or bf16")
    L = _lib.lib()
    st = stream_of(x.device)
    with _lib.on_device(x.device):
        for r0, r1 in _blocks(csr, x):
            rp = ctypes.c_void_p(csr.rowptr.data_ptr() + 4 * r0)
            if x.dtype == torch.bfloat16:
                yd = _lib.GNNEA_BF16 if out.dtype == torch.bfloat16 else _lib.GNNEA_F32
                check(L.gnnea_spmm_csr_bf16(rp, ptr(csr.col), ptr(csr.val), r1 - r0, x.shape[1],
                                            ptr(x), x.stride(0), float(beta), _off(out, r0),
                                            out.stride(0), yd, int(act), st))
            elif beta == 0.0:
                check(L.gnnea_spmm_csr_f32(rp, ptr(csr.col), ptr(csr.val), r1 - r0, x.shape[1],
                                           ptr(x), x.stride(0), _off(out, r0), out.stride(0),
                                           int(act), st))
            else:
                check(L.gnnea_spmm_csr_beta_f32(rp, ptr(csr.col), ptr(csr.val), r1 - r0,
                                                x.shape[1], ptr(x), x.stride(0), float(beta),
                                                _off(out, r0), out.stride(0), int(act), st))
    return out


def act_bwd(dy, y, act):
    y = _featc(y)
    dy = _featc(dy, y.dtype)
    g = torch.empty_like(y)
    fn = _lib.lib().gnnea_act_bwd_bf16 if y.dtype == torch.bfloat16 else \
        _lib.lib().gnnea_act_bwd_f32
    with _lib.on_device(y.device):
        check(fn(ptr(dy), ptr(y), ptr(g), y.numel(), int(act), stream_of(y.device)))
    return g


# ------------------------------------------------------------------------------------------ #
# slice-major feature tables (gnnea_spmm_sliced_*)                                            #
# ------------------------------------------------------------------------------------------ #
SLICE_BYTES = 256  # one slice row: 64 fp32 / 128 bf16 columns
SLICE_W = SLICE_BYTES // 4
SLICED = True  # use the slice-major path where it applies (tests switch it off to compare)


def slice_w(dtype):
    return SLICE_BYTES // torch.empty((), dtype=dtype).element_size()


def use_sliced(n_src, D, dtype):
    """The slice-major aggregation applies to fp32 / bf16 tables at least two slices wide whose
    row-major form exceeds the Infinity Cache (cfg-4: 1M rows x 300 per KG): one 256-B slice of
    a 1M-row KG is 256 MB and its gathers are 256-B line pairs.  Measured on one KG of cfg-4
    (profiles/r01_scale_probe_sliced.json): 300 fp32 columns 4.28 -> 3.46 ms, 152 columns
    1.85 -> 1.79 ms, 76 columns 1.08 -> 1.11 ms (row-major kept below two slices)."""
    if not SLICED or dtype not in FEATURE_DTYPES or D % 4:
        return False
    es = 4 if dtype == torch.float32 else 2
    return D * es >= 2 * SLICE_BYTES and n_src * D * es > INFINITY_CACHE_BYTES


def sliced_empty(n, D, device, dtype=torch.float32, W=None):
    """Uninitialised [S, n, W] table for an [n, D] matrix (W = 256 B of ``dtype`` by default,
    64 columns for the GAT tables; S = ceil(D/W)); columns past D in the last slice are never
    read."""
    W = W or slice_w(dtype)
    S = (D + W - 1) // W
    return torch.empty((S, n, W), dtype=dtype, device=device)


def _sfn(name, dtype):
    return getattr(_lib.lib(), name + ("_bf16" if dtype == torch.bfloat16 else "_f32"))


def slice_pack(x):
    """Row-major [n, D] (fp32 / bf16) -> slice-major table (gnnea_slice_pack_*)."""
    x = _rows(x)
    n, D = x.shape
    xs = sliced_empty(n, D, x.device, x.dtype)
    with _lib.on_device(x.device):
        check(_sfn("gnnea_slice_pack", x.dtype)(ptr(x), _ld(x), n, D, ptr(xs), xs.stride(0),
                                               stream_of(x.device)))
    return xs


def act_bwd_sliced(dy, y, act):
    """Gs = dy * act'(y) written slice-major (the transposed aggregation's input)."""
    y = _rows(y)
    dy = _rows(dy, y.dtype)
    n, D = y.shape
    gs = sliced_empty(n, D, y.device, y.dtype)
    with _lib.on_device(y.device):
        check(_sfn("gnnea_act_bwd_sliced", y.dtype)(ptr(dy), _ld(dy), ptr(y), _ld(y), n, D,
                                                    int(act), ptr(gs), gs.stride(0),
                                                    stream_of(y.device)))
    return gs


def spmm_sliced(csr, xs, D, act=_lib.GNNEA_ACT_IDENTITY, out=None, out_dtype=None):
    """out = act(A @ X) with X held slice-major in ``xs`` ([S, n_src, W], fp32 or bf16),
    launched per diagonal (KG) block; out row-major [n_rows, D] (xs's dtype by default; an
    fp32 out for a bf16 table keeps the sums unrounded)."""
    _lib.require_device(xs)
    if xs.dtype not in FEATURE_DTYPES:
        raise TypeError("gnnea.spmm_sliced: fp32 or bf16 table required")
    W = slice_w(xs.dtype)
    S = (D + W - 1) // W
    if xs.dim() != 3 or xs.shape[0] < S or xs.shape[2] != W or xs.shape[1] < csr.n_cols or \
            not xs.is_contiguous():
        raise ValueError("gnnea.spmm_sliced: xs must be a contiguous [%d, >=%d, %d] table"
                         % (S, csr.n_cols, W))
    if out is None:
        out = torch.empty((csr.n_rows, D), dtype=out_dtype or xs.dtype, device=xs.device)
    if out.shape != (csr.n_rows, D) or out.stride(1) != 1 or out.dtype not in FEATURE_DTYPES \
            or (xs.dtype == torch.float32 and out.dtype != torch.float32):
        raise ValueError("gnnea.spmm_sliced: out must be [%d, %d] (fp32 for an fp32 table)"
                         % (csr.n_rows, D))
    L = _lib.lib()
    st = stream_of(xs.device)
    with _lib.on_device(xs.device):
        for r0, r1 in csr.row_blocks():
            if xs.dtype == torch.bfloat16:
                yd = _lib.GNNEA_BF16 if out.dtype == torch.bfloat16 else _lib.GNNEA_F32
                check(L.gnnea_spmm_sliced_bf16(_off32(csr.rowptr, r0), ptr(csr.col),
                                               ptr(csr.val), r1 - r0, D, ptr(xs), xs.stride(0),
                                               _off(out, r0), _ld(out), yd, int(act), st))
            else:
                check(L.gnnea_spmm_sliced_f32(_off32(csr.rowptr, r0), ptr(csr.col),
                                              ptr(csr.val), r1 - r0, D, ptr(xs), xs.stride(0),
                                              _off(out, r0), _ld(out), int(act), st))
    return out


def spmm_sliced_m(csr, xs, D):
    """(relu(A @ X), sign bits of it) for an fp32 slice-major X (gnnea_spmm_sliced_m_f32): the
    bits [n_rows, D / 4] bytes replace the output in the backward (act_bwd_sliced_bits)."""
    out = torch.empty((csr.n_rows, D), dtype=torch.float32, device=xs.device)
    ldm = (D + 3) // 4
    mask = torch.empty((csr.n_rows, ldm), dtype=torch.uint8, device=xs.device)
    if xs.dtype != torch.float32 or xs.dim() != 3 or xs.shape[2] != slice_w(xs.dtype) or \
            xs.shape[1] < csr.n_cols or not xs.is_contiguous():
        raise ValueError("gnnea.spmm_sliced_m: a contiguous fp32 slice table required")
    L = _lib.lib()
    with _lib.on_device(xs.device):
        for r0, r1 in csr.row_blocks():
            check(L.gnnea_spmm_sliced_m_f32(_off32(csr.rowptr, r0), ptr(csr.col), ptr(csr.val),
                                            r1 - r0, D, ptr(xs), xs.stride(0), _off(out, r0),
                                            _ld(out), ctypes.c_void_p(mask.data_ptr() + r0 * ldm),
                                            ldm, stream_of(xs.device)))
    return out, mask


def act_bwd_sliced_bits(dy, mask, D):
    """Gs = dy * relu'(y) slice-major with relu' from spmm_sliced_m's sign bits."""
    dy = _rows(dy, torch.float32)
    n = dy.shape[0]
    gs = sliced_empty(n, D, dy.device, torch.float32)
    with _lib.on_device(dy.device):
        check(_lib.lib().gnnea_act_bwd_sliced_bits_f32(ptr(dy), _ld(dy), ptr(mask), mask.stride(0),
                                                       n, D, ptr(gs), gs.stride(0),
                                                       stream_of(dy.device)))
    return gs


def spmm_sliced64(csr, xs, D, act=_lib.GNNEA_ACT_IDENTITY, out=None, out_dtype=None):
    """out = act(A @ X) for a bf16 X held in 64-column slices ([S, n_src, 64]: 128 B per row
    piece, one cfg-5 KG slice = 256 MB; slice_pack64's layout), per diagonal (KG) block."""
    _lib.require_device(xs)
    if xs.dtype != torch.bfloat16:
        raise TypeError("gnnea.spmm_sliced64: bf16 table required")
    S = (D + 63) // 64
    if xs.dim() != 3 or xs.shape[0] < S or xs.shape[2] != 64 or xs.shape[1] < csr.n_cols or \
            not xs.is_contiguous():
        raise ValueError("gnnea.spmm_sliced64: xs must be a contiguous [%d, >=%d, 64] table"
                         % (S, csr.n_cols))
    if out is None:
        out = torch.empty((csr.n_rows, D), dtype=out_dtype or xs.dtype, device=xs.device)
    if out.shape != (csr.n_rows, D) or out.stride(1) != 1 or out.dtype not in FEATURE_DTYPES:
        raise ValueError("gnnea.spmm_sliced64: out must be [%d, %d]" % (csr.n_rows, D))
    L = _lib.lib()
    st = stream_of(xs.device)
    yd = _lib.GNNEA_BF16 if out.dtype == torch.bfloat16 else _lib.GNNEA_F32
    with _lib.on_device(xs.device):
        for r0, r1 in csr.row_blocks():
            check(L.gnnea_spmm_sliced64_bf16(_off32(csr.rowptr, r0), ptr(csr.col), ptr(csr.val),
                                             r1 - r0, D, ptr(xs), xs.stride(0), _off(out, r0),
                                             _ld(out), yd, int(act), st))
    return out


def gemm_sliced(x, weight, bias=None):
    """hidden = x W^T + b written slice-major (gnnea_gemm_sliced_{f32,bf16}): the projection of
    a GCN layer hands the aggregation its table at no extra pass.  bf16 operands give a bf16
    table (fp32 accumulate)."""
    bf = x.dtype == torch.bfloat16 or weight.dtype == torch.bfloat16
    dt = torch.bfloat16 if bf else torch.float32
    x = _rows(x, dt)
    weight = _featc(weight, dt) if bf else _rows(weight, dt)
    M, K = x.shape
    N = weight.shape[0]
    if weight.shape[1] != K:
        raise ValueError("gnnea.gemm_sliced: inner dimensions differ")
    hs = sliced_empty(M, N, x.device, dt)
    if bias is not None:
        bias = _featc(bias, torch.float32)
    L = _lib.lib()
    x3 = not bf and _use_x3(M, N, K, None)
    ws_fn = L.gnnea_gemm_bf16_ws_bytes if bf else (
        L.gnnea_gemm_x3_ws_bytes if x3 else L.gnnea_gemm_ws_bytes)
    ws_bytes = _ws_query(ws_fn, M, N, K)
    ws = _gemm_ws(x.device, ws_bytes) if ws_bytes > 0 else None
    fn = L.gnnea_gemm_sliced_bf16 if bf else (
        L.gnnea_gemm_x3_sliced_f32 if x3 else L.gnnea_gemm_sliced_f32)
    with _lib.on_device(x.device):
        check(fn(0, 1, M, N, K, ptr(x), _ld(x), ptr(weight), _ld(weight), ptr(bias), 0.0,
                 ptr(hs), hs.stride(0), ptr(ws), ws_bytes if ws is not None else 0,
                 stream_of(x.device)))
    return hs


def aggregate_t_into(csr, dy, y, act, out=None):
    """out = Aᵀ·(dy ⊙ act'(y)): the backward of act(A·hidden), slice-major when it applies."""
    csrT = csr.transpose()
    D = y.shape[1]
    if use_sliced(csrT.n_cols, D, y.dtype) and \
            (out is None or y.dtype == torch.bfloat16 or out.dtype == torch.float32):
        gs = act_bwd_sliced(dy, y, act)
        return spmm_sliced(csrT, gs, D, out=out)
    g = _featc(dy, y.dtype) if act == _lib.GNNEA_ACT_IDENTITY else act_bwd(dy, y, act)
    return spmm(csrT, g, out=out)


class AggregateFn(torch.autograd.Function):
    """support = act(A · hidden) (layers/layers.py:34-38); backward A^T · (dY ⊙ act'(Y)).
    Above the Infinity Cache (fp32) the aggregation runs over a slice-major copy of hidden
    (gnnea_slice_pack_f32 + gnnea_spmm_sliced_f32) and the backward writes dY ⊙ act'(Y)
    slice-major in the same elementwise pass."""

    @staticmethod
    def forward(ctx, hidden, csr, act):
        if use_sliced(csr.n_cols, hidden.shape[1], hidden.dtype):
            out = spmm_sliced(csr, slice_pack(hidden), hidden.shape[1], act)
        else:
            out = spmm(csr, hidden, act)
        ctx.csr = csr
        ctx.act = act
        ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, dy):
        (out,) = ctx.saved_tensors
        return aggregate_t_into(ctx.csr, dy, out, ctx.act), None, None


class GCNLayerFn(torch.autograd.Function):
    """A whole graph convolution act(A · (x Wᵀ + b)) (layers/layers.py:30-39, dropout inactive)
    with the hidden kept slice-major: the projection GEMM writes it as the sliced aggregation
    reads it (never row-major in HBM); backward dY ⊙ act'(Y) is written slice-major by one
    elementwise pass (fp32 relu: act' from the sign bits the forward wrote instead of Y),
    Aᵀ·G gives d hidden row-major for dx = dh·W, dW = dhᵀ·x, db = colsum(dh)."""

    @staticmethod
    def forward(ctx, x, weight, bias, csr, act):
        hs = gemm_sliced(x, weight, bias)
        D = weight.shape[0]
        # fp32 relu with a sliced backward: the output's sign bits are what the backward keeps
        ctx.bits = int(act) == _lib.GNNEA_ACT_RELU and hs.dtype == torch.float32 and \
            D % 4 == 0 and use_sliced(csr.n_rows, D, torch.float32)
        if ctx.bits:
            out, keep = spmm_sliced_m(csr, hs, D)
        else:
            out = spmm_sliced(csr, hs, D, act)
            keep = out
        ctx.csr, ctx.act = csr, act
        ctx.save_for_backward(x, weight, keep)
        return out

    @staticmethod
    def backward(ctx, dy):
        x, weight, keep = ctx.saved_tensors
        if ctx.bits:
            dh = spmm_sliced(ctx.csr.transpose(), act_bwd_sliced_bits(dy, keep, weight.shape[0]),
                             weight.shape[0])
        else:
            dh = aggregate_t_into(ctx.csr, dy, keep, ctx.act)
        need_x, need_w, need_b = ctx.needs_input_grad[:3]
        dx = gemm(dh, weight) if need_x else None
        dw, db = _wgrads(dh, x, need_w, need_b)
        return dx, dw, db, None, None


def gcn_layer(adj, x, weight, bias, act_fn):
    """Fused GCN layer (GCNLayerFn) when the slice-major path applies, else None.  ``adj``: the
    reference's sparse adjacency, or a DistAdj whose rank aggregates without exchange."""
    code = act_code(act_fn)
    if code is None or x.dtype not in FEATURE_DTYPES or weight.dtype != x.dtype or \
            x.shape[1] != weight.shape[1]:
        return None
    if hasattr(adj, "local_csr"):
        csr = adj.local_csr()
        if csr is None:
            return None
    elif getattr(adj, "is_sparse", False):
        csr = csr_of(adj)
    else:
        return None
    if not use_sliced(csr.n_cols, weight.shape[0], x.dtype) or x.shape[0] != csr.n_cols:
        return None
    return GCNLayerFn.apply(_rows(x), weight, bias, csr, code)


def aggregate(adj, hidden, act_fn=None):
    """Drop-in for ``act(torch.spmm(adj, hidden))``: fused when ``act_fn`` is known."""
    csr = csr_of(adj)
    code = act_code(act_fn) if act_fn is not None else _lib.GNNEA_ACT_IDENTITY
    if code is None:
        return act_fn(AggregateFn.apply(hidden, csr, _lib.GNNEA_ACT_IDENTITY))
    return AggregateFn.apply(hidden, csr, code)


def highway_fwd(csr, hidden, gate_pre, resid, bias_gate, act):
    """S = act(A·hidden); g = sigmoid(gate_pre + bias_gate); out = g*S + (1-g)*resid in one
    kernel (gnnea_spmm_highway_*), per diagonal block.  ``hidden`` has csr.n_cols rows, the
    others csr.n_rows.  Returns (out, S, g)."""
    hidden = _rows(hidden)
    gate_pre = _rows(gate_pre, hidden.dtype)
    resid = _rows(resid, hidden.dtype)
    N, D = csr.n_rows, hidden.shape[1]
    if hidden.shape[0] < csr.n_cols or gate_pre.shape != (N, D) or resid.shape != (N, D):
        raise ValueError("gnnea.highway: shape mismatch")
    out = torch.empty((N, D), dtype=hidden.dtype, device=hidden.device)
    S = torch.empty_like(out)
    G = torch.empty_like(out)
    bias = _featc(bias_gate, torch.float32) if bias_gate is not None else None
    fn = _lib.lib().gnnea_spmm_highway_bf16 if hidden.dtype == torch.bfloat16 else \
        _lib.lib().gnnea_spmm_highway_f32
    with _lib.on_device(hidden.device):
        for r0, r1 in _blocks(csr, hidden):
            check(fn(
                ctypes.c_void_p(csr.rowptr.data_ptr() + 4 * r0), ptr(csr.col), ptr(csr.val),
                r1 - r0, D, ptr(hidden), hidden.stride(0), _off(gate_pre, r0),
                gate_pre.stride(0), ptr(bias), _off(resid, r0), resid.stride(0),
                _off(out, r0), out.stride(0), _off(S, r0), _off(G, r0), S.stride(0),
                int(act), stream_of(hidden.device)))
    return out, S, G


def highway_bwd(dy, S, G, resid, act, want_dresid=True, dS=None, dgate=None, dresid=None):
    """Elementwise HighWay backward (gnnea_highway_bwd_ld_*): returns (dS_pre, dgate, dresid)
    with dS_pre = dy*g*act'(S) (to be aggregated by A^T), dgate = dy*(S-x)*g*(1-g),
    dresid = dy*(1-g) (None unless wanted).  dy, S, G, resid share one row stride; the outputs
    may be caller-provided column blocks of wider buffers."""
    S = _featc(S)
    dy = _featc(dy, S.dtype)
    G = _featc(G, S.dtype)
    resid = _featc(resid, S.dtype)
    dS = torch.empty_like(S) if dS is None else dS
    dgate = torch.empty_like(S) if dgate is None else dgate
    if want_dresid and dresid is None:
        dresid = torch.empty_like(S)
    for t in (dS, dgate) + ((dresid,) if want_dresid else ()):
        if t.shape != S.shape or t.dtype != S.dtype or t.stride(1) != 1:
            raise ValueError("gnnea.highway_bwd: output block shape / dtype mismatch")
    fn = _lib.lib().gnnea_highway_bwd_ld_bf16 if S.dtype == torch.bfloat16 else \
        _lib.lib().gnnea_highway_bwd_ld_f32
    N, D = S.shape
    with _lib.on_device(S.device):
        check(fn(
            ptr(dy), ptr(S), ptr(G), ptr(resid), S.stride(0), N, D, ptr(dS), _ld(dS),
            ptr(dgate), _ld(dgate), ptr(dresid if want_dresid else None),
            _ld(dresid) if want_dresid else D, int(act), stream_of(S.device)))
    return dS, dgate, (dresid if want_dresid else None)


class HighwayFn(torch.autograd.Function):
    """HighWay GCN tail (layers/layers.py:64-76) in one kernel:
    S = act(A·hidden); g = sigmoid(gate_pre + bias_gate); out = g*S + (1-g)*resid."""

    @staticmethod
    def forward(ctx, hidden, gate_pre, resid, bias_gate, csr, act):
        resid = _featc(resid, _featc(hidden).dtype)
        out, S, G = highway_fwd(csr, hidden, gate_pre, resid, bias_gate, act)
        ctx.csr = csr
        ctx.act = act
        ctx.save_for_backward(S, G, resid)
        return out

    @staticmethod
    def backward(ctx, dy):
        S, G, resid = ctx.saved_tensors
        dS, dgate, dres = highway_bwd(dy, S, G, resid, ctx.act, ctx.needs_input_grad[2])
        dh = spmm(ctx.csr.transpose(), dS)
        return dh, dgate, dres, None, None, None


def gate_offset(D):
    """First column of gate_pre in the fused HighWay projection table: D rounded up to a whole
    64-column slice, so that output slice q's gate columns are exactly table slice goff/64 + q
    (one 256-B piece per row for the aggregation's epilogue and the backward, not two partial
    ones); the padding columns' weights are zero."""
    return (D + SLICE_W - 1) // SLICE_W * SLICE_W


def highway_fwd_sliced(csr, Zs, D, resid, bias_gate, act, save_g=True, goff=None, save_s=True):
    """HighWay tail over the slice-major projection table Zs ([S, N, 64] holding x·[Wᵀ | 0 | K_g]
    + [b | 0]: hidden in columns [0, D), gate_pre in [goff, goff + D), goff = D by default), per
    diagonal block (gnnea_spmm_highway_sliced_f32).  Returns (out, S, g), row-major; g is None
    with ``save_g=False`` (the backward recomputes it from Zs: highway_bwd_sliced_zg)."""
    goff = D if goff is None else goff
    resid = _rows(resid, torch.float32)
    N = csr.n_rows
    if Zs.dim() != 3 or Zs.shape[2] != SLICE_W or Zs.shape[1] < csr.n_cols or \
            Zs.shape[0] * SLICE_W < goff + D or goff < D or resid.shape != (N, D):
        raise ValueError("gnnea.highway_sliced: shape mismatch")
    out = torch.empty((N, D), dtype=torch.float32, device=Zs.device)
    S = torch.empty_like(out) if save_s else None
    G = torch.empty_like(out) if save_g else None
    bias = _featc(bias_gate, torch.float32) if bias_gate is not None else None
    L = _lib.lib()
    with _lib.on_device(Zs.device):
        for r0, r1 in csr.row_blocks():
            check(L.gnnea_spmm_highway_sliced_f32(
                _off32(csr.rowptr, r0), ptr(csr.col), ptr(csr.val), r1 - r0, D, ptr(Zs),
                Zs.stride(0), ctypes.c_void_p(Zs.data_ptr() + 4 * r0 * SLICE_W), Zs.stride(0),
                goff, ptr(bias), _off(resid, r0), resid.stride(0), _off(out, r0), out.stride(0),
                _off(S, r0) if save_s else None, _off(G, r0) if save_g else None, D, int(act),
                stream_of(Zs.device)))
    return out, S, G


def highway_fwd_sliced_m(csr, Zs, D, resid, bias_gate, goff):
    """highway_fwd_sliced (relu) storing S's sign mask instead of S (gnnea_spmm_highway_sliced_m_f32):
    returns (out, mask), mask uint8 [N, 16 * ceil(D / 64)]."""
    resid = _rows(resid, torch.float32)
    N = csr.n_rows
    if Zs.dim() != 3 or Zs.shape[2] != SLICE_W or Zs.shape[1] < csr.n_cols or \
            Zs.shape[0] * SLICE_W < goff + D or goff < D or resid.shape != (N, D):
        raise ValueError("gnnea.highway_sliced_m: shape mismatch")
    out = torch.empty((N, D), dtype=torch.float32, device=Zs.device)
    ldm = 16 * ((D + SLICE_W - 1) // SLICE_W)
    mask = torch.empty((N, ldm), dtype=torch.uint8, device=Zs.device)
    bias = _featc(bias_gate, torch.float32) if bias_gate is not None else None
    L = _lib.lib()
    with _lib.on_device(Zs.device):
        for r0, r1 in csr.row_blocks():
            check(L.gnnea_spmm_highway_sliced_m_f32(
                _off32(csr.rowptr, r0), ptr(csr.col), ptr(csr.val), r1 - r0, D, ptr(Zs),
                Zs.stride(0), ctypes.c_void_p(Zs.data_ptr() + 4 * r0 * SLICE_W), Zs.stride(0),
                goff, ptr(bias), _off(resid, r0), resid.stride(0), _off(out, r0), out.stride(0),
                ctypes.c_void_p(mask.data_ptr() + r0 * ldm), ldm, _lib.GNNEA_ACT_RELU,
                stream_of(Zs.device)))
    return out, mask


def highway_bwd_sliced_zgm(dy, out, mask, Zs, D, bias_gate, resid, act, want_dresid, dgate, goff):
    """The fused HighWay layer's backward without S (gnnea_highway_bwd_sliced_zgm_f32): act'
    from the forward's relu sign mask (None for identity), S - resid from its output."""
    out = _featc(out)
    dy = _featc(dy, out.dtype)
    resid = _featc(resid, out.dtype)
    N = out.shape[0]
    dSs = sliced_empty(N, D, out.device)
    dres = torch.empty_like(out) if want_dresid else None
    bias = _featc(bias_gate, torch.float32) if bias_gate is not None else None
    with _lib.on_device(out.device):
        check(_lib.lib().gnnea_highway_bwd_sliced_zgm_f32(
            ptr(dy), ptr(out), ptr(Zs), Zs.stride(0), goff, ptr(bias), ptr(resid), out.stride(0),
            N, D, ptr(mask), mask.stride(0) if mask is not None else 0, ptr(dSs), dSs.stride(0),
            ptr(dgate), _ld(dgate), ptr(dres), _ld(dres) if want_dresid else D, int(act),
            stream_of(out.device)))
    return dSs, dres


def highway_bwd_sliced_zg(dy, S, Zs, D, bias_gate, resid, act, want_dresid, dgate, goff=None):
    """highway_bwd_sliced with g = sigmoid(gate_pre + bias_gate) recomputed from the projection
    table Zs (gate_pre at column goff, D by default; gnnea_highway_bwd_sliced_zg_f32) instead of
    a saved G."""
    goff = D if goff is None else goff
    S = _featc(S)
    dy = _featc(dy, S.dtype)
    resid = _featc(resid, S.dtype)
    N = S.shape[0]
    dSs = sliced_empty(N, D, S.device)
    dres = torch.empty_like(S) if want_dresid else None
    bias = _featc(bias_gate, torch.float32) if bias_gate is not None else None
    with _lib.on_device(S.device):
        check(_lib.lib().gnnea_highway_bwd_sliced_zg_f32(
            ptr(dy), ptr(S), ptr(Zs), Zs.stride(0), goff, ptr(bias), ptr(resid), S.stride(0), N, D,
            ptr(dSs), dSs.stride(0), ptr(dgate), _ld(dgate), ptr(dres),
            _ld(dres) if want_dresid else D, int(act), stream_of(S.device)))
    return dSs, dres


def highway_bwd_sliced(dy, S, G, resid, act, want_dresid, dgate):
    """highway_bwd with dS_pre written slice-major (gnnea_highway_bwd_sliced_f32); dgate is a
    caller-provided row-major (column-block) buffer.  Returns (dS slices, dresid or None)."""
    S = _featc(S)
    dy = _featc(dy, S.dtype)
    G = _featc(G, S.dtype)
    resid = _featc(resid, S.dtype)
    N, D = S.shape
    dSs = sliced_empty(N, D, S.device)
    dres = torch.empty_like(S) if want_dresid else None
    with _lib.on_device(S.device):
        check(_lib.lib().gnnea_highway_bwd_sliced_f32(
            ptr(dy), ptr(S), ptr(G), ptr(resid), S.stride(0), N, D, ptr(dSs), dSs.stride(0),
            ptr(dgate), _ld(dgate), ptr(dres), _ld(dres) if want_dresid else D, int(act),
            stream_of(S.device)))
    return dSs, dres


_ONES = {}


def _ones(n, device):
    key = (str(device), n)
    o = _ONES.get(key)
    if o is None:
        if len(_ONES) > 16:
            _ONES.clear()
        o = _ONES[key] = torch.ones((n, 1), dtype=torch.float32, device=device)
    return o


def colsum(t, out_dtype=None):
    """Column sums of a row-major [N, D] matrix (the bias gradients): one streaming pass with
    a deterministic two-stage sum (gnnea_colsum_*, the attention-gradient pass with unit
    weights) instead of a [1, N]·[N, D] split-K GEMM; fp32 sums, returned in ``out_dtype``
    (default t's dtype).  t may be a column block of a wider row-major buffer."""
    t = _rows(t)
    N, D = t.shape
    out_dtype = out_dtype or t.dtype
    es = t.element_size()
    if ((t.stride(0) * es) % 4 or t.data_ptr() % 4 or N == 0 or t.stride(0) < D
            or t.dtype not in FEATURE_DTYPES):
        t = _featc(t)
        ones = torch.ones((1, N), dtype=t.dtype, device=t.device)
        return gemm(ones, t, out_dtype=out_dtype if t.dtype == torch.bfloat16 else None).view(-1)
    L = _lib.lib()
    ws_bytes = int(L.gnnea_gat_da_ws_bytes(N, D))
    ws = _gemm_ws(t.device, ws_bytes)
    s = torch.empty(D, dtype=torch.float32, device=t.device)
    fn = L.gnnea_colsum_bf16 if t.dtype == torch.bfloat16 else L.gnnea_colsum_f32
    with _lib.on_device(t.device):
        check(fn(ptr(t), t.stride(0), N, D, ptr(s), ptr(ws), ws_bytes, stream_of(t.device)))
    return s if out_dtype == torch.float32 else s.to(out_dtype)


class HighwayLayerFn(torch.autograd.Function):
    """A whole HighWay graph convolution (layers/layers.py:58-77, dropout inactive), fp32:

      forward   Z = x·[Wᵀ | K_g] + [b | 0]        ONE MFMA pass over x (hidden | gate_pre)
                out, S, g = highway(A, Z[:, :D], Z[:, D:], x, b_g)      (gnnea_spmm_highway)
      backward  dS, [dh | dgate], dres = highway_bwd(...)   dgate written next to dh
                dh = Aᵀ·dS                                   into the same [N, 2D] buffer
                dx = dres + [dh | dgate]·[W ; K_gᵀ]           ONE GEMM accumulating into dres
                dW = dhᵀ·x,  db = colsum(dh)
    which replaces two forward GEMMs, two input-gradient GEMMs and the two autograd additions
    of the three uses of x with one GEMM each way."""

    @staticmethod
    def forward(ctx, x, weight, bias, kernel_gate, bias_gate, agg, act):
        D = weight.shape[0]
        wcat = torch.cat([weight.t(), kernel_gate.to(weight.dtype)], dim=1)  # [Din, 2D]
        bcat = torch.cat([bias, torch.zeros_like(bias)]) if bias is not None else None
        ctx.sliced = agg.sliced_ok(D, x.dtype)
        if ctx.sliced:
            # above the Infinity Cache: Z written slice-major by the GEMM, the HighWay SpMM
            # gathers the hidden slices and reads gate_pre from the same table, starting at the
            # first whole slice past the hidden columns (gate_offset: zero weight columns in
            # between); the gate itself is not stored: the backward recomputes it from Z (kept
            # alive instead)
            goff = gate_offset(D)
            if goff != D:
                pad = torch.zeros((wcat.shape[0], goff - D), dtype=wcat.dtype, device=wcat.device)
                wcat = torch.cat([wcat[:, :D], pad, wcat[:, D:]], dim=1)
                if bcat is not None:
                    bcat = torch.cat([bias, torch.zeros(goff, dtype=bias.dtype, device=bias.device)])
            Zs = gemm_sliced(x, wcat.t(), bcat)
            # relu / identity: S is not stored either -- the backward takes act' from a sign
            # mask (relu) and S - x from the output (g (S - x) = out - x)
            ctx.masked = int(act) in (_lib.GNNEA_ACT_RELU, _lib.GNNEA_ACT_IDENTITY) and \
                hasattr(agg, "highway_fwd_sliced_m")
            if ctx.masked and int(act) == _lib.GNNEA_ACT_RELU:
                out, S = agg.highway_fwd_sliced_m(Zs, D, x, bias_gate, goff)  # S: the mask
            elif ctx.masked:
                out, S, _ = agg.highway_fwd_sliced(Zs, D, x, bias_gate, act, goff=goff,
                                                   save_s=False)  # (S None)
            else:
                out, S, _ = agg.highway_fwd_sliced(Zs, D, x, bias_gate, act, goff=goff)
            G = Zs
            ctx.goff = goff
        else:
            Z = gemm(x, wcat, bias=bcat)
            out, S, G = agg.highway_fwd(Z[:, :D], Z[:, D:], x, bias_gate, act)
        ctx.agg, ctx.act = agg, act
        # bias_gate goes through save_for_backward too (the sliced backward recomputes the gate
        # from it): an in-place update between forward and backward raises autograd's version
        # error instead of silently using the new value
        if ctx.sliced and ctx.masked:
            ctx.save_for_backward(x, weight, kernel_gate, S, G, bias_gate, out)
        else:
            ctx.save_for_backward(x, weight, kernel_gate, S, G, bias_gate)
        return out

    @staticmethod
    def backward(ctx, dy):
        if ctx.sliced and ctx.masked:
            x, weight, Kg, S, G, bias_gate, out = ctx.saved_tensors  # (S: the relu mask or None)
        else:
            x, weight, Kg, S, G, bias_gate = ctx.saved_tensors
            out = None
        N, D = x.shape[0], weight.shape[0]
        need_x, need_w, need_b = ctx.needs_input_grad[:3]
        pdt = torch.float32 if (ctx.sliced and ctx.masked) else S.dtype
        P = torch.empty((N, 2 * D), dtype=pdt, device=x.device)
        if ctx.sliced and ctx.masked:  # (G is the projection table Zs here)
            dSs, dres = highway_bwd_sliced_zgm(dy, out, S, G, D, bias_gate, x, ctx.act,
                                               need_x, P[:, D:], ctx.goff)
            ctx.agg.aggregate_t_sliced(dSs, D, P[:, :D])
        elif ctx.sliced:
            dSs, dres = highway_bwd_sliced_zg(dy, S, G, D, bias_gate, x, ctx.act, need_x,
                                              P[:, D:], goff=ctx.goff)
            ctx.agg.aggregate_t_sliced(dSs, D, P[:, :D])
        else:
            dS, _, dres = highway_bwd(dy, S, G, x, ctx.act, want_dresid=need_x, dgate=P[:, D:])
            ctx.agg.aggregate_t(dS, P[:, :D])
        dh = P[:, :D]
        dx = dw = db = None
        if need_x:
            w2 = torch.cat([weight, Kg.t().to(weight.dtype)], dim=0)  # [2D, Din]
            dx = gemm(P, w2, out=dres, beta=1.0)
        dw, db = _wgrads(dh, x, need_w, need_b)
        return dx, dw, db, None, None, None, None


class LocalAgg:
    """The aggregation of one whole adjacency on this device (the sharded counterpart with the
    same two methods is gnnea.dist_graph.DistAdj)."""

    def __init__(self, csr):
        self.csr = csr

    def highway_fwd(self, hidden, gate_pre, resid, bias_gate, act):
        return highway_fwd(self.csr, hidden, gate_pre, resid, bias_gate, act)

    def aggregate_t(self, g, out):
        """out = Aᵀ·g (out may be a column block of a wider buffer)."""
        return spmm(self.csr.transpose(), g, out=out)

    def sliced_ok(self, D, dtype):
        return dtype == torch.float32 and use_sliced(self.csr.n_cols, D, dtype)

    def highway_fwd_sliced(self, Zs, D, resid, bias_gate, act, goff=None, save_s=True):
        return highway_fwd_sliced(self.csr, Zs, D, resid, bias_gate, act, save_g=False,
                                  goff=goff, save_s=save_s)

    def highway_fwd_sliced_m(self, Zs, D, resid, bias_gate, goff):
        return highway_fwd_sliced_m(self.csr, Zs, D, resid, bias_gate, goff)

    def aggregate_t_sliced(self, gs, D, out):
        return spmm_sliced(self.csr.transpose(), gs, D, out=out)


def highway_layer(adj, x, weight, bias, kernel_gate, bias_gate, act_fn):
    """Fused HighWay layer when it applies (fp32, fusable act), else None.  ``adj``: the
    reference's sparse adjacency or a DistAdj shard."""
    code = act_code(act_fn)
    if code is None or x.dtype != torch.float32 or weight.dtype != torch.float32 or \
            x.shape[1] != weight.shape[1] or weight.shape[0] != x.shape[1]:
        return None
    agg = adj if hasattr(adj, "aggregate_t") else LocalAgg(csr_of(adj))
    return HighwayLayerFn.apply(_rows(x), weight, bias, kernel_gate, bias_gate, agg, code)


def highway(adj, hidden, gate_pre, resid, bias_gate, act_fn):
    csr = csr_of(adj)
    code = act_code(act_fn)
    if code is None:
        # non-fusable activation: aggregate in HIP, finish the blend in torch
        s = act_fn(AggregateFn.apply(hidden, csr, _lib.GNNEA_ACT_IDENTITY))
        g = torch.sigmoid(gate_pre + bias_gate) if bias_gate is not None else torch.sigmoid(gate_pre)
        return g * s + (1.0 - g) * resid
    return HighwayFn.apply(hidden, gate_pre, resid, bias_gate, csr, code)


# ------------------------------------------------------------------------------------------ #
# GAT (all heads, one edge pass)                                                              #
# ------------------------------------------------------------------------------------------ #
def _gat_fn(name, dtype):
    """C-ABI entry of a GAT kernel for the feature storage dtype (fp32 or bf16)."""
    return getattr(_lib.lib(), name + ("_bf16" if dtype == torch.bfloat16 else "_f32"))


def gat_scores(H, a_all, heads, d_head):
    N = H.shape[0]
    s1 = torch.empty((N, heads), dtype=torch.float32, device=H.device)
    s2 = torch.empty_like(s1)
    with _lib.on_device(H.device):
        check(_gat_fn("gnnea_gat_scores", H.dtype)(ptr(H), H.stride(0), N, heads, d_head,
                                                   ptr(a_all), ptr(s1), ptr(s2),
                                                   stream_of(H.device)))
    return s1, s2


def _pad4(t, D, dtype=None):
    """[N, roundup4(D)] row-major tensor, rows aligned for one 4-element vector per lane (16 B
    fp32, 8 B bf16), whose first D columns are t (in ``dtype``); t itself when it qualifies."""
    dtype = dtype or (t.dtype if t.dtype in FEATURE_DTYPES else torch.float32)
    Dp = (D + 3) // 4 * 4
    es = torch.empty((), dtype=dtype).element_size()
    if (t.dtype == dtype and t.stride(1) == 1 and t.stride(0) == Dp
            and t.data_ptr() % (4 * es) == 0
            and (t.storage_offset() + t.shape[0] * Dp) * es <= t.untyped_storage().nbytes()):
        return t
    out = torch.zeros((t.shape[0], Dp), dtype=dtype, device=t.device)
    out[:, :D] = t
    return out


# tests switch it off (monkeypatch) to compare with the row-major edge pass
GAT_SLICED = True
# bf16 storage (cfg-5): the sliced passes are built and parity-tested but not the default.  At
# cfg-5 (2 x 2M rows, 84M edges) the passes are bound by per-edge work, not by gathered bytes:
# five 128-B slice passes cost five times the per-edge overhead of one 600-B row-major pass
# (per KG: forward 6.4 ms sliced + 1.3 ms row statistics vs 6.3 ms row-major; source pass 8.7
# vs 10.8 ms but the side passes add ~6 ms per layer; GAT-EA step 145 vs 133 ms).
GAT_SLICED_BF16 = False


def gat_two_heads_per_slice(heads, d_head):
    """The sliced GAT kernels keep two heads per 64-column slice (h0 / h1, two product partials
    per edge): every slice s must satisfy min((64s+63)//d, H-1) - (64s)//d <= 1 (d_head >= 64,
    or 32 / 48 / ...; d_head = 40 puts heads 1, 2, 3 in slice 1 and is refused)."""
    if heads < 1 or d_head < 32:
        return False
    D = heads * d_head
    return all(min((64 * s + 63) // d_head, heads - 1) - (64 * s) // d_head <= 1
               for s in range((D + 63) // 64))


def gat_sliced_wanted(n_rows, heads, d_head, dtype):
    """The GAT passes run over 64-column slice-major tables (fp32: 256 B, bf16: 128 B per row
    piece; one KG slice of cfg-4 fp32 / cfg-5 bf16 is 256 MB) when the row-major table of
    ``n_rows`` projected rows exceeds the Infinity Cache and spans at least two slices.  The
    projection GEMM asks this before writing its sliced copy (att_layers.GraphAttentionLayer),
    so no copy is made that the forward would not consume."""
    D = heads * d_head
    es = torch.tensor([], dtype=dtype).element_size()
    return (GAT_SLICED and (dtype == torch.float32 or
                            (dtype == torch.bfloat16 and GAT_SLICED_BF16))
            and gat_two_heads_per_slice(heads, d_head)
            and D % 4 == 0 and heads <= 8 and 128 <= D <= 1024
            and n_rows * D * es > INFINITY_CACHE_BYTES
            # (the sliced passes address a slice with 32-bit offsets: one slice < 4 GB; larger
            # tables take the row-major head-grouped passes)
            and n_rows * 64 * es < (1 << 32) - (1 << 24))


def _gat_sliced_applies(H, heads, d_head, Y):
    return Y.shape[1] == heads * d_head and gat_sliced_wanted(H.shape[0], heads, d_head, H.dtype)


def slice_pack64(x):
    """Row-major [n, D] (fp32 / bf16) -> the 64-column slice-major GAT table."""
    x = _rows(x)
    n, D = x.shape
    xs = sliced_empty(n, D, x.device, x.dtype, W=64)
    with _lib.on_device(x.device):
        check(_sfn("gnnea_slice_pack64", x.dtype)(ptr(x), _ld(x), n, D, ptr(xs), xs.stride(0),
                                                 stream_of(x.device)))
    return xs


def gat_forward(csr, H, a32, heads, d_head, alpha, act, em=None, row0=0):
    """All heads of the GAT aggregation over ``csr`` (one edge pass per KG block).

    H: the source table (every row the CSR references, row-major, 4-aligned rows: _pad4).
    The CSR's destination row i is row ``row0 + i`` of H's index space (row0 = 0 for the whole
    graph; the first owned row for a row shard, gnnea.dist_graph).  Returns (Y [n_rows, Dp],
    m, den, s1, s2): Y and the per-row softmax records of the destination rows, the logits
    s1 / s2 of every H row."""
    D = heads * d_head
    N = csr.n_rows
    s1, s2 = gat_scores(H, a32, heads, d_head)
    Y = torch.empty((N, (D + 3) // 4 * 4), dtype=H.dtype, device=H.device)
    m = torch.empty((N, heads), dtype=torch.float32, device=H.device)
    den = torch.empty_like(m)
    if _gat_sliced_applies(H, heads, d_head, Y):
        # above the Infinity Cache: the table slice-major (64-column slices, one 256-MB table
        # per KG slice), row statistics once, then the slices one after another
        Hs = sliced_copy_of(H, D) if H.dtype == torch.float32 else None
        if Hs is None:
            Hs = slice_pack64(H[:, :D])
        wgt = torch.empty((max(csr.nnz, 1), heads), dtype=torch.float32, device=H.device)
        fs = _gat_fn("gnnea_gat_fwd_sliced", H.dtype)
        with _lib.on_device(H.device):
            for r0, r1 in _blocks(csr, H):
                check(fs(_off32(csr.rowptr, r0), ptr(csr.col), r1 - r0, ptr(Hs), Hs.stride(0),
                         heads, d_head, _off(s1, row0 + r0), ptr(s2), float(alpha), ptr(em),
                         int(act), _off(Y, r0), Y.stride(0), _off(m, r0), _off(den, r0),
                         ptr(wgt), stream_of(H.device)))
        return Y, m, den, s1, s2
    fwd = _gat_fn("gnnea_gat_fwd", H.dtype)
    with _lib.on_device(H.device):
        for r0, r1 in _blocks(csr, H):  # per KG block when H exceeds the Infinity Cache
            check(fwd(_off32(csr.rowptr, r0), ptr(csr.col), r1 - r0, ptr(H), H.stride(0),
                      heads, d_head, _off(s1, row0 + r0), ptr(s2), float(alpha), ptr(em),
                      int(act), _off(Y, r0), Y.stride(0), _off(m, r0), _off(den, r0),
                      stream_of(H.device)))
    return Y, m, den, s1, s2


def gat_backward(csr, H, a32, s1, s2, m, den, Y, dY, heads, d_head, alpha, act, em=None,
                 row0=0, need_da=True):
    """Gradients of sum(Y ⊙ dY) for gat_forward's outputs: (dH [rows of H, Dp], da or None).

    One prep pass over the destination rows (G = dY·act', softmax records), one gather sweep
    over Aᵀ (per source row j: SDDMM, softmax backward, dH_j and ds2_j, no atomics), one pass
    over the destination rows through the transpose position map (ds1_i, dH_{row0+i} += ...).
    Above the Infinity Cache (use_sliced) G is slice-major and the sweep runs slice by slice
    (_gat_backward_sliced), as gat_forward does.
    For a row shard dH and da are this shard's partials (summed across the KG group / world by
    the caller)."""
    csrT = csr.transpose()
    D = heads * d_head
    dY = _pad4(dY, D, H.dtype)
    if dY.shape[1] != Y.shape[1]:
        dY = _pad4(dY[:, :D].contiguous(), D, H.dtype)
    N = csr.n_rows
    dev = H.device
    rec = torch.empty((N, heads, 4), dtype=torch.float32, device=dev)
    dH = torch.empty_like(H)
    dzT = torch.empty((max(csr.nnz, 1), heads), dtype=torch.float32, device=dev)
    ds1 = torch.empty((N, heads), dtype=torch.float32, device=dev)
    ds2 = torch.empty((H.shape[0], heads), dtype=torch.float32, device=dev)
    if _gat_sliced_applies(H, heads, d_head, Y):
        _gat_backward_sliced(csr, csrT, H, a32, s1, s2, m, den, Y, dY, heads, d_head,
                             alpha, act, em, row0, rec, dH, dzT, ds1, ds2)
    else:
        _gat_backward_rows(csr, csrT, H, a32, s1, s2, m, den, Y, dY, heads, d_head, alpha,
                           act, em, row0, rec, dH, dzT, ds1, ds2)
    da = None
    if need_da:
        # da1[h] = sum_i ds1[i,h] H_{row0+i},h ; da2[h] = sum_j ds2[j,h] H_j,h: one streaming
        # pass over H each (gnnea_gat_da_*), only the diagonal head blocks
        if row0 == 0 and H.shape[0] == N:  # both weight the same rows: one pass
            p1, p2 = gat_da(H, ds1, heads, d_head, ds2)
        else:
            p1 = gat_da(H[row0:row0 + N], ds1, heads, d_head)
            p2 = gat_da(H, ds2, heads, d_head)
        da = torch.cat([p1.view(heads, d_head), p2.view(heads, d_head)], dim=1)
    return dH, da


def _gat_backward_sliced(csr, csrT, H, a32, s1, s2, m, den, Y, dY, heads, d_head, alpha,
                         act, em, row0, rec, dH, dzT, ds1, ds2):
    """The backward over a slice-major G (gnnea_gat_bwd_*_sliced_{f32,bf16}): G's 64-column
    slices are 256-MB tables per KG (cfg-4 fp32, cfg-5 bf16) that the source-side gathers of one
    slice pass stay inside."""
    D = heads * d_head
    N = csr.n_rows
    dev = H.device
    st = stream_of(dev)
    Gs = sliced_empty(N, D, dev, H.dtype, W=64)
    S = Gs.shape[0]
    nnzT = csrT.nnz
    wT = torch.empty((max(nnzT, 1), heads), dtype=torch.float32, device=dev)
    pd = torch.empty((S, max(nnzT, 1), 2), dtype=torch.float32, device=dev)
    # ds2 (x) a2 rides the destination pass when source and destination rows coincide
    fold = row0 == 0 and H.shape[0] == N and csrT.n_rows == N
    with _lib.on_device(dev):
        check(_gat_fn("gnnea_gat_bwd_prep_sliced", H.dtype)(
            N, heads, d_head, ptr(dY), ptr(Y), Y.stride(0), _off(s1, row0), ptr(m), ptr(den),
            int(act), ptr(Gs), Gs.stride(0), ptr(rec), st))
        for j0, j1 in _blocks(csrT, Y):  # source rows j of A^T, per KG block
            check(_gat_fn("gnnea_gat_bwd_src_sliced", H.dtype)(
                _off32(csrT.rowptr, j0), ptr(csrT.col), ptr(csrT.perm), j1 - j0, heads, d_head,
                _off(H, j0), H.stride(0), _off(s2, j0), alpha, ptr(em), ptr(rec), ptr(Gs),
                Gs.stride(0), ptr(wT), ptr(pd), nnzT, _off(dH, j0), dH.stride(0), st))
        check(_gat_fn("gnnea_gat_bwd_edge_sliced", H.dtype)(
            ptr(csrT.rowptr), ptr(csrT.col), ptr(csrT.perm), csrT.n_rows, heads, d_head, ptr(s2),
            alpha, ptr(em), ptr(rec), ptr(pd), nnzT, ptr(a32), None if fold else ptr(dH),
            dH.stride(0), ptr(dzT), ptr(ds2), st))
        if csrT.n_rows < H.shape[0]:  # H rows no edge references: no gradient
            dH[csrT.n_rows:].zero_()
            ds2[csrT.n_rows:].zero_()
        check(_gat_fn("gnnea_gat_bwd_dst_sliced", H.dtype)(
            ptr(csr.rowptr), ptr(csr.tpos()), N, heads, d_head, ptr(dzT), ptr(a32),
            ptr(ds2) if fold else None, _off(dH, row0), dH.stride(0), ptr(ds1), st))


def _gat_backward_rows(csr, csrT, H, a32, s1, s2, m, den, Y, dY, heads, d_head, alpha,
                       act, em, row0, rec, dH, dzT, ds1, ds2):
    """The backward over row-major G (gnnea_gat_bwd_prep / _src / _dst)."""
    tpos = csr.tpos()
    N = csr.n_rows
    dev = H.device
    st = stream_of(dev)
    G = torch.empty_like(Y)
    with _lib.on_device(dev):
        # G = dL/dh' and the per-node record {s1, m, 1/den, G.h'} (relu / identity: Y = h')
        check(_gat_fn("gnnea_gat_bwd_prep", H.dtype)(
            N, heads, d_head, ptr(dY), ptr(Y), Y.stride(0), _off(s1, row0), ptr(m), ptr(den),
            int(act), ptr(G), ptr(rec), st))
        src = _gat_fn("gnnea_gat_bwd_src", H.dtype)
        L = _lib.lib()
        for j0, j1 in _blocks(csrT, G):  # source rows j of A^T, per KG block
            if H.dtype == torch.bfloat16:  # G rows gathered as 16-B windows (G's rows known)
                check(L.gnnea_gat_bwd_src_rows_bf16(
                    _off32(csrT.rowptr, j0), ptr(csrT.col), ptr(csrT.perm), j1 - j0, heads,
                    d_head, _off(H, j0), H.stride(0), _off(s2, j0), alpha, ptr(em), ptr(rec),
                    ptr(G), G.stride(0), G.shape[0], ptr(a32), _off(dH, j0), dH.stride(0),
                    ptr(dzT), _off(ds2, j0), st))
                continue
            check(src(_off32(csrT.rowptr, j0), ptr(csrT.col), ptr(csrT.perm), j1 - j0, heads,
                      d_head, _off(H, j0), H.stride(0), _off(s2, j0), alpha, ptr(em),
                      ptr(rec), ptr(G), G.stride(0), ptr(a32), _off(dH, j0), dH.stride(0),
                      ptr(dzT), _off(ds2, j0), st))
        if csrT.n_rows < H.shape[0]:  # H rows no edge references: no gradient
            dH[csrT.n_rows:].zero_()
            ds2[csrT.n_rows:].zero_()
        check(_gat_fn("gnnea_gat_bwd_dst", H.dtype)(
            ptr(csr.rowptr), ptr(tpos), N, heads, d_head, ptr(dzT), ptr(a32), _off(dH, row0),
            dH.stride(0), ptr(ds1), st))


def gat_da(H, ds, heads, d_head, ds2=None):
    """out[c] = sum_r ds[r, c // d_head] * H[r, c] (fp32, heads*d_head values); with ``ds2`` the
    pair (out from ds, out from ds2) in one pass over H (gnnea_gat_da2_*)."""
    L = _lib.lib()
    n = H.shape[0]
    D = heads * d_head
    ws_bytes = int(L.gnnea_gat_da_ws_bytes(n, D))
    ws = _gemm_ws(H.device, ws_bytes)
    out = torch.empty(D, dtype=torch.float32, device=H.device)
    ds = _featc(ds, torch.float32)
    with _lib.on_device(H.device):
        if ds2 is not None:
            ds2 = _featc(ds2, torch.float32)
            out2 = torch.empty(D, dtype=torch.float32, device=H.device)
            check(_gat_fn("gnnea_gat_da2", H.dtype)(ptr(H), H.stride(0), n, heads, d_head,
                                                    ptr(ds), ptr(ds2), ptr(out), ptr(out2),
                                                    ptr(ws), ws_bytes, stream_of(H.device)))
            return out, out2
        check(_gat_fn("gnnea_gat_da", H.dtype)(ptr(H), H.stride(0), n, heads, d_head, ptr(ds),
                                               ptr(out), ptr(ws), ws_bytes,
                                               stream_of(H.device)))
    return out


class GATFn(torch.autograd.Function):
    """h'_i = sum_j softmax_j(-LeakyReLU(a·[h_i||h_j])) h_j for all heads at once
    (layers/att_layers.py:29-61 per head, concatenated at :86).  H in fp32 or bf16 storage (the
    output, the saved activations and dH follow it; logits and softmax records are fp32)."""

    @staticmethod
    def forward(ctx, H, a_all, csr, heads, d_head, alpha, act, edge_mask):
        D = heads * d_head
        H = _pad4(H, D)
        a32 = _featc(a_all, torch.float32)
        em = _featc(edge_mask, torch.float32) if edge_mask is not None else None
        Y, m, den, s1, s2 = gat_forward(csr, H, a32, heads, d_head, alpha, act, em)
        ctx.csr = csr
        ctx.meta = (heads, d_head, float(alpha), int(act))
        ctx.save_for_backward(H, a32, s1, s2, m, den, Y, em if em is not None else torch.empty(0))
        ctx.has_mask = em is not None
        return Y if Y.shape[1] == D else Y[:, :D]

    @staticmethod
    def backward(ctx, dY):
        H, a_all, s1, s2, m, den, Y, em = ctx.saved_tensors
        heads, d_head, alpha, act = ctx.meta
        em = em if ctx.has_mask else None
        D = heads * d_head
        dH, da = gat_backward(ctx.csr, H, a_all, s1, s2, m, den, Y, dY, heads, d_head, alpha,
                              act, em, need_da=ctx.needs_input_grad[1])
        return (dH if dH.shape[1] == D else dH[:, :D]), da, None, None, None, None, None, None


def gat(adj, H, a_all, heads, d_head, alpha, act_fn, edge_mask=None):
    csr = csr_of(adj)
    code = act_code(act_fn) if act_fn is not None else _lib.GNNEA_ACT_IDENTITY
    if code not in (_lib.GNNEA_ACT_IDENTITY, _lib.GNNEA_ACT_RELU):
        y = GATFn.apply(H, a_all, csr, heads, d_head, alpha, _lib.GNNEA_ACT_IDENTITY, edge_mask)
        return act_fn(y)
    return GATFn.apply(H, a_all, csr, heads, d_head, alpha, code, edge_mask)
