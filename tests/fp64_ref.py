"""Whole-graph fp64 torch references ON THE DEVICE for the BASELINE-size tests (test-only).

The CPU oracle (oracle/local.py) checks sampled rows; the weight gradients are sums over every
row of the graph, so they are checked against this fp64 restatement evaluated with plain torch
ops (index_add aggregation in edge chunks, vendor fp64 GEMMs) on the same device.  Formulas:
  GraphConvolution          layers/layers.py:30-39
  HighWayGraphConvolution   layers/layers.py:59-77
  EAModel.get_loss          models/models_ea.py:103-123
  GraphAttentionLayer       layers/att_layers.py:29-61, 82-91 (per head, concatenated)
ReLU's branch inside the rounding band of 0 follows the tested output (see oracle/local.py);
the number of elements that fell in the band is counted in BAND (reported by the tests).
"""
import torch

CHUNK = 1 << 22
TAU = 1e-5
BAND = {"band": 0, "total": 0}


def reset_band():
    BAND["band"] = BAND["total"] = 0


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


def relu_mask(pre, tested=None, tau=TAU):
    """relu'(pre) as a 0/1 fp64 tensor; inside |pre| <= tau*max|pre| the tested output's sign."""
    band = pre.abs() <= tau * pre.abs().max().clamp_min(1e-300)
    m = pre > 0
    if tested is not None:
        m = torch.where(band, tested > 0, m)
        BAND["band"] += int(band.sum())
        BAND["total"] += band.numel()
    return m.to(pre.dtype)


class WAgg(torch.autograd.Function):
    """out_i = sum_e w_e h[c_e] over the edges e of row r_e (differentiable in h and in the
    per-edge weights w; edge chunks, no E x D tensor is kept for the backward)."""

    @staticmethod
    def forward(ctx, h, w, r, c, n_out):
        ctx.save_for_backward(h, w)
        ctx.graph = (r, c)
        out = torch.zeros((n_out, h.shape[1]), dtype=h.dtype, device=h.device)
        for e0 in range(0, r.numel(), CHUNK):
            sl = slice(e0, e0 + CHUNK)
            out.index_add_(0, r[sl], h[c[sl]] * w[sl].unsqueeze(1))
        return out

    @staticmethod
    def backward(ctx, g):
        h, w = ctx.saved_tensors
        r, c = ctx.graph
        dh = torch.zeros_like(h)
        dw = torch.empty_like(w)
        for e0 in range(0, r.numel(), CHUNK):
            sl = slice(e0, e0 + CHUNK)
            gr = g[r[sl]]
            dw[sl] = (gr * h[c[sl]]).sum(1)
            dh.index_add_(0, c[sl], gr * w[sl].unsqueeze(1))
        return dh, dw, None, None, None


class BF16Store(torch.autograd.Function):
    """Identity that rounds its value to bf16 in the forward and its gradient to bf16 in the
    backward: the storage points of the bf16 path (a projection / activation written as bf16
    and its gradient written as bf16), so an fp64 restatement with these inserted differs from
    the bf16 kernels only by fp32-vs-fp64 accumulation, not by the storage roundings."""

    @staticmethod
    def forward(ctx, t):
        return t.to(torch.bfloat16).to(t.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


def bf16_store(t):
    return BF16Store.apply(t)


class F32Store(torch.autograd.Function):
    """The fp32 path's storage points (a projection / layer output written as fp32, its gradient
    as fp32), as BF16Store for bf16: an fp64 restatement with these inserted differs from the fp32
    kernels by their arithmetic only, not by the roundings of what they store."""

    @staticmethod
    def forward(ctx, t):
        return t.to(torch.float32).to(t.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.float32).to(g.dtype)


def f32_store(t):
    return F32Store.apply(t)


def gat_layer(x, Ws, As, r, c, alpha=0.2, relu=True, tested=None, tau=TAU, store=None):
    """GraphAttentionLayer forward (concat of the heads) in the precision of x: Ws [H, in, d],
    As [H, 1, 2d]; edges (r, c) coalesced (unique pairs); exp(-LeakyReLU(z)) without a shift,
    as the reference.  ``tested``: the layer's output under test (relu's rounding band).
    ``store``: applied to each head's projection and to the output (bf16_store emulates the
    bf16 path's storage)."""
    n = x.shape[0]
    outs = []
    d = Ws.shape[2]
    for h_ in range(Ws.shape[0]):
        hh = x @ Ws[h_]
        if store is not None:
            hh = store(hh)
        s1 = hh @ As[h_, 0, :d]
        s2 = hh @ As[h_, 0, d:]
        e = torch.exp(-torch.nn.functional.leaky_relu(s1[r] + s2[c], alpha))
        den = torch.zeros(n, dtype=x.dtype, device=x.device).index_add(0, r, e)
        o = WAgg.apply(hh, e, r, c, n) / den.unsqueeze(1)
        if relu:
            with torch.no_grad():
                m = relu_mask(o, None if tested is None else tested[:, h_ * d:(h_ + 1) * d], tau)
            o = o * m
        outs.append(o)
    y = torch.cat(outs, dim=1)
    return store(y) if store is not None else y


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



def highway_s_sign(out):
    """relu(S)'s sign as the fused HighWay layer took it (its saved mask, bit (c % 4) of byte
    [row][16 (c // 64) + (c % 64) // 4]), or None where the layer kept no mask."""
    fn = out.grad_fn
    if fn is None or type(fn).__name__ != "HighwayLayerFnBackward":
        return None
    mask = fn.saved_tensors[3]
    if mask is None or mask.dtype != torch.uint8:
        return None
    cols = torch.arange(out.shape[1], device=out.device)
    return ((mask[:, 16 * (cols // 64) + (cols % 64) // 4] >> (cols % 4).to(torch.uint8)) & 1
            ).to(torch.float32)


def ea_step_grads(m, model, x, r, c, v, ix, t, k, outputs, enc_acts, dec_acts, er=None, ec=None,
                  tau=TAU, store=None, dtype=torch.float64):
    """Every parameter gradient of one EA step (run/train_ea.py:55-66) through the fp64
    restatement of ``m`` (EAModel with the weights it holds; encoders models/encoders.py, decoders
    models/decoders.py), differentiated with the cotangent of the reference loss formula
    (models/models_ea.py:103-123) at OUR ``outputs``: the margin loss's sign pattern is chaotic
    under rounding (which sign(x_a - x_b) flip depends on the last bits of the outputs), so the
    cotangent is taken where our step took it and what is compared is the backward itself.
    ReLU branches inside the rounding band follow our activations (``enc_acts``: each encoder
    layer's output -- HGCN: relu(S)'s sign as the fused layer saved it, or None -- and
    ``dec_acts``: the MLP decoder's two relu outputs).  ``store``: bf16 storage
    emulation (bf16_store) after every projection / layer output.  ``dtype``: torch.float32
    evaluates the same restatement in fp32 (the accuracy any fp32 evaluation of these sums has,
    reported beside ours).  Returns ({name: grad} in m.named_parameters() names, outputs)."""
    p64 = {}

    def P(name, t_):
        q = t_.detach().to(dtype).requires_grad_(True)
        p64[name] = q
        return q
    st = store if store is not None else (lambda z: z)
    N = x.shape[0]
    h = x.to(dtype)
    v = v.to(dtype)
    for i, L in enumerate(m.encoder.layers):
        pre_n = "encoder.layers.%d." % i
        tst = enc_acts[i].to(dtype) if enc_acts[i] is not None else None
        if model == "GCN":
            W, b = P(pre_n + "linear.weight", L.linear.weight), P(pre_n + "linear.bias", L.linear.bias)
            pre = Agg.apply(st(h @ W.t() + b), r, c, v, N)
            with torch.no_grad():
                mk = relu_mask(pre, tst, tau)
            h = st(pre * mk)
        elif model == "HGCN":
            W, b = P(pre_n + "linear.weight", L.linear.weight), P(pre_n + "linear.bias", L.linear.bias)
            s = Agg.apply(h @ W.t() + b, r, c, v, N)
            with torch.no_grad():
                mk = relu_mask(s, tst, tau)
            g = torch.sigmoid(h @ L.kernel_gate.to(dtype) + L.bias_gate.to(dtype))
            h = g * (s * mk) + (1.0 - g) * h
        else:
            Ws = torch.stack([P(pre_n + "attention_%d.W" % j, a.W)
                              for j, a in enumerate(L.attentions)])
            As = torch.stack([P(pre_n + "attention_%d.a" % j, a.a)
                              for j, a in enumerate(L.attentions)])
            h = gat_layer(h, Ws, As, er, ec, 0.2, True, tested=tst, tau=tau, store=store)
    if model == "HGCN":
        L = m.decoder.cls
        W, b = P("decoder.cls.linear.weight", L.linear.weight), P("decoder.cls.linear.bias",
                                                                   L.linear.bias)
        s = Agg.apply(h @ W.t() + b, r, c, v, N)
        g = torch.sigmoid(h @ L.kernel_gate.to(dtype) + L.bias_gate.to(dtype))
        h = g * s + (1.0 - g) * h
    else:
        for i, L in enumerate(m.decoder.cls):
            pre_n = "decoder.cls.%d." % i
            W, b = P(pre_n + "linear.weight", L.linear.weight), P(pre_n + "linear.bias", L.linear.bias)
            h = st(h @ W.t() + b)
            if i < 2:
                with torch.no_grad():
                    mk = relu_mask(h, dec_acts[i].to(dtype), tau)
                h = h * mk
    o64 = outputs.detach().double().requires_grad_(True)
    margin_loss(o64, *ix, t, k).backward()
    cot = o64.grad
    if store is not None:
        cot = cot.to(torch.bfloat16).double()  # as the bf16 outputs receive it
    h.backward(cot.to(dtype))
    return {n: q.grad for n, q in p64.items()}, h.detach()
