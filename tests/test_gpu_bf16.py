"""bf16 feature storage (cfg-5) on the HIP path (run on an MI355X).

Tolerances: the kernels read bf16 rows, compute in fp32 and round the result once.  So
  * with an fp32 output they match the fp64 aggregation of the SAME bf16 inputs to fp32
    accumulation error (<= 1e-5 norm-relative);
  * their bf16 output is bit-identical to torch's round-to-nearest-even of that fp32 output;
  * against the fp32 reference path (fp32 inputs) the stated bf16 tolerance is 1e-2
    norm-relative.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import rel_err

pytestmark = pytest.mark.gpu
TOL_BF16 = 1e-2
TOL_ACC = 1e-5


def _graph(rng, n, nnz, hub=False):
    r = rng.integers(0, n, nnz)
    c = rng.integers(0, n, nnz)
    if hub:  # one row with far more than 64 neighbours
        r = np.concatenate([r, np.zeros(300, dtype=r.dtype)])
        c = np.concatenate([c, rng.integers(0, n, 300)])
    v = rng.standard_normal(r.size).astype(np.float32)
    return r, c, v


def _csr(r, c, v, n, dev):
    from gnnea.graph import DeviceCSR
    return DeviceCSR.from_coo(torch.from_numpy(r).to(dev), torch.from_numpy(c).to(dev),
                              torch.from_numpy(v).to(dev), n, n)


def _agg64(r, c, v, n, x64):
    y = np.zeros((n, x64.shape[1]))
    np.add.at(y, r, v[:, None].astype(np.float64) * x64[c])
    return y


@pytest.mark.parametrize("D", [4, 75 * 4, 300, 302, 1024])
@pytest.mark.parametrize("hub", [False, True])
def test_spmm_bf16_vs_fp64(device, D, hub):
    from gnnea import ops
    rng = np.random.default_rng(D + hub)
    n = 700
    r, c, v = _graph(rng, n, 6000, hub)
    csr = _csr(r, c, v, n, device)
    x = torch.from_numpy(rng.standard_normal((n, D)).astype(np.float32)).to(device)
    xb = x.to(torch.bfloat16)
    y32 = ops.spmm(csr, xb, out_dtype=torch.float32)
    assert y32.dtype == torch.float32
    ref = _agg64(r, c, v, n, xb.float().cpu().double().numpy())
    assert rel_err(y32.cpu(), ref) < TOL_ACC
    yb = ops.spmm(csr, xb)
    assert yb.dtype == torch.bfloat16
    assert torch.equal(yb.view(torch.int16), y32.to(torch.bfloat16).view(torch.int16))
    ref32 = _agg64(r, c, v, n, x.cpu().double().numpy())
    assert rel_err(yb.float().cpu(), ref32) < TOL_BF16


@pytest.mark.parametrize("act", ["relu", "tanh"])
def test_spmm_bf16_act_and_beta(device, act):
    from gnnea import _lib, ops
    rng = np.random.default_rng(3)
    n, D = 500, 300
    r, c, v = _graph(rng, n, 4000)
    csr = _csr(r, c, v, n, device)
    xb = torch.from_numpy(rng.standard_normal((n, D)).astype(np.float32)).to(device).bfloat16()
    code = _lib.GNNEA_ACT_RELU if act == "relu" else _lib.GNNEA_ACT_TANH
    fn = torch.relu if act == "relu" else torch.tanh
    base = _agg64(r, c, v, n, xb.float().cpu().double().numpy())
    y = ops.spmm(csr, xb, act=code, out_dtype=torch.float32)
    assert rel_err(y.cpu(), fn(torch.from_numpy(base))) < TOL_ACC
    # beta: out = act(A x + beta * out), out fp32 (gradient partials)
    prev = torch.from_numpy(rng.standard_normal((n, D)).astype(np.float32)).to(device)
    out = prev.clone()
    ops.spmm(csr, xb, act=code, out=out, beta=0.5)
    want = fn(torch.from_numpy(base + 0.5 * prev.cpu().double().numpy()))
    assert rel_err(out.cpu(), want) < TOL_ACC


def test_aggregate_bf16_autograd(device):
    from gnnea import ops
    rng = np.random.default_rng(5)
    n, D = 600, 300
    r, c, v = _graph(rng, n, 5000)
    idx = torch.from_numpy(np.stack([r, c]).astype(np.int64))
    adj = torch.sparse_coo_tensor(idx, torch.from_numpy(v), (n, n)).to(device)
    x = torch.from_numpy(rng.standard_normal((n, D)).astype(np.float32))
    R = torch.from_numpy(rng.standard_normal((n, D)).astype(np.float32))
    xb = x.to(device).bfloat16().requires_grad_(True)
    y = ops.aggregate(adj, xb, F.relu)
    assert y.dtype == torch.bfloat16
    (y.float() * R.to(device)).sum().backward()
    assert xb.grad.dtype == torch.bfloat16
    # reference at the bf16-rounded input: a ReLU boundary flipped by input rounding is a
    # property of the input precision, not of the kernels
    xo = xb.detach().float().cpu().double().requires_grad_(True)
    yo = torch.relu(torch.sparse_coo_tensor(idx, torch.from_numpy(v).double(), (n, n)) @ xo)
    (yo * R.double()).sum().backward()
    assert rel_err(y.detach().float().cpu(), yo.detach()) < TOL_BF16
    assert rel_err(xb.grad.float().cpu(), xo.grad) < 2 * TOL_BF16


def test_highway_bf16(device):
    from gnnea import ops
    rng = np.random.default_rng(9)
    n, D = 400, 300
    r, c, v = _graph(rng, n, 3000)
    idx = torch.from_numpy(np.stack([r, c]).astype(np.int64))
    adj = torch.sparse_coo_tensor(idx, torch.from_numpy(v), (n, n)).to(device)
    f = lambda *s: torch.from_numpy(rng.standard_normal(s).astype(np.float32))
    hidden, gate_pre, resid, bias, R = f(n, D), f(n, D), f(n, D), f(D), f(n, D)
    hb = hidden.to(device).bfloat16().requires_grad_(True)
    gb = gate_pre.to(device).bfloat16().requires_grad_(True)
    rb = resid.to(device).bfloat16().requires_grad_(True)
    y = ops.highway(adj, hb, gb, rb, bias.to(device), F.relu)
    assert y.dtype == torch.bfloat16
    (y.float() * R.to(device)).sum().backward()
    A = torch.sparse_coo_tensor(idx, torch.from_numpy(v).double(), (n, n))
    ho, go, ro = (t.detach().float().cpu().double().requires_grad_(True) for t in (hb, gb, rb))
    s = torch.relu(A @ ho)
    g = torch.sigmoid(go + bias.double())
    yo = g * s + (1 - g) * ro
    (yo * R.double()).sum().backward()
    assert rel_err(y.detach().float().cpu(), yo.detach()) < TOL_BF16
    for got, want in ((hb.grad, ho.grad), (gb.grad, go.grad), (rb.grad, ro.grad)):
        assert got.dtype == torch.bfloat16
        assert rel_err(got.float().cpu(), want) < 2 * TOL_BF16


def test_bf16_rejects_misaligned_gracefully(device):
    """Odd strides take the scalar path (no 8-B vector loads) and still agree."""
    from gnnea import ops
    rng = np.random.default_rng(11)
    n, D = 300, 300
    r, c, v = _graph(rng, n, 2000)
    csr = _csr(r, c, v, n, device)
    big = torch.from_numpy(rng.standard_normal((n, D + 3)).astype(np.float32)).to(device)
    xb = big.bfloat16()[:, 1:D + 1]  # row stride D + 3, offset 2 bytes: scalar path
    y = ops.spmm(csr, xb, out_dtype=torch.float32)
    ref = _agg64(r, c, v, n, xb.float().cpu().double().numpy())
    assert rel_err(y.cpu(), ref) < TOL_ACC


@pytest.mark.parametrize("shape", [(1, 1, 1), (37, 300, 300), (300, 75, 300), (513, 600, 300),
                                   (300, 300, 20000), (5, 300, 7), (2048, 300, 300)])
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gemm_bf16_vs_fp64(device, shape, ta, tb):
    from gnnea import ops
    M, N, K = shape
    rng = np.random.default_rng(M + N + K + 10 * ta + tb)
    a = torch.from_numpy(rng.standard_normal((K, M) if ta else (M, K)).astype(np.float32))
    b = torch.from_numpy(rng.standard_normal((N, K) if tb else (K, N)).astype(np.float32))
    bias = torch.from_numpy(rng.standard_normal(N).astype(np.float32))
    ab, bb = a.to(device).bfloat16(), b.to(device).bfloat16()
    y32 = ops.gemm(ab, bb, bool(ta), bool(tb), bias=bias.to(device), out_dtype=torch.float32)
    a64, b64 = ab.float().cpu().double().numpy(), bb.float().cpu().double().numpy()
    ref = (a64.T if ta else a64) @ (b64.T if tb else b64) + bias.double().numpy()
    assert rel_err(y32.cpu(), ref) < TOL_ACC
    yb = ops.gemm(ab, bb, bool(ta), bool(tb), bias=bias.to(device))
    assert yb.dtype == torch.bfloat16
    assert torch.equal(yb.view(torch.int16), y32.to(torch.bfloat16).view(torch.int16))


@pytest.mark.parametrize("M,N,K", [(70001, 300, 300), (65536, 256, 256), (131077, 600, 300),
                                   (66000, 200, 64), (65600, 300, 30), (65536, 164, 290),
                                   (66000, 320, 320), (65601, 300, 298)])
@pytest.mark.parametrize("tb", [0, 1])
@pytest.mark.parametrize("wres", ["1", "0"])
def test_gemm_bf16_pipelined_vs_fp64(device, monkeypatch, M, N, K, tb, wres):
    """The tall projection form (M >= 64K): with K in (288, 320] and N % 4 == 0 on
    k_gemm_bf16w (the weight tile resident in LDS, activations streamed into registers, the
    transposed product stored from registers; wres=1), otherwise -- and with
    GNNEA_BF16_WRES=0 -- on k_gemm_bf16p (persistent LDS-DMA ring, the bias joined exactly as
    three bf16 terms against A's ones, 4-B / 16-B A granules).  fp32 and bf16 outputs vs fp64 of
    the same bf16 operands, ragged M / N, K tails inside a 16-B chunk (290, 298), the slice-major
    bf16 output and beta accumulation."""
    from gnnea import ops
    monkeypatch.setenv("GNNEA_BF16_WRES", wres)
    rng = np.random.default_rng(M + N + K + tb)
    a = torch.from_numpy(rng.standard_normal((M, K)).astype(np.float32)).to(device).bfloat16()
    b = torch.from_numpy(rng.standard_normal((N, K) if tb else (K, N)).astype(np.float32))
    bb = b.to(device).bfloat16()
    bias = torch.from_numpy(rng.standard_normal(N).astype(np.float32)).to(device)
    ref = a.double() @ (bb.double().t() if tb else bb.double()) + bias.double()
    y32 = ops.gemm(a, bb, False, bool(tb), bias=bias, out_dtype=torch.float32)
    assert rel_err(y32.cpu(), ref.cpu()) < TOL_ACC
    yb = ops.gemm(a, bb, False, bool(tb), bias=bias)
    assert torch.equal(yb.view(torch.int16), y32.to(torch.bfloat16).view(torch.int16))
    y0 = ops.gemm(a, bb, False, bool(tb), out_dtype=torch.float32)  # no bias
    assert rel_err(y0.cpu(), (ref - bias.double()).cpu()) < TOL_ACC
    prev = torch.from_numpy(rng.standard_normal((M, N)).astype(np.float32)).to(device)
    acc = prev.clone()
    ops.gemm(a, bb, False, bool(tb), out=acc, beta=0.5)
    assert rel_err(acc.cpu(), (y0.double() + 0.5 * prev.double()).cpu()) < TOL_ACC
    if N % 4 == 0 and not tb:  # the slice-major bf16 table (gnnea_gemm_sliced_bf16)
        hs = ops.gemm_sliced(a, bb.t().contiguous(), bias)
        W = hs.shape[2]
        for q in range(hs.shape[0]):
            c1 = min(N, (q + 1) * W)
            assert torch.equal(hs[q, :, :c1 - q * W].view(torch.int16),
                               yb[:, q * W:c1].view(torch.int16))


def test_linear_bf16_autograd(device):
    from gnnea import ops
    rng = np.random.default_rng(21)
    n, fin, fout = 1000, 300, 300
    x = torch.from_numpy(rng.standard_normal((n, fin)).astype(np.float32))
    W = torch.from_numpy((rng.standard_normal((fout, fin)) * 0.05).astype(np.float32))
    bvec = torch.from_numpy(rng.standard_normal(fout).astype(np.float32))
    R = torch.from_numpy(rng.standard_normal((n, fout)).astype(np.float32))
    xb, Wb, bb = (t.to(device).bfloat16().requires_grad_(True) for t in (x, W, bvec))
    y = ops.linear(xb, Wb, bb)
    assert y.dtype == torch.bfloat16
    (y.float() * R.to(device)).sum().backward()
    xo, Wo, bo = (t.detach().float().cpu().double().requires_grad_(True) for t in (xb, Wb, bb))
    yo = xo @ Wo.t() + bo
    (yo * R.double()).sum().backward()
    assert rel_err(y.detach().float().cpu(), yo.detach()) < TOL_BF16
    for got, want in ((xb.grad, xo.grad), (Wb.grad, Wo.grad), (bb.grad, bo.grad)):
        assert got.dtype == torch.bfloat16
        assert rel_err(got.float().cpu(), want) < TOL_BF16


def _gat_ref64(r, c, n, H, a, heads, d, alpha):
    """fp64 GAT over given projections H [n, heads*d] (att_layers.py:29-61 per head, concat)."""
    outs = []
    for h in range(heads):
        Hh = H[:, h * d:(h + 1) * d]
        z = Hh[r] @ a[h, :d] + Hh[c] @ a[h, d:]
        e = torch.exp(-F.leaky_relu(z, alpha))
        num = torch.zeros((n, d), dtype=H.dtype).index_add(0, torch.from_numpy(r), e[:, None] * Hh[c])
        den = torch.zeros(n, dtype=H.dtype).index_add(0, torch.from_numpy(r), e)
        outs.append(torch.relu(num / den[:, None]))
    return torch.cat(outs, dim=1)


@pytest.mark.parametrize("heads,d", [(4, 75), (1, 300), (8, 16), (3, 20)])
def test_gat_bf16_vs_fp64(device, heads, d):
    from gnnea import ops
    rng = np.random.default_rng(31 + heads)
    n = 400
    r = rng.integers(0, n, 3000)
    c = rng.integers(0, n, 3000)
    r = np.concatenate([r, np.arange(n), np.zeros(200, dtype=r.dtype)])  # self loops + a hub row
    c = np.concatenate([c, np.arange(n), rng.integers(0, n, 200)])
    # one entry per (i, j), as the reference's adjacency (a dict) has
    pairs = np.unique(np.stack([r, c], axis=1), axis=0)
    r, c = pairs[:, 0].copy(), pairs[:, 1].copy()
    v = np.ones(r.size, dtype=np.float32)
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.stack([r, c]).astype(np.int64)),
                                  torch.from_numpy(v), (n, n)).to(device)
    D = heads * d
    H = torch.from_numpy((rng.standard_normal((n, D)) * 0.5).astype(np.float32))
    A = torch.from_numpy((rng.standard_normal((heads, 2 * d)) * 0.3).astype(np.float32))
    R = torch.from_numpy(rng.standard_normal((n, D)).astype(np.float32))
    Hb = H.to(device).bfloat16().requires_grad_(True)
    At = A.to(device).requires_grad_(True)
    y = ops.gat(adj, Hb, At, heads, d, 0.2, F.relu)
    assert y.dtype == torch.bfloat16
    (y.float() * R.to(device)).sum().backward()
    Ho = Hb.detach().float().cpu().double().requires_grad_(True)
    Ao = A.double().requires_grad_(True)
    yo = _gat_ref64(r, c, n, Ho, Ao, heads, d, 0.2)
    (yo * R.double()).sum().backward()
    assert rel_err(y.detach().float().cpu(), yo.detach()) < TOL_BF16
    assert Hb.grad.dtype == torch.bfloat16
    assert rel_err(Hb.grad.float().cpu(), Ho.grad) < 2 * TOL_BF16
    assert rel_err(At.grad.cpu(), Ao.grad) < 2 * TOL_BF16
    # the same storage in fp32 gives the fp32 path's answer to bf16 rounding
    y32 = ops.gat(adj, Hb.detach().float(), At.detach(), heads, d, 0.2, F.relu)
    assert rel_err(y.detach().float().cpu(), y32.cpu()) < TOL_BF16


@pytest.mark.parametrize("model", ["GCN", "GAT", "HGCN"])
def test_model_bf16_end_to_end(golden, device, model):
    """A whole drop-in encoder/decoder converted with .bfloat16() runs forward, margin loss and
    backward on the bf16 kernels and stays within the bf16 tolerance of the fp32 model."""
    from models.decoders import model2decoder
    from models.encoders import model2encoder
    from gnnea.margin import margin_loss
    from test_dropin_cpu import make_args
    g = golden("graph_cfg1")
    a = make_args(model)
    a.cuda, a.device = 0, device
    torch.manual_seed(10086)
    enc = model2encoder[model](a).to(device)
    dec = model2decoder[model](a).to(device)
    idx = torch.from_numpy(np.stack([g["row"], g["col"]]).astype(np.int64))
    adj = torch.sparse_coo_tensor(idx, torch.from_numpy(g["val"]), (2000, 2000)).to(device)
    x = torch.from_numpy(g["X"]).to(device)
    rng = np.random.default_rng(0)
    t, k = 200, 5
    left, right = rng.integers(0, 1000, t), rng.integers(1000, 2000, t)
    negs = [rng.integers(0, 2000, t * k) for _ in range(4)]

    def run(dtype):
        e, d = enc.to(dtype), dec.to(dtype)
        for m in (e, d):
            for mod in m.modules():  # HighWay's plain-tensor gate weights follow the model
                if hasattr(mod, "kernel_gate") and torch.is_tensor(mod.kernel_gate):
                    mod.kernel_gate = mod.kernel_gate.to(dtype)
        e.zero_grad()
        d.zero_grad()
        out = d.decode(e.encode(x.to(dtype), adj), adj)
        loss = margin_loss(out, np.repeat(left, 1), right, np.repeat(left, k), negs[0],
                           negs[1], np.repeat(right, k), t, k)
        loss.backward()
        grads = [p.grad.float().cpu().clone() for p in list(e.parameters()) + list(d.parameters())]
        return out.detach().float().cpu(), float(loss), grads

    out32, loss32, g32 = run(torch.float32)
    outb, lossb, gb = run(torch.bfloat16)
    assert rel_err(outb, out32) < 3 * TOL_BF16
    assert abs(lossb - loss32) <= 3 * TOL_BF16 * abs(loss32)
    # the margin loss's gradient is a sum of sign(u - v) terms: bf16 rounding of the embeddings
    # flips the signs of near-zero differences, so the bf16 gradients are compared by direction
    # (measured cosines 0.85-0.99); the last decoder bias has an analytically zero gradient (the
    # loss depends on differences of rows only) and is skipped: both runs hold rounding noise
    top = max(float(p.norm()) for p in g32)
    for p16, p32 in zip(gb, g32):
        assert torch.isfinite(p16).all()
        if float(p32.norm()) < 1e-4 * top:
            continue
        cos = float(torch.nn.functional.cosine_similarity(p16.flatten().double(),
                                                          p32.flatten().double(), dim=0))
        assert cos > 0.8, cos


@pytest.mark.parametrize("M,N,K", [(300, 300, 4_000_000), (300, 300, 1_000_003), (152, 300, 4099),
                                   (300, 168, 999), (8, 8, 128), (320, 320, 100_000),
                                   (300, 300, 20_000)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gemm_weight_grad_full_width(device, M, N, K, dt):
    """dW = Aᵀ·B (A [K][M], B [K][N]) on the whole-width split-K kernel (gemm_ta.hip: all M
    rows x a 160-column half per workgroup, operands read transposed from LDS): fp32 through the
    three-way bf16 split (fp32-level error), bf16 operands with fp32 / bf16 output; a column
    block of a wider buffer as A (the fused HighWay layer's dh = P[:, :D]), bias and beta, K tails
    inside a 32-row step, the table's last row ending inside a 16-B chunk (bf16 M = 300)."""
    from gnnea import ops
    torch.manual_seed(M + N + K)
    if K >= 1_000_000 and dt == torch.float32:
        K //= 2  # the cfg-4 row count
    wide = torch.randn(K, M + 4, device=device).to(dt)
    a = wide[:, :M]
    b = torch.randn(K, N, device=device).to(dt)
    bias = torch.randn(N, device=device)
    ref = (a.double().t() @ b.double()).cpu()
    tol = 1e-5 if dt == torch.float32 else TOL_ACC
    y = ops.gemm(a, b, trans_a=True, out_dtype=torch.float32)
    assert rel_err(y.cpu(), ref) < tol
    yb = ops.gemm(a, b, trans_a=True, bias=bias, out_dtype=torch.float32)
    assert rel_err(yb.cpu(), ref + bias.double().cpu()) < tol
    prev = torch.randn(M, N, device=device)
    acc = prev.clone()
    ops.gemm(a, b, trans_a=True, out=acc, beta=0.5)
    assert rel_err(acc.cpu(), ref + 0.5 * prev.double().cpu()) < tol
    if dt == torch.bfloat16:
        y16 = ops.gemm(a, b, trans_a=True)
        assert y16.dtype == torch.bfloat16
        assert torch.equal(y16.view(torch.int16), y.to(torch.bfloat16).view(torch.int16))
