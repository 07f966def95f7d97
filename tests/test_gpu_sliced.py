"""Slice-major aggregation path (gnnea_spmm_sliced_f32, gnnea_gemm_sliced_f32,
gnnea_slice_pack_f32, gnnea_act_bwd_sliced_f32) vs the CPU oracle and the row-major path.

The sliced kernel sums each row's neighbours in four interleaved partial sums, so it agrees with
the oracle (fp64) and the row-major kernel (CSR-order chain) to fp32 rounding: norm-relative
1e-4, the fp32 tolerance of SURVEY.md §8c.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import rel_err

pytestmark = pytest.mark.gpu
TOL32 = 1e-4


def _unslice(hs, D):
    S, n, w = hs.shape
    return hs.permute(1, 0, 2).reshape(n, S * w)[:, :D]


def _graph(rng, n, nnz, device, hub=True):
    from gnnea.graph import DeviceCSR
    r = rng.integers(0, n, nnz)
    c = rng.integers(0, n, nnz)
    keep = (r > 3) & (r < n - 3)  # empty rows at both ends
    r, c = r[keep], c[keep]
    if hub:  # one row with > 64 and > 128 neighbours (several 64-edge batches)
        r = np.concatenate([r, np.full(300, 17)])
        c = np.concatenate([c, rng.integers(0, n, 300)])
    v = rng.standard_normal(r.size).astype(np.float32)
    csr = DeviceCSR.from_coo(torch.from_numpy(r).to(device), torch.from_numpy(c).to(device),
                             torch.from_numpy(v).to(device), n, n)
    return r, c, v, csr


@pytest.mark.parametrize("D", [4, 60, 68, 128, 132, 300, 512])
def test_spmm_sliced_vs_oracle(device, D):
    from gnnea import ops
    from oracle.gnn import coo_aggregate
    rng = np.random.default_rng(D + 11)
    n = 900
    r, c, v, csr = _graph(rng, n, 8000, device)
    x = torch.from_numpy(rng.standard_normal((n, D)).astype(np.float32)).to(device)
    xs = ops.slice_pack(x)
    assert xs.shape == ((D + 63) // 64, n, 64)
    assert torch.equal(_unslice(xs, D), x)
    for act, fn in ((0, lambda t: t), (1, torch.relu), (4, torch.sigmoid), (5, torch.tanh)):
        y = ops.spmm_sliced(csr, xs, D, act).cpu()
        ref = fn(coo_aggregate(r, c, v, n, x.cpu().double()))
        assert rel_err(y, ref) < TOL32, (D, act)
        assert rel_err(y, ops.spmm(csr, x, act).cpu()) < TOL32
    assert torch.all(ops.spmm_sliced(csr, xs, D)[:4].cpu() == 0)


@pytest.mark.parametrize("D", [4, 60, 68, 128, 132, 300])
def test_spmm_sliced64_bf16_vs_oracle(device, D):
    """bf16 over 64-column slices (gnnea_spmm_sliced64_bf16, 128-B row pieces): vs the fp64
    oracle on the bf16-rounded table (fp32 sums, one bf16 rounding of the output: 1e-2; fp32
    output 1e-4) and vs the 128-column bf16 kernel on the same table."""
    from gnnea import ops
    from oracle.gnn import coo_aggregate
    rng = np.random.default_rng(D + 29)
    n = 900
    r, c, v, csr = _graph(rng, n, 8000, device)
    x = torch.from_numpy(rng.standard_normal((n, D)).astype(np.float32)).to(device)
    xb = x.to(torch.bfloat16)
    xs = ops.slice_pack64(xb)
    assert xs.shape == ((D + 63) // 64, n, 64)
    for act, fn in ((0, lambda t: t), (1, torch.relu), (5, torch.tanh)):
        ref = fn(coo_aggregate(r, c, v, n, xb.float().cpu().double()))
        y32 = ops.spmm_sliced64(csr, xs, D, act, out_dtype=torch.float32).cpu()
        assert rel_err(y32, ref) < TOL32, (D, act)
        y16 = ops.spmm_sliced64(csr, xs, D, act).cpu()
        assert y16.dtype == torch.bfloat16 and rel_err(y16.float(), ref) < 1e-2, (D, act)
        if D % 4 == 0 and D >= 128:
            y128 = ops.spmm_sliced(csr, ops.slice_pack(xb), D, act, out_dtype=torch.float32)
            assert rel_err(y32, y128.cpu()) < TOL32
    assert torch.all(ops.spmm_sliced64(csr, xs, D)[:4].float().cpu() == 0)


def test_slice_pack_strided_and_rejects(device):
    from gnnea import ops
    big = torch.randn(333, 320, device=device)
    x = big[:, :300]  # row stride 320
    assert torch.equal(_unslice(ops.slice_pack(x), 300), x)
    with pytest.raises(Exception):  # D % 4 != 0 has no slice-major form
        ops.slice_pack(torch.randn(10, 30, device=device)[:, :29])


def test_spmm_sliced_output_column_block(device):
    """out may be a column block of a wider buffer (the HighWay layer's [dh | dgate])."""
    from gnnea import ops
    rng = np.random.default_rng(3)
    n, D = 500, 300
    _, _, _, csr = _graph(rng, n, 4000, device)
    x = torch.randn(n, D, device=device)
    P = torch.full((n, 2 * D), 7.0, device=device)
    ops.spmm_sliced(csr, ops.slice_pack(x), D, 1, out=P[:, :D])
    assert rel_err(P[:, :D].cpu(), ops.spmm(csr, x, 1).cpu()) < TOL32
    assert torch.all(P[:, D:] == 7.0)


@pytest.mark.parametrize("M,N,K", [(1000, 300, 300), (777, 128, 64), (64, 68, 300),
                                   (4097, 300, 17), (70001, 300, 300), (65600, 600, 296)])
def test_gemm_sliced_vs_fp64(device, M, N, K):
    from gnnea import ops
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=device)
    W = torch.randn(N, K, device=device)
    b = torch.randn(N, device=device)
    hs = ops.gemm_sliced(x, W, b)
    ref = x.double().cpu() @ W.double().cpu().t() + b.double().cpu()
    assert rel_err(_unslice(hs, N).cpu(), ref) < TOL32
    # the same bits as the row-major GEMM (same tiles, only the store address differs)
    assert torch.equal(_unslice(hs, N), ops.gemm(x, W, trans_b=True, bias=b))


@pytest.mark.parametrize("act,fn", [(1, torch.relu), (2, F.elu), (5, torch.tanh)])
def test_act_bwd_sliced(device, act, fn):
    from gnnea import ops
    y = fn(torch.randn(300, 132, device=device))
    dy = torch.randn(300, 132, device=device)
    gs = ops.act_bwd_sliced(dy, y, act)
    assert torch.equal(_unslice(gs, 132), ops.act_bwd(dy, y, act))


@pytest.mark.parametrize("D", [4, 68, 300])
def test_relu_sign_bits_sliced(device, D):
    """spmm_sliced_m: the relu aggregation bit-identical to spmm_sliced, its sign bits = (y > 0)
    (byte q: elements 4 q .. 4 q + 3); act_bwd_sliced_bits from them = act_bwd_sliced from y,
    bit for bit (the GCN layer's fp32 relu backward keeps only the bits)."""
    from gnnea import _lib, ops
    rng = np.random.default_rng(12)
    n = 1500
    _, _, _, csr = _graph(rng, n, 12000, device)
    xs = ops.slice_pack(torch.randn(n, D, device=device))
    y, m = ops.spmm_sliced_m(csr, xs, D)
    assert torch.equal(y, ops.spmm_sliced(csr, xs, D, _lib.GNNEA_ACT_RELU))
    cols = torch.arange(D, device=device)
    bits = (m[:, cols // 4] >> (cols % 4).to(torch.uint8)) & 1
    assert torch.equal(bits.bool(), y > 0)
    dy = torch.randn(n, D, device=device)
    assert torch.equal(_unslice(ops.act_bwd_sliced_bits(dy, m, D), D),
                       _unslice(ops.act_bwd_sliced(dy, y, _lib.GNNEA_ACT_RELU), D))


def test_gcn_layer_sliced_vs_oracle(device, monkeypatch):
    """GraphConvolution through GCNLayerFn (hidden written slice-major by the GEMM, sliced
    aggregation, sliced backward) vs the fp64 oracle: output, dx, dW, db."""
    from gnnea import ops
    from layers.layers import GraphConvolution
    from oracle.gnn import gcn_layer, layer_with_grads
    monkeypatch.setattr(ops, "INFINITY_CACHE_BYTES", 0)  # force the sliced path at test size
    rng = np.random.default_rng(5)
    n = 1200
    r, c, v, csr = _graph(rng, n, 10000, device)
    idx = torch.from_numpy(np.stack([r, c]).astype(np.int64))
    adj = torch.sparse_coo_tensor(idx, torch.from_numpy(v), (n, n)).to(device)
    torch.manual_seed(0)
    layer = GraphConvolution(300, 300, 0.0, F.relu, True).to(device)
    x = torch.from_numpy(rng.standard_normal((n, 300)).astype(np.float32) * 0.1).to(device)
    R = torch.randn(n, 300, device=device)
    calls = []
    orig = ops.gemm_sliced

    def spy(*a, **k):
        calls.append(1)
        return orig(*a, **k)
    monkeypatch.setattr(ops, "gemm_sliced", spy)
    xx = x.clone().requires_grad_(True)
    out, _ = layer((xx, adj))
    (out * R).sum().backward()
    assert calls, "the fused sliced layer was not used"
    W = layer.linear.weight.detach().cpu().double()
    b = layer.linear.bias.detach().cpu().double()
    o_ref, dx_ref, (dW_ref, db_ref) = layer_with_grads(
        lambda xv, Wv, bv: gcn_layer(xv, Wv, bv, r, c, v), x.cpu().double(), [W, b],
        R.cpu().double())
    assert rel_err(out.detach().cpu(), o_ref) < TOL32
    assert rel_err(xx.grad.cpu(), dx_ref) < TOL32
    assert rel_err(layer.linear.weight.grad.cpu(), dW_ref) < TOL32
    assert rel_err(layer.linear.bias.grad.cpu(), db_ref) < TOL32


def test_aggregate_sliced_matches_rowmajor_two_kg(device, monkeypatch):
    """Two-KG graph above the Infinity Cache: AggregateFn takes the pack + sliced path per
    diagonal block; forward and backward agree with the row-major kernels."""
    from gnnea import ops, synth
    from gnnea.graph import DeviceCSR
    n = 300000
    tr = synth.kg_pair_triples(n, 3 * n, 500, seed=4)
    r, c, v = synth.adjacency_coo(tr, 2 * n, reference_order=False)
    csr = DeviceCSR.from_coo(torch.from_numpy(r).to(device), torch.from_numpy(c).to(device),
                             torch.from_numpy(v).to(device), 2 * n, 2 * n)
    assert csr.row_blocks() == [(0, n), (n, 2 * n)]
    h = torch.randn(2 * n, 128, device=device)
    assert ops.use_sliced(2 * n, 128, torch.float32)
    dy = torch.randn(2 * n, 128, device=device)

    def run():  # tanh: relu's derivative flips on pre-activations within rounding of 0
        hh = h.clone().requires_grad_(True)
        y = ops.AggregateFn.apply(hh, csr, 5)
        (g,) = torch.autograd.grad(y, (hh,), dy)
        return y.detach(), g
    y_s, g_s = run()
    monkeypatch.setattr(ops, "SLICED", False)
    y_r, g_r = run()
    assert rel_err(y_s.cpu(), y_r.cpu()) < TOL32
    assert rel_err(g_s.cpu(), g_r.cpu()) < TOL32


@pytest.mark.parametrize("act", [F.relu, torch.tanh])
def test_highway_layer_sliced_matches_rowmajor(device, monkeypatch, act):
    """HighWayGraphConvolution through the fused layer with the projection Z = x·[Wᵀ | K_g]
    written slice-major (hidden and gate_pre in ONE table), the sliced HighWay SpMM, dS written
    slice-major and the transposed sliced aggregation, against the row-major fused layer:
    output, dx, dW, db."""
    from gnnea import ops
    from layers.layers import HighWayGraphConvolution
    rng = np.random.default_rng(8)
    n = 1500
    r, c, v, csr = _graph(rng, n, 12000, device)
    idx = torch.from_numpy(np.stack([r, c]).astype(np.int64))
    adj = torch.sparse_coo_tensor(idx, torch.from_numpy(v), (n, n)).to(device)
    torch.manual_seed(1)
    layer = HighWayGraphConvolution(300, 300, 0.0, act, True, 0, device).to(device)
    layer.bias_gate = torch.randn(300, device=device) * 0.1
    x = torch.from_numpy(rng.standard_normal((n, 300)).astype(np.float32) * 0.1).to(device)
    R = torch.randn(n, 300, device=device)

    def run():
        layer.zero_grad()
        xx = x.clone().requires_grad_(True)
        out, _ = layer((xx, adj))
        (out * R).sum().backward()
        return [out.detach(), xx.grad, layer.linear.weight.grad.clone(),
                layer.linear.bias.grad.clone()]
    calls = []
    orig, orig_m = ops.highway_fwd_sliced, ops.highway_fwd_sliced_m

    def spy(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    def spy_m(*a, **k):  # (relu: the sign-mask form, S not stored)
        calls.append(2)
        return orig_m(*a, **k)
    monkeypatch.setattr(ops, "highway_fwd_sliced", spy)
    monkeypatch.setattr(ops, "highway_fwd_sliced_m", spy_m)
    monkeypatch.setattr(ops, "INFINITY_CACHE_BYTES", 0)  # force the sliced path at test size
    got = run()
    assert calls, "the sliced HighWay layer was not used"
    monkeypatch.setattr(ops, "SLICED", False)
    ref = run()
    assert len(calls) == 1
    for g, w in zip(got, ref):
        assert rel_err(g.cpu(), w.cpu()) < TOL32

@pytest.mark.parametrize("act", [1, 0])
def test_highway_layer_fn_sliced_without_s(device, monkeypatch, act):
    """HighwayLayerFn on the sliced path with relu (code 1: sign mask saved, S not stored) and
    identity (code 0: nothing but the output) against the torch fp32 formula
    out = g S + (1 - g) x, S = act(A (x Wᵀ + b)), g = sigmoid(x K_g + b_g): output and the
    gradients of x (through the gate too), W and b."""
    from gnnea import _lib, ops
    rng = np.random.default_rng(11)
    n, D = 1300, 300
    r, c, v, csr = _graph(rng, n, 10000, device)
    A = torch.sparse_coo_tensor(torch.from_numpy(np.stack([r, c]).astype(np.int64)),
                                torch.from_numpy(v), (n, n)).to(device).coalesce()
    torch.manual_seed(3)
    x0 = torch.randn(n, D, device=device) * 0.1
    W0 = torch.randn(D, D, device=device) * 0.05
    b0 = torch.randn(D, device=device) * 0.1
    K0 = torch.randn(D, D, device=device) * 0.05
    bg = torch.randn(D, device=device) * 0.1
    R = torch.randn(n, D, device=device)
    code = _lib.GNNEA_ACT_RELU if act else _lib.GNNEA_ACT_IDENTITY
    monkeypatch.setattr(ops, "INFINITY_CACHE_BYTES", 0)
    agg = ops.LocalAgg(csr)
    assert agg.sliced_ok(D, torch.float32)
    leaves = [t.clone().requires_grad_(True) for t in (x0, W0, b0, K0)]
    out = ops.HighwayLayerFn.apply(leaves[0], leaves[1], leaves[2], leaves[3], bg, agg, code)
    (out * R).sum().backward()
    ref_leaves = [t.clone().requires_grad_(True) for t in (x0, W0, b0, K0)]
    x, W, b, K = ref_leaves
    S = torch.sparse.mm(A, x @ W.t() + b)
    S = torch.relu(S) if act else S
    g = torch.sigmoid(x @ K + bg)
    ref = g * S + (1.0 - g) * x
    (ref * R).sum().backward()
    assert rel_err(out.detach().cpu(), ref.detach().cpu()) < TOL32
    for got, want in zip(leaves[:3], ref_leaves[:3]):  # (K_g is a constant, as in the reference)
        assert rel_err(got.grad.cpu(), want.grad.cpu()) < TOL32



def test_distadj_world1_takes_sliced_layers(device, monkeypatch):
    """A DistAdj whose rank aggregates without exchange (world 1: the whole graph) runs the
    fused slice-major GCN and HighWay layers; results match the row-major layers on the
    reference sparse adjacency."""
    from gnnea import ops, synth
    from gnnea.dist_graph import DistAdj
    from layers.layers import GraphConvolution, HighWayGraphConvolution
    n, t = 600, 2400
    tr = synth.kg_pair_triples(n, t, 30)
    dadj = DistAdj.from_triples(tr, n, t, 0, 1, device)
    R, C, V = synth.adjacency_coo(tr, 2 * n, reference_order=False)
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.stack([R, C])).long(),
                                  torch.from_numpy(V), (2 * n, 2 * n)).to(device)
    torch.manual_seed(2)
    l1 = GraphConvolution(300, 300, 0.0, F.relu, True).to(device)
    l2 = HighWayGraphConvolution(300, 300, 0.0, F.relu, True, 0, device).to(device)
    x = torch.from_numpy(synth.features(2 * n, 300, seed=4)).to(device)
    Rw = torch.randn(2 * n, 300, device=device)
    used = []
    for name in ("gemm_sliced", "highway_fwd_sliced", "highway_fwd_sliced_m"):
        orig = getattr(ops, name)
        monkeypatch.setattr(ops, name, (lambda f, nm: lambda *a, **k: (used.append(nm),
                                                                        f(*a, **k))[1])(orig, name))

    def run(a):
        l1.zero_grad()
        l2.zero_grad()
        xx = x.clone().requires_grad_(True)
        out = l2(l1((xx, a)))[0]
        (out * Rw).sum().backward()
        return [out.detach(), xx.grad] + [p.grad.clone() for p in
                                          list(l1.parameters()) + list(l2.parameters())]
    monkeypatch.setattr(ops, "INFINITY_CACHE_BYTES", 0)
    got = run(dadj)
    assert "gemm_sliced" in used and {"highway_fwd_sliced", "highway_fwd_sliced_m"} & set(used)
    monkeypatch.setattr(ops, "SLICED", False)
    ref = run(adj)
    for g, w in zip(got, ref):
        assert rel_err(g.cpu(), w.cpu()) < TOL32


# ---- bf16 storage: 128-column slices (cfg-5's dtype), fp32 arithmetic ------------------------
TOL_BF16 = 1e-2  # one bf16 rounding of the output (2^-8) plus summation order


@pytest.mark.parametrize("D", [4, 128, 132, 300, 512])
def test_spmm_sliced_bf16_vs_oracle(device, D):
    from gnnea import ops
    from oracle.gnn import coo_aggregate
    rng = np.random.default_rng(D + 23)
    n = 900
    r, c, v, csr = _graph(rng, n, 8000, device)
    xb = torch.from_numpy(rng.standard_normal((n, D)).astype(np.float32)).to(device).bfloat16()
    xs = ops.slice_pack(xb)
    assert xs.dtype == torch.bfloat16 and xs.shape == ((D + 127) // 128, n, 128)
    assert torch.equal(_unslice(xs, D), xb)
    ref32 = coo_aggregate(r, c, v, n, xb.float().cpu().double())
    for act, fn in ((0, lambda t: t), (1, torch.relu), (5, torch.tanh)):
        ref = fn(ref32)
        y32 = ops.spmm_sliced(csr, xs, D, act, out_dtype=torch.float32).cpu()
        assert rel_err(y32, ref) < TOL32, (D, act)  # exact bf16 inputs, fp32 sums
        yb = ops.spmm_sliced(csr, xs, D, act).cpu()
        assert yb.dtype == torch.bfloat16
        assert rel_err(yb.float(), ref) < TOL_BF16, (D, act)
        assert rel_err(yb.float(), ops.spmm(csr, xb, act).float().cpu()) < TOL_BF16


def test_gemm_and_act_bwd_sliced_bf16(device):
    from gnnea import ops
    torch.manual_seed(3)
    x = torch.randn(1000, 300, device=device).bfloat16()
    W = torch.randn(300, 300, device=device).bfloat16()
    b = torch.randn(300, device=device)
    hs = ops.gemm_sliced(x, W, b)
    assert hs.dtype == torch.bfloat16 and hs.shape == (3, 1000, 128)
    assert torch.equal(_unslice(hs, 300), ops.gemm(x, W, trans_b=True, bias=b))
    y = torch.relu(torch.randn(500, 300, device=device)).bfloat16()
    dy = torch.randn(500, 300, device=device).bfloat16()
    gs = ops.act_bwd_sliced(dy, y, 1)
    assert torch.equal(_unslice(gs, 300), ops.act_bwd(dy, y, 1))


def test_gcn_layer_sliced_bf16_matches_rowmajor(device, monkeypatch):
    """A bf16 GraphConvolution through GCNLayerFn (bf16 GEMM writing 128-column slices, sliced
    aggregation and backward) against the row-major bf16 layer."""
    from gnnea import ops
    from layers.layers import GraphConvolution
    rng = np.random.default_rng(12)
    n = 1200
    r, c, v, csr = _graph(rng, n, 10000, device)
    idx = torch.from_numpy(np.stack([r, c]).astype(np.int64))
    adj = torch.sparse_coo_tensor(idx, torch.from_numpy(v), (n, n)).to(device)
    torch.manual_seed(0)
    layer = GraphConvolution(300, 300, 0.0, torch.tanh, True).to(device).bfloat16()
    x = torch.from_numpy(rng.standard_normal((n, 300)).astype(np.float32) * 0.1).to(device)
    x = x.bfloat16()
    R = torch.randn(n, 300, device=device).bfloat16()

    def run():
        layer.zero_grad()
        xx = x.clone().requires_grad_(True)
        out, _ = layer((xx, adj))
        (out.float() * R.float()).sum().backward()
        return [out.detach(), xx.grad, layer.linear.weight.grad.clone(),
                layer.linear.bias.grad.clone()]
    calls = []
    orig = ops.gemm_sliced
    monkeypatch.setattr(ops, "gemm_sliced", lambda *a, **k: (calls.append(1), orig(*a, **k))[1])
    monkeypatch.setattr(ops, "INFINITY_CACHE_BYTES", 0)
    got = run()
    assert calls
    monkeypatch.setattr(ops, "SLICED", False)
    ref = run()
    for g, w in zip(got, ref):
        assert g.dtype == w.dtype
        assert rel_err(g.float().cpu(), w.float().cpu()) < 2e-2


@pytest.mark.parametrize("N,D,dt", [(1, 300, torch.float32), (2_000_001, 300, torch.float32),
                                    (30000, 12, torch.bfloat16), (777, 10, torch.float32),
                                    (100_003, 300, torch.bfloat16), (1001, 302, torch.bfloat16),
                                    (513, 7, torch.bfloat16), (4_000_000, 300, torch.bfloat16)])
def test_colsum_vs_fp64(device, N, D, dt):
    """Bias gradients: streaming column sums (gnnea_colsum_*), also over a column block (bf16
    D = 300: the table's last row ends inside a 16-B granule and takes the element path)."""
    from gnnea import ops
    torch.manual_seed(N)
    t = torch.randn(N, D, device=device).to(dt)
    ref = t.double().sum(0).cpu()
    got = ops.colsum(t)
    assert got.dtype == dt
    tol = 1e-5 if dt == torch.float32 else 1e-2
    assert rel_err(got.float().cpu(), ref) < tol
    if D % 4 == 0 and N < 3_000_000:
        wide = torch.randn(N, 2 * D + 4, device=device).to(dt)
        assert rel_err(ops.colsum(wide[:, :D]).float().cpu(), wide[:, :D].double().sum(0).cpu()) < tol
        # a right-hand block whose last row ends at the buffer's end (bf16 D = 300: the granules
        # cover 304 columns, so the last row must not read past the allocation)
        right = wide[:, D + 4:]
        assert right.data_ptr() + right.shape[1] * right.element_size() == \
            wide.data_ptr() + wide.shape[1] * wide.element_size()
        assert rel_err(ops.colsum(right).float().cpu(), right.double().sum(0).cpu()) < tol


@pytest.mark.parametrize("N,heads,d_head,dt", [
    (4_000_000, 4, 75, torch.bfloat16), (2_000_000, 4, 75, torch.float32),
    (10_007, 1, 300, torch.float32), (10_007, 2, 64, torch.bfloat16), (999, 8, 32, torch.float32),
    (3001, 4, 6, torch.bfloat16), (3001, 3, 50, torch.float32), (1, 4, 75, torch.bfloat16)])
def test_gat_da_pair_vs_fp64(device, N, heads, d_head, dt):
    """Attention-vector gradient pieces out[c] = sum_r ds[r, c // d_head] H[r, c]: one set
    (gnnea_gat_da_*) and both sets in one pass over H (gnnea_gat_da2_*) vs fp64; four heads with
    d_head >= a granule's elements pick a granule's two heads once, the rest read per element."""
    from gnnea import ops
    torch.manual_seed(N + heads)
    D = heads * d_head
    Hm = torch.randn(N, D, device=device).to(dt)
    ds1 = torch.randn(N, heads, device=device)
    ds2 = torch.randn(N, heads, device=device)
    Hd = Hm.double().view(N, heads, d_head)
    ref1 = (Hd * ds1.double()[:, :, None]).sum(0).reshape(-1).cpu()
    ref2 = (Hd * ds2.double()[:, :, None]).sum(0).reshape(-1).cpu()
    tol = 1e-5 if dt == torch.float32 else 1e-2
    p1, p2 = ops.gat_da(Hm, ds1, heads, d_head, ds2)
    assert rel_err(p1.cpu(), ref1) < tol and rel_err(p2.cpu(), ref2) < tol
    q1 = ops.gat_da(Hm, ds1, heads, d_head)
    assert torch.equal(q1, p1)  # the same per-lane chains and the same partial order


@pytest.mark.parametrize("heads,d_head,act", [(4, 75, 1), (2, 64, 0), (1, 300, 1), (8, 32, 1)])
def test_gat_fwd_sliced_vs_rowmajor_and_oracle(device, monkeypatch, heads, d_head, act):
    """gnnea_gat_fwd_sliced_f32 (slice-major table, row statistics first) vs the fp64 oracle
    (att_layers.py:29-61 x heads, oracle/gnn.gat_layer) and vs the row-major edge pass; the
    saved row max / denominator are the row-major kernel's; the backward runs on them."""
    from gnnea import ops, synth
    from oracle.gnn import gat_layer
    n = 700
    tr = synth.kg_pair_triples(n, 4 * n, 40, seed=11)
    r, c, v = synth.adjacency_coo(tr, 2 * n, reference_order=False)
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.stack([r, c])), torch.from_numpy(v),
                                  (2 * n, 2 * n)).to(device)
    rng = np.random.default_rng(heads * 100 + d_head)
    D = heads * d_head
    x = rng.standard_normal((2 * n, 64)).astype(np.float32)
    W = (rng.standard_normal((heads, 64, d_head)) * 0.2).astype(np.float32)
    A = (rng.standard_normal((heads, 1, 2 * d_head)) * 0.3).astype(np.float32)
    R = rng.standard_normal((2 * n, D)).astype(np.float32)
    actf = torch.relu if act else (lambda z: z)

    def run(sliced):
        monkeypatch.setattr(ops, "INFINITY_CACHE_BYTES", 1 if sliced else 1 << 40)
        monkeypatch.setattr(ops, "GAT_SLICED", sliced)
        xt = torch.from_numpy(x).to(device).requires_grad_(True)
        H = ops.matmul(xt, torch.cat(list(torch.from_numpy(W).to(device)), dim=1))
        y = ops.gat(adj, H, torch.from_numpy(A).to(device).view(heads, 2 * d_head), heads,
                    d_head, 0.2, actf if act else None)
        (y * torch.from_numpy(R).to(device)).sum().backward()
        return y.detach().cpu(), xt.grad.cpu()

    ys, gs = run(True)
    yr, gr = run(False)
    xo = torch.from_numpy(x).double()
    yo = gat_layer(xo, torch.from_numpy(W).double(), torch.from_numpy(A).double(), r, c, 0.2,
                   act=actf)
    assert rel_err(ys, yo) < 1e-4
    assert rel_err(ys, yr) < 1e-5
    assert rel_err(gs, gr) < 1e-5


@pytest.mark.parametrize("M,N,K,bias", [(5000, 300, 300, True), (4100, 128, 64, False),
                                        (300, 300, 36, False), (70001, 300, 300, True),
                                        (66000, 128, 320, False)])
def test_gemm_x3_dual_output(device, M, N, K, bias):
    """gnnea_gemm_x3_dual_f32: the row-major product and its slice-major copy from one GEMM
    (the copy is stored from the same registers: bit-identical to packing the product)."""
    from gnnea import ops
    g = torch.Generator(device="cpu").manual_seed(M + N)
    a = torch.randn(M, K, generator=g).to(device)
    b = torch.randn(K, N, generator=g).to(device)
    bb = torch.randn(N, generator=g).to(device) if bias else None
    xs = ops.sliced_empty(M, N, device, torch.float32)
    y = ops.gemm(a, b, bias=bb, x3=True, sliced_out=xs)
    ref = ops.gemm(a, b, bias=bb, x3=True)
    assert torch.equal(y, ref)
    assert torch.equal(ops.slice_pack(y), xs) or all(
        torch.equal(xs[s, :, :min(64, N - 64 * s)], y[:, 64 * s:64 * s + 64])
        for s in range(xs.shape[0]))
    ref64 = a.double() @ b.double() + (bb.double() if bias else 0)
    assert rel_err(y.cpu(), ref64.cpu()) < 1e-5


@pytest.mark.parametrize("M,N,K,bias", [(70001, 300, 300, True), (66000, 600, 300, False),
                                        (65536, 128, 320, True)])
def test_gemm_x3_tall_accumulate(device, M, N, K, bias):
    """The weight-resident kernel (tall M, K in (288, 320]) with C = A·B + bias + C (beta = 1,
    the epilogue reads C) against fp64."""
    from gnnea import ops
    g = torch.Generator(device="cpu").manual_seed(M + K)
    a = torch.randn(M, K, generator=g).to(device)
    b = torch.randn(K, N, generator=g).to(device)
    bb = torch.randn(N, generator=g).to(device) if bias else None
    c0 = torch.randn(M, N, generator=g).to(device)
    y = ops.gemm(a, b, bias=bb, x3=True, out=c0.clone(), beta=1.0)
    ref = c0.double() + a.double() @ b.double() + (bb.double() if bias else 0)
    assert rel_err(y.cpu(), ref.cpu()) < 1e-5
    y0 = ops.gemm(a, b, bias=bb, x3=True)
    ref0 = a.double() @ b.double() + (bb.double() if bias else 0)
    assert rel_err(y0.cpu(), ref0.cpu()) < 1e-5


@pytest.mark.parametrize("heads,d_head,act,mask,row0", [
    (4, 75, 1, True, 0), (2, 64, 0, False, 0), (1, 300, 1, True, 0), (8, 32, 1, False, 0),
    (3, 48, 1, True, 0), (4, 75, 1, True, 300), (2, 64, 0, False, 250)])
def test_gat_bwd_sliced_vs_rowmajor(device, monkeypatch, heads, d_head, act, mask, row0):
    """gnnea_gat_bwd_{prep,src,edge,dst}_sliced_f32 (G slice-major, per-slice product partials
    summed per head in slice order) against the row-major backward on the same forward records:
    dH and da.  row0 > 0: a row shard (destination rows row0.. of a wider H, ds2 (x) a2 applied
    by the edge pass instead of the destination pass)."""
    from gnnea import ops
    from gnnea.graph import DeviceCSR
    rng = np.random.default_rng(heads * 1000 + d_head + row0)
    n = 1500
    N = n if row0 == 0 else 700
    D = heads * d_head
    r = rng.integers(0, N, 14000)
    c = rng.integers(0, n, 14000)
    keep = (r > 2) & (r < N - 2)
    r = np.concatenate([r[keep], np.full(200, 9)])  # one row with several 64-edge chunks
    c = np.concatenate([c[keep], rng.integers(0, n, 200)])
    c[:50] = 7  # and a source row with many in-edges
    v = np.ones(r.size, np.float32)
    csr = DeviceCSR.from_coo(torch.from_numpy(r).to(device), torch.from_numpy(c).to(device),
                             torch.from_numpy(v).to(device), N, n)
    H = torch.from_numpy(rng.standard_normal((n, D)).astype(np.float32) * 0.5).to(device)
    a32 = torch.from_numpy(rng.standard_normal((heads, 2 * d_head)).astype(np.float32)
                           * 0.3).to(device)
    em = None
    if mask:
        em = torch.from_numpy(((rng.random((csr.nnz, heads)) > 0.3) / 0.7).astype(np.float32)
                              ).to(device)
    monkeypatch.setattr(ops, "GAT_SLICED", False)
    Y, m, den, s1, s2 = ops.gat_forward(csr, H, a32, heads, d_head, 0.2, act, em, row0=row0)
    dY = torch.from_numpy(rng.standard_normal((N, D)).astype(np.float32)).to(device)
    dH_r, da_r = ops.gat_backward(csr, H, a32, s1, s2, m, den, Y, dY, heads, d_head, 0.2, act,
                                  em, row0=row0)
    calls = []
    orig = ops._gat_backward_sliced
    monkeypatch.setattr(ops, "_gat_backward_sliced",
                        lambda *a, **k: (calls.append(1), orig(*a, **k))[1])
    monkeypatch.setattr(ops, "GAT_SLICED", True)
    monkeypatch.setattr(ops, "INFINITY_CACHE_BYTES", 1)
    dH_s, da_s = ops.gat_backward(csr, H, a32, s1, s2, m, den, Y, dY, heads, d_head, 0.2, act,
                                  em, row0=row0)
    assert calls, "the sliced backward was not taken"
    assert rel_err(dH_s.cpu(), dH_r.cpu()) < 1e-5
    assert rel_err(da_s.cpu(), da_r.cpu()) < 1e-5


@pytest.mark.parametrize("heads,d_head,act,mask", [(4, 75, 1, False), (8, 32, 1, True),
                                                   (3, 48, 0, True), (1, 300, 1, False)])
def test_gat_bf16_sliced_vs_rowmajor_and_oracle(device, monkeypatch, heads, d_head, act, mask):
    """bf16 storage (cfg-5): gnnea_gat_{fwd,bwd_*}_sliced_bf16 over 64-column (128-B) slices
    against the row-major bf16 passes and the fp64 oracle (att_layers.py:29-61 x heads) on the
    same bf16-rounded H: outputs, dH and da at the bf16 tolerance (each stored value rounded
    once per pass), the sliced passes actually taken."""
    from gnnea import ops
    from gnnea.graph import DeviceCSR
    rng = np.random.default_rng(7 * heads + d_head)
    n = 1500
    D = heads * d_head
    r = rng.integers(0, n, 16000)
    c = rng.integers(0, n, 16000)
    r = np.concatenate([r, np.arange(n), np.full(150, 11)])  # self loops; one long row
    c = np.concatenate([c, np.arange(n), rng.integers(0, n, 150)])
    v = np.ones(r.size, np.float32)
    csr = DeviceCSR.from_coo(torch.from_numpy(r).to(device), torch.from_numpy(c).to(device),
                             torch.from_numpy(v).to(device), n, n)
    H = torch.from_numpy(rng.standard_normal((n, D)).astype(np.float32) * 0.5).to(device)
    Hb = H.bfloat16()
    a32 = torch.from_numpy(rng.standard_normal((heads, 2 * d_head)).astype(np.float32)
                           * 0.3).to(device)
    em = None
    if mask:
        em = torch.from_numpy(((rng.random((csr.nnz, heads)) > 0.3) / 0.7).astype(np.float32)
                              ).to(device)
    dY = torch.from_numpy(rng.standard_normal((n, D)).astype(np.float32)).to(device).bfloat16()

    monkeypatch.setattr(ops, "GAT_SLICED_BF16", True)

    def run(sliced):
        monkeypatch.setattr(ops, "GAT_SLICED", sliced)
        monkeypatch.setattr(ops, "INFINITY_CACHE_BYTES", 1 if sliced else 1 << 40)
        calls = []
        orig = ops._gat_backward_sliced
        monkeypatch.setattr(ops, "_gat_backward_sliced",
                            lambda *a, **k: (calls.append(1), orig(*a, **k))[1])
        Y, m, den, s1, s2 = ops.gat_forward(csr, Hb, a32, heads, d_head, 0.2, act, em)
        dH, da = ops.gat_backward(csr, Hb, a32, s1, s2, m, den, Y, dY, heads, d_head, 0.2, act,
                                  em)
        monkeypatch.setattr(ops, "_gat_backward_sliced", orig)
        assert bool(calls) == sliced
        assert Y.dtype == dH.dtype == torch.bfloat16
        return Y.float().cpu(), dH.float().cpu(), da.cpu()

    ys, dhs, das = run(True)
    yr, dhr, dar = run(False)
    assert rel_err(ys, yr) < 1e-2
    assert rel_err(dhs, dhr) < 2e-2
    assert rel_err(das, dar) < 2e-2
    # fp64 oracle of the same forward on the bf16 H (edge mask as the numerator multiplier)
    H64 = Hb.double().cpu()
    A64 = a32.double().cpu()
    rr = torch.from_numpy(np.repeat(np.arange(n), np.diff(csr.rowptr.cpu().numpy())))
    cc = csr.col.long().cpu()
    H64.requires_grad_(True)
    A64.requires_grad_(True)
    outs = []
    for h in range(heads):
        hh = H64[:, h * d_head:(h + 1) * d_head]
        z = hh[rr] @ A64[h, :d_head] + hh[cc] @ A64[h, d_head:]
        e = torch.exp(-torch.nn.functional.leaky_relu(z, 0.2))
        den = torch.zeros(n, dtype=torch.float64).index_add(0, rr, e)
        w = e * (em[:, h].double().cpu() if mask else 1.0)
        num = torch.zeros((n, d_head), dtype=torch.float64).index_add(0, rr, w.unsqueeze(1) * hh[cc])
        o = num / den.unsqueeze(1)
        outs.append(torch.relu(o) if act else o)
    yo = torch.cat(outs, 1)
    (yo * dY.double().cpu()).sum().backward()
    assert rel_err(ys, yo.detach()) < 1e-2
    assert rel_err(dhs, H64.grad) < 2e-2
    assert rel_err(das, A64.grad) < 2e-2


def test_gat_dhead40_takes_rowmajor(device, monkeypatch):
    """d_head = 40 puts three heads into slice 1: the sliced gate refuses it and the layer runs
    the row-major passes (same results as with the sliced path switched off)."""
    from gnnea import ops
    from gnnea.graph import DeviceCSR
    rng = np.random.default_rng(40)
    n, heads, d_head = 900, 4, 40
    D = heads * d_head
    r = np.concatenate([rng.integers(0, n, 8000), np.arange(n)])
    c = np.concatenate([rng.integers(0, n, 8000), np.arange(n)])
    csr = DeviceCSR.from_coo(torch.from_numpy(r).to(device), torch.from_numpy(c).to(device),
                             torch.ones(r.size, device=device), n, n)
    H = torch.from_numpy(rng.standard_normal((n, D)).astype(np.float32)).to(device)
    a32 = torch.from_numpy(rng.standard_normal((heads, 2 * d_head)).astype(np.float32)
                           * 0.3).to(device)
    dY = torch.randn(n, D, device=device)
    out = []
    for sliced in (True, False):
        monkeypatch.setattr(ops, "GAT_SLICED", sliced)
        monkeypatch.setattr(ops, "INFINITY_CACHE_BYTES", 1)
        Y, m, den, s1, s2 = ops.gat_forward(csr, H, a32, heads, d_head, 0.2, 1)
        out.append((Y, ops.gat_backward(csr, H, a32, s1, s2, m, den, Y, dY, heads, d_head, 0.2,
                                        1)[0]))
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
