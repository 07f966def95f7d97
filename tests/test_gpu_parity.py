"""HIP path vs the reference fixtures and the CPU oracle (run on an MI355X: pytest -m gpu).

Tolerance: norm-relative ||y - y_ref||_inf / ||y_ref||_inf <= 1e-4 for fp32
outputs (measured fp32-vs-fp64 error of the reference itself: 1.8e-7 .. 4.1e-7); fp64 Sinkhorn
(both device paths, resident-K scaling form and log domain): 1e-9 relative on plans and scalars.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import rel_err

pytestmark = pytest.mark.gpu
TOL32 = 1e-4
TOL64 = 1e-9


def _adj(g, dev, n=None):
    n = int(g["N"]) if n is None else n
    idx = torch.from_numpy(np.stack([g["row"], g["col"]]).astype(np.int64))
    return torch.sparse_coo_tensor(idx, torch.from_numpy(g["val"]), (n, n)).to(dev)


def _R(dev):
    torch.manual_seed(7)
    return torch.randn(2000, 300).to(dev)


# ------------------------------------------------------------------------------------------ #
# a1: COO -> CSR                                                                              #
# ------------------------------------------------------------------------------------------ #
def test_csr_matches_scipy(golden, device):
    import scipy.sparse as sp
    from gnnea.graph import DeviceCSR
    g = golden("graph_cfg1")
    rng = np.random.default_rng(0)
    # append duplicates and an explicit zero to exercise coalescing
    dup = rng.integers(0, g["row"].size, 500)
    row = np.concatenate([g["row"], g["row"][dup], [5]])
    col = np.concatenate([g["col"], g["col"][dup], [1999]])
    val = np.concatenate([g["val"], g["val"][dup] * 0.5, [0.0]]).astype(np.float32)
    csr = DeviceCSR.from_coo(torch.from_numpy(row).to(device), torch.from_numpy(col).to(device),
                             torch.from_numpy(val).to(device), 2000, 2000)
    ref = sp.coo_matrix((val.astype(np.float64), (row, col)), shape=(2000, 2000)).tocsr()
    ref.sort_indices()
    assert np.array_equal(csr.rowptr.cpu().numpy(), ref.indptr)
    assert np.array_equal(csr.col.cpu().numpy(), ref.indices)
    assert np.allclose(csr.val.cpu().numpy(), ref.data, rtol=1e-6, atol=0)
    assert (5, 1999) in set(zip(np.repeat(np.arange(2000), np.diff(ref.indptr)).tolist(),
                                ref.indices.tolist()))
    t = csr.transpose()
    refT = ref.T.tocsr()
    refT.sort_indices()
    assert np.array_equal(t.rowptr.cpu().numpy(), refT.indptr)
    assert np.array_equal(t.col.cpu().numpy(), refT.indices)
    perm = t.perm.cpu().numpy()
    assert np.array_equal(csr.val.cpu().numpy()[perm], t.val.cpu().numpy())


def test_csr_rejects_out_of_range(device):
    from gnnea.graph import DeviceCSR
    r = torch.tensor([0, 1, 7], device=device)
    c = torch.tensor([0, 1, 2], device=device)
    with pytest.raises(ValueError):
        DeviceCSR.from_coo(r, c, torch.ones(3, device=device), 4, 4)


# ------------------------------------------------------------------------------------------ #
# a2-a4: GCN / HighWay layers vs the reference fixtures                                       #
# ------------------------------------------------------------------------------------------ #
def _layer_case(layer, x, adj, R):
    xx = x.clone().requires_grad_(True)
    out = layer((xx, adj))[0]
    (out * R[:, :out.shape[1]]).sum().backward()
    return out.detach().cpu().numpy(), xx.grad.cpu().numpy()


def test_gcn_layer_vs_reference(golden, device):
    from layers.layers import GraphConvolution
    g, L = golden("graph_cfg1"), golden("layers_cfg1")
    gc = GraphConvolution(300, 300, 0.0, F.relu, True).to(device)
    with torch.no_grad():
        gc.linear.weight.copy_(torch.from_numpy(L["gcn_W"]))
        gc.linear.bias.copy_(torch.from_numpy(L["gcn_b"]))
    gc.train()
    out, dx = _layer_case(gc, torch.from_numpy(g["X"]).to(device), _adj(g, device), _R(device))
    assert rel_err(out, L["gcn_out"]) < TOL32
    assert rel_err(dx, L["gcn_dx"]) < TOL32
    assert rel_err(gc.linear.weight.grad.cpu(), L["gcn_dW"]) < TOL32
    assert rel_err(gc.linear.bias.grad.cpu(), L["gcn_db"]) < TOL32


def test_highway_layer_vs_reference(golden, device):
    from layers.layers import HighWayGraphConvolution
    g, L = golden("graph_cfg1"), golden("layers_cfg1")
    hw = HighWayGraphConvolution(300, 300, 0.0, F.relu, True, 0, device).to(device)
    with torch.no_grad():
        hw.linear.weight.copy_(torch.from_numpy(L["hw_W"]))
        hw.linear.bias.copy_(torch.from_numpy(L["hw_b"]))
    hw.kernel_gate = torch.from_numpy(L["hw_Kg"]).to(device)
    out, dx = _layer_case(hw, torch.from_numpy(g["X"]).to(device), _adj(g, device), _R(device))
    assert rel_err(out, L["hw_out"]) < TOL32
    assert rel_err(dx, L["hw_dx"]) < TOL32
    assert rel_err(hw.linear.weight.grad.cpu(), L["hw_dW"]) < TOL32
    assert rel_err(hw.linear.bias.grad.cpu(), L["hw_db"]) < TOL32


def test_gat_layer_vs_reference(golden, device):
    from layers.att_layers import GraphAttentionLayer
    g, L = golden("graph_cfg1"), golden("layers_cfg1")
    ga = GraphAttentionLayer(300, 75, 0.0, F.relu, 0.2, 4, True).to(device)
    with torch.no_grad():
        for h, att in enumerate(ga.attentions):
            att.W.copy_(torch.from_numpy(L["gat_W"][h]))
            att.a.copy_(torch.from_numpy(L["gat_a"][h]))
    out, dx = _layer_case(ga, torch.from_numpy(g["X"]).to(device), _adj(g, device), _R(device))
    assert rel_err(out, L["gat_out"]) < TOL32
    assert rel_err(dx, L["gat_dx"]) < TOL32
    dW = np.stack([a.W.grad.cpu().numpy() for a in ga.attentions])
    da = np.stack([a.a.grad.cpu().numpy() for a in ga.attentions])
    assert rel_err(dW, L["gat_dW"]) < TOL32
    assert rel_err(da, L["gat_da"]) < TOL32


@pytest.mark.parametrize("model", ["GCN", "GAT", "HGCN"])
def test_encoder_decoder_vs_reference(golden, device, model):
    from models.decoders import model2decoder
    from models.encoders import model2encoder
    from test_dropin_cpu import make_args
    g, E = golden("graph_cfg1"), golden("encoders_cfg1")
    a = make_args(model)
    a.cuda, a.device = 0, device
    torch.manual_seed(10086)  # reference init order reproduces the fixture's weights
    enc = model2encoder[model](a).to(device).eval()
    dec = model2decoder[model](a).to(device).eval()
    adj = _adj(g, device)
    xs = torch.from_numpy(g["X"]).to_sparse().to(device)  # sparse-COO features, as the ref
    with torch.no_grad():
        out = dec.decode(enc.encode(xs, adj), adj)
    assert rel_err(out.cpu(), E[model + "_out"]) < TOL32


# ------------------------------------------------------------------------------------------ #
# kernels vs the oracle on edge cases                                                         #
# ------------------------------------------------------------------------------------------ #
def _random_coo(rng, n_rows, n_cols, nnz, dup=True):
    r = rng.integers(0, n_rows, nnz)
    c = rng.integers(0, n_cols, nnz)
    if dup:
        r = np.concatenate([r, r[: nnz // 10]])
        c = np.concatenate([c, c[: nnz // 10]])
    v = rng.standard_normal(r.size).astype(np.float32)
    return r, c, v


@pytest.mark.parametrize("D", [1, 3, 4, 64, 72, 75, 76, 128, 148, 152, 252, 300, 512, 1024])
def test_spmm_shapes_vs_oracle(device, D):
    from gnnea import ops
    from gnnea.graph import DeviceCSR
    from oracle.gnn import coo_aggregate
    rng = np.random.default_rng(D)
    n = 700
    r, c, v = _random_coo(rng, n, n, 6000)
    # one very long row (>64 and >128 neighbours) and empty rows at both ends
    r = np.concatenate([r[(r > 3) & (r < n - 3)], np.full(200, 17)])
    c = np.concatenate([c[: r.size - 200], rng.integers(0, n, 200)])
    v = rng.standard_normal(r.size).astype(np.float32)
    x = rng.standard_normal((n, D)).astype(np.float32)
    csr = DeviceCSR.from_coo(torch.from_numpy(r).to(device), torch.from_numpy(c).to(device),
                             torch.from_numpy(v).to(device), n, n)
    for act, fn in ((0, lambda t: t), (1, torch.relu), (4, torch.sigmoid), (5, torch.tanh)):
        y = ops.spmm(csr, torch.from_numpy(x).to(device), act).cpu()
        ref = fn(coo_aggregate(r, c, v, n, torch.from_numpy(x).double()))
        assert rel_err(y, ref) < TOL32, (D, act)
    assert torch.all(ops.spmm(csr, torch.from_numpy(x).to(device))[:3].cpu() == 0)


def test_spmm_strided_input(device):
    from gnnea import ops
    from gnnea.graph import DeviceCSR
    from oracle.gnn import coo_aggregate
    rng = np.random.default_rng(1)
    r, c, v = _random_coo(rng, 300, 300, 3000)
    big = torch.from_numpy(rng.standard_normal((300, 320)).astype(np.float32)).to(device)
    x = big[:, :300]  # ld = 320
    csr = DeviceCSR.from_coo(torch.from_numpy(r).to(device), torch.from_numpy(c).to(device),
                             torch.from_numpy(v).to(device), 300, 300)
    y = ops.spmm(csr, x).cpu()
    assert rel_err(y, coo_aggregate(r, c, v, 300, x.cpu().double())) < TOL32


@pytest.mark.parametrize("heads,d,hub", [(1, 300, False), (4, 75, False), (2, 7, False),
                                         (8, 16, False), (3, 20, False), (6, 10, False),
                                         (2, 300, False), (8, 128, False), (4, 64, False),
                                         (4, 75, True), (1, 300, True)])
def test_gat_fwd_bwd_vs_oracle(device, heads, d, hub):
    from gnnea import ops
    from oracle.gnn import gat_layer
    rng = np.random.default_rng(heads * 100 + d)
    n, fin = 400, 48
    r, c, _ = _random_coo(rng, n, n, 3000, dup=False)
    if hub:
        keep = c != 0
        r, c = r[keep], c[keep]  # node 0 is a neighbour of every node: one source row with n in-edges (> 64)
        r = np.concatenate([r, np.arange(1, n)])
        c = np.concatenate([c, np.zeros(n - 1, dtype=c.dtype)])
    r = np.concatenate([r, np.arange(n)])  # every node has a self loop (reference needs >=1)
    c = np.concatenate([c, np.arange(n)])
    v = np.ones(r.size, dtype=np.float32)
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.stack([r, c])), torch.from_numpy(v),
                                  (n, n)).to(device)
    x = rng.standard_normal((n, fin)).astype(np.float32)
    W = (rng.standard_normal((heads, fin, d)) * 0.3).astype(np.float32)
    A = (rng.standard_normal((heads, 1, 2 * d)) * 0.3).astype(np.float32)
    Rr = rng.standard_normal((n, heads * d)).astype(np.float32)
    xt = torch.from_numpy(x).to(device).requires_grad_(True)
    Wt = torch.from_numpy(W).to(device).requires_grad_(True)
    At = torch.from_numpy(A).to(device).requires_grad_(True)
    H = ops.matmul(xt, torch.cat(list(Wt), dim=1))
    y = ops.gat(adj, H, At.view(heads, 2 * d), heads, d, 0.2, F.relu)
    (y * torch.from_numpy(Rr).to(device)).sum().backward()
    xo = torch.from_numpy(x).double().requires_grad_(True)
    Wo = torch.from_numpy(W).double().requires_grad_(True)
    Ao = torch.from_numpy(A).double().requires_grad_(True)
    yo = gat_layer(xo, Wo, Ao, r, c, 0.2)
    (yo * torch.from_numpy(Rr).double()).sum().backward()
    assert rel_err(y.detach().cpu(), yo.detach()) < TOL32
    assert rel_err(xt.grad.cpu(), xo.grad) < TOL32
    assert rel_err(Wt.grad.cpu(), Wo.grad) < TOL32
    assert rel_err(At.grad.cpu(), Ao.grad) < 3e-4


@pytest.mark.parametrize("shape", [(1, 1, 1), (37, 300, 300), (300, 75, 300), (513, 600, 300),
                                   (300, 300, 20000), (5, 300, 7), (70, 40, 12), (129, 321, 36)])
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gemm_vs_fp64(device, shape, ta, tb):
    from gnnea import ops
    M, N, K = shape
    rng = np.random.default_rng(M + N + K)
    a = rng.standard_normal((K, M) if ta else (M, K)).astype(np.float32)
    b = rng.standard_normal((N, K) if tb else (K, N)).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    y = ops.gemm(torch.from_numpy(a).to(device), torch.from_numpy(b).to(device), bool(ta),
                 bool(tb), bias=torch.from_numpy(bias).to(device)).cpu()
    ref = (a.T if ta else a).astype(np.float64) @ (b.T if tb else b).astype(np.float64) + bias
    assert rel_err(y, ref) < 1e-5
    # the same product through the three-way bf16 split (gnnea_gemm_x3_f32): fp32-level error
    y3 = ops.gemm(torch.from_numpy(a).to(device), torch.from_numpy(b).to(device), bool(ta),
                  bool(tb), bias=torch.from_numpy(bias).to(device), x3=True).cpu()
    assert rel_err(y3, ref) < 1e-5
    # magnitudes spread over many binades (the split terms of small entries are subnormal-free)
    scale = np.exp2(rng.integers(-20, 20, a.shape)).astype(np.float32)
    a2 = a * scale
    y3 = ops.gemm(torch.from_numpy(a2).to(device), torch.from_numpy(b).to(device), bool(ta),
                  bool(tb), x3=True).cpu()
    ref2 = (a2.T if ta else a2).astype(np.float64) @ (b.T if tb else b).astype(np.float64)
    assert rel_err(y3, ref2) < 1e-5


# ------------------------------------------------------------------------------------------ #
# a9-a12: Sinkhorn family vs the reference fixtures                                           #
# ------------------------------------------------------------------------------------------ #
@pytest.fixture(params=["onchip", "sweep", "logdomain"])
def sk_path(request, monkeypatch):
    """Run a Sinkhorn test through every device path."""
    import gnnea.sinkhorn
    # onchip: KNOPP with K held in registers + LDS by the persistent k_sk_res where it fits
    # (STAB family and larger problems take the sweep); sweep: flag GNNEA_SK_NO_ONCHIP, the
    # resident-K sweep for every mode; logdomain: variant 1
    monkeypatch.setattr(gnnea.sinkhorn, "DEFAULT_VARIANT", 1 if request.param == "logdomain" else 0)
    if request.param == "sweep":
        monkeypatch.setattr(gnnea.sinkhorn, "DEFAULT_FLAGS", gnnea.sinkhorn._lib.GNNEA_SK_NO_ONCHIP)
    return request.param


@pytest.mark.parametrize("tag", ["s", "m"])
@pytest.mark.parametrize("reg", [0.05, 0.01])
def test_sinkhorn_family_vs_reference(golden, device, tag, reg, sk_path):
    import SinkhornOT.sinkhorn_loss as SK
    from utils.ot_loss import sinkhorn
    S = golden("sinkhorn")
    M = torch.from_numpy(S["%s_M" % tag]).to(device)
    I, J = M.shape
    key = "%s_r%g" % (tag, reg)
    P, loss = sinkhorn(torch.ones(I, device=device), torch.ones(J, device=device), M, reg=reg)
    assert P.dtype == torch.float64
    assert rel_err(P.cpu(), S[key + "_knopp_P"]) < TOL64
    assert abs(loss.item() - float(S[key + "_knopp_loss"])) <= TOL64 * abs(loss.item())
    C = M.double().view(1, I, J)
    mu = torch.full((1, I, 1), 1.0 / I, dtype=torch.float64, device=device)
    nu = torch.full((1, 1, J), 1.0 / J, dtype=torch.float64, device=device)
    for name, fn in (("stab", lambda: SK.sinkhorn_iteration(C, mu, nu, reg)),
                     ("gen", lambda: SK.gsinkhorn_iteration(C, mu, nu, 1.0, reg)),
                     ("relax", lambda: SK.forward_relax_sinkhorn_iteration(C, mu, nu, 1.0, reg))):
        t, m1, m2, K = fn()
        assert K.shape == (1, I, J) and K.dtype == torch.float64
        for v, ref in ((t, "transport"), (m1, "m1"), (m2, "m2")):
            r = float(S["%s_%s_%s" % (key, name, ref)])
            assert abs(v.item() - r) <= 1e-8 * max(abs(r), 1e-12), (name, ref, v.item(), r)
        kk = "%s_%s_K" % (key, name)
        if kk in S:
            assert rel_err(K[0].cpu(), S[kk]) < TOL64, name


def test_sinkhorn_underflow_break(golden, device, sk_path):
    from utils.ot_loss import sinkhorn
    S = golden("sinkhorn")
    M = torch.from_numpy(S["under_M"]).to(device)
    P, loss = sinkhorn(torch.ones(M.shape[0], device=device),
                       torch.ones(M.shape[1], device=device), M, reg=0.01)
    assert rel_err(P.cpu(), S["under_P"]) < TOL64


def test_sinkhorn_reference_test_config(golden, device, sk_path):
    import SinkhornOT.sinkhorn_loss as SK
    S = golden("sinkhorn")
    M = torch.from_numpy(S["test_M"]).to(device).view(1, 100, 100)
    a = torch.full((1, 100, 1), 0.01, dtype=torch.float64, device=device)
    b = torch.full((1, 1, 100), 0.01, dtype=torch.float64, device=device)
    t, m1, m2, K = SK.sinkhorn_iteration(M, a, b, 1e-4)
    assert abs(t.item() - float(S["test_transport"])) <= 1e-8 * abs(float(S["test_transport"]))
    assert rel_err(K[0].cpu(), S["test_K"]) < 1e-8


def test_sinkhorn_vs_oracle_random(device):
    from oracle import sinkhorn as osk
    from utils.ot_loss import sinkhorn
    rng = np.random.default_rng(11)
    for I, J, reg in ((50, 70, 0.1), (257, 129, 0.02), (1000, 1000, 0.01)):
        M = rng.uniform(0, 1, (I, J))
        a = rng.uniform(0.5, 1.5, I)
        b = rng.uniform(0.5, 1.5, J)
        b *= a.sum() / b.sum()
        P, loss = sinkhorn(torch.from_numpy(a).to(device), torch.from_numpy(b).to(device),
                           torch.from_numpy(M).to(device), reg=reg, numItermax=300)
        Po, lo, _, _ = osk.knopp(a, b, M, reg, 300)
        assert rel_err(P.cpu(), Po) < TOL64, (I, J)
        assert abs(loss.item() - lo) <= TOL64 * abs(lo)


@pytest.mark.parametrize("I,J,reg,tol", [(1, 1, 0.1, 1e-9), (3, 5, 0.1, 1e-9),
                                         (144, 256, 0.05, 1e-9), (145, 257, 0.05, 1e-12),
                                         (1000, 1000, 0.01, 1e-9), (3000, 3000, 0.01, 1e-9),
                                         (5000, 1500, 0.02, 1e-10), (700, 9000, 0.02, 1e-9)])
def test_sinkhorn_onchip_matches_sweep(device, monkeypatch, I, J, reg, tol):
    """The persistent on-chip KNOPP kernel (k_sk_res: K in registers + LDS, workgroups exchanging
    row / column partials inside one launch per batch) against the resident-K sweep and the fp64
    oracle: same stop iteration and reason, plan and loss at 1e-12 (the two sum in different
    orders), over block shapes at and past the 144 x 256 tile, grids of 1 to 252 workgroups and
    solves spanning several launches (the host's batches 2, 10, 20, ...)."""
    from gnnea import sinkhorn as gsk
    from gnnea import _lib
    from oracle import sinkhorn as osk
    rng = np.random.default_rng(I * 7 + J)
    M = rng.uniform(0, 1, (I, J))
    a = rng.uniform(0.5, 1.5, I)
    b = rng.uniform(0.5, 1.5, J)
    b *= a.sum() / b.sum()
    Mt, at, bt = (torch.from_numpy(x).to(device) for x in (M, a, b))
    res = {}
    for path in ("onchip", "sweep"):
        # the scaling form (variant 0): with the on-chip path off, GNNEA_SK_AUTO would take the
        # fused log-domain sweep instead
        res[path] = gsk.solve(_lib.GNNEA_SK_KNOPP, Mt, at, bt, reg, tol, 400, variant=0,
                              flags=_lib.GNNEA_SK_NO_ONCHIP if path == "sweep" else 0)
    r0, r1 = res["onchip"], res["sweep"]
    assert (r0.path, r1.path) == ("onchip", "sweep")
    assert (r0.iters, r0.reason) == (r1.iters, r1.reason), ((r0.iters, r0.reason),
                                                            (r1.iters, r1.reason))
    assert rel_err(r0.plan.cpu(), r1.plan.cpu()) < 1e-12
    assert abs(r0.loss - r1.loss) <= 1e-12 * abs(r1.loss)
    # err = ||v (K^T u) - b||: absolute rounding ~1e-16 ||b|| once converged
    assert abs(r0.err - r1.err) <= 1e-9 * abs(r1.err) + 1e-12 * float(np.linalg.norm(b))
    if I * J <= 1_000_000:
        Po, lo, _, _ = osk.knopp(a, b, M, reg, 400, stop_thr=tol)
        assert rel_err(r0.plan.cpu(), Po) < TOL64
        assert abs(r0.loss - lo) <= TOL64 * abs(lo)


def test_sinkhorn_onchip_bad_u_break(device):
    """k_sk_res's numerical-error break on u (ot_loss.py:57-62: a row of K underflows to 0, so
    Kp v = 0 and u = inf at iteration 0): the same iteration count, reason and reverted plan as
    the sweep path."""
    import os
    from gnnea import sinkhorn as gsk
    from gnnea import _lib
    rng = np.random.default_rng(3)
    I, J = 600, 500
    M = rng.uniform(0, 1, (I, J))
    M[17] = 50.0  # exp(-50 / 0.05) underflows: K row 17 is 0
    a, b = np.ones(I), np.ones(J) * I / J
    Mt, at, bt = (torch.from_numpy(x).to(device) for x in (M, a, b))
    out = []
    for fl in (0, _lib.GNNEA_SK_NO_ONCHIP):
        out.append(gsk.solve(_lib.GNNEA_SK_KNOPP, Mt, at, bt, 0.05, 1e-9, 50, variant=0,
                             flags=fl))
    r0, r1 = out
    assert (r0.path, r1.path) == ("onchip", "sweep")
    assert (r0.iters, r0.reason) == (r1.iters, r1.reason) and r0.reason == 2, \
        ((r0.iters, r0.reason), (r1.iters, r1.reason))
    assert torch.equal(torch.isfinite(r0.plan), torch.isfinite(r1.plan))
    f = torch.isfinite(r1.plan)
    assert rel_err(r0.plan[f].cpu(), r1.plan[f].cpu()) < 1e-12


@pytest.mark.parametrize("bad", [float("nan"), float("-inf")])
def test_sinkhorn_logdomain_nonfinite_cost(device, monkeypatch, bad):
    """A NaN (or -inf) in M: the reference breaks at iteration 0 (K^T u has a NaN / inf, so v
    does, ot_loss.py:57-62) and returns the initial scalings' plan.  The log-domain KNOPP
    passes scan C at init and keep the NaN-propagating exact terms then (their scaled fast path
    clamps -inf / NaN exponents): same stop iteration and reason as the scaling form, the same
    plan where it is finite."""
    from gnnea import sinkhorn as gsk
    from gnnea import _lib
    rng = np.random.default_rng(8)
    M = rng.uniform(0, 1, (300, 200))
    M[7, 11] = bad
    w = torch.ones(300, dtype=torch.float64, device=device)
    wb = torch.full((200,), 1.5, dtype=torch.float64, device=device)
    Mt = torch.from_numpy(M).to(device)
    r0 = gsk.solve(_lib.GNNEA_SK_KNOPP, Mt, w, wb, 0.05, 1e-9, 50, variant=0,
                   flags=_lib.GNNEA_SK_NO_ONCHIP)
    r1 = gsk.solve(_lib.GNNEA_SK_KNOPP, Mt, w, wb, 0.05, 1e-9, 50, variant=1)
    assert (r1.iters, r1.reason) == (r0.iters, r0.reason), ((r1.iters, r1.reason),
                                                            (r0.iters, r0.reason))
    f = torch.isfinite(r0.plan)
    assert torch.equal(f, torch.isfinite(r1.plan))
    assert rel_err(r1.plan[f].cpu(), r0.plan[f].cpu()) < 1e-12


def test_spmm_beta_accumulate(device):
    from gnnea import ops
    from gnnea.graph import DeviceCSR
    from oracle.gnn import coo_aggregate
    rng = np.random.default_rng(5)
    r, c, v = _random_coo(rng, 500, 500, 4000)
    x = rng.standard_normal((500, 300)).astype(np.float32)
    y0 = rng.standard_normal((500, 300)).astype(np.float32)
    csr = DeviceCSR.from_coo(torch.from_numpy(r).to(device), torch.from_numpy(c).to(device),
                             torch.from_numpy(v).to(device), 500, 500)
    out = torch.from_numpy(y0).to(device)
    ops.spmm(csr, torch.from_numpy(x).to(device), 1, out=out, beta=1.0)
    ref = torch.relu(coo_aggregate(r, c, v, 500, torch.from_numpy(x).double()) +
                     torch.from_numpy(y0).double())
    assert rel_err(out.cpu(), ref) < TOL32


@pytest.mark.parametrize("world", [4, 8])
def test_shard_slice_pipeline_on_device(device, world):
    """The row-shard aggregation as the multi-GPU path runs it (gnnea.dist.KGShard.aggregate,
    gnnea.dist_graph.DistAdj.staged_aggregate): the KG's 64-column slice tables, slice q
    aggregated over the shard's CSR (KG-local columns) into the output's column block, per rank
    on one device (the halo filled locally); equal to the single-GPU rows."""
    from gnnea import ops, synth
    from gnnea.dist import Partition, shard_coo
    from gnnea.graph import DeviceCSR
    n, t = 800, 3000
    tr = synth.kg_pair_triples(n, t, 50)
    H = torch.from_numpy(synth.features(2 * n, 300, seed=2)).to(device)
    R, C, V = synth.adjacency_coo(tr, 2 * n, reference_order=False)
    full = DeviceCSR.from_coo(torch.from_numpy(R).to(device), torch.from_numpy(C).to(device),
                              torch.from_numpy(V).to(device), 2 * n, 2 * n)
    ref = ops.spmm(full, H, 1).cpu()
    for rank in range(world):
        p = Partition(n, rank, world)
        r, c, v = shard_coo(tr, n, t, p)
        csr = DeviceCSR.from_coo(torch.from_numpy(r).to(device), torch.from_numpy(c).to(device),
                                 torch.from_numpy(v).to(device), p.n_rows, n)
        tables = ops.slice_pack(H[p.kg * n:(p.kg + 1) * n])
        y = torch.empty(p.n_rows, 300, device=device)
        for q in range(tables.shape[0]):
            c0, c1 = 64 * q, min(300, 64 * q + 64)
            ops.spmm_sliced(csr, tables[q:q + 1], c1 - c0, 1, out=y[:, c0:c1])
        g0 = p.global_row0
        assert rel_err(y.cpu(), ref[g0:g0 + p.n_rows]) < TOL32


@pytest.mark.parametrize("variant", [0, 1])
def test_sinkhorn_rectangular_vs_oracle(device, variant):
    """Rectangular problems (I != J, b != a) agree with the oracle for both solver families."""
    from gnnea import _lib
    from gnnea.sinkhorn import solve
    from oracle import sinkhorn as osk
    rng = np.random.default_rng(variant)
    I, J, reg = 333, 517, 0.02
    M = rng.uniform(0, 1, (I, J))
    a = np.ones(I)
    b = np.ones(J) * I / J
    res = solve(_lib.GNNEA_SK_KNOPP, torch.from_numpy(M).to(device),
                torch.from_numpy(a).to(device), torch.from_numpy(b).to(device),
                reg, 1e-9, 200, variant=variant)
    Po, _, _, _ = osk.knopp(a, b, M, reg, 200)
    assert rel_err(res.plan.cpu(), Po) < TOL64
    res = solve(_lib.GNNEA_SK_STAB, torch.from_numpy(M).to(device),
                torch.from_numpy(a / I).to(device),
                torch.from_numpy(b / I).to(device), reg, 1e-9, 100, variant=variant)
    t, m1, m2, K = osk.stabilized(M, a / I, b / I, reg, 100, 1e-9)
    assert rel_err(res.plan.cpu(), K) < TOL64
    assert abs(res.transport_new - t) <= 1e-9 * abs(t)


@pytest.mark.parametrize("world", [4, 8])
def test_feature_partition_on_device(device, world):
    """Feature-column sharding: each rank's slice of relu(A.H) over its whole KG equals the
    matching columns of the single-GPU result."""
    from gnnea import ops, synth
    from gnnea.dist import Partition, shard_coo
    from gnnea.graph import DeviceCSR
    n, t = 800, 3000
    tr = synth.kg_pair_triples(n, t, 50)
    H = torch.from_numpy(synth.features(2 * n, 300, seed=2)).to(device)
    R, C, V = synth.adjacency_coo(tr, 2 * n, reference_order=False)
    full = DeviceCSR.from_coo(torch.from_numpy(R).to(device), torch.from_numpy(C).to(device),
                              torch.from_numpy(V).to(device), 2 * n, 2 * n)
    ref = ops.spmm(full, H, 1).cpu()
    for rank in range(world):
        p = Partition(n, rank, world, "features", 300)
        r, c, v = shard_coo(tr, n, t, p)
        csr = DeviceCSR.from_coo(torch.from_numpy(r).to(device), torch.from_numpy(c).to(device),
                                 torch.from_numpy(v).to(device), n, n)
        h = H[p.kg * n:(p.kg + 1) * n, p.col0:p.col1].contiguous()
        y = ops.spmm(csr, h, 1).cpu()
        assert rel_err(y, ref[p.kg * n:(p.kg + 1) * n, p.col0:p.col1]) < TOL32


# ------------------------------------------------------------------------------------------ #
# end-to-end drop-in: 3 epochs of run/train_ea.py's loop vs the reference's trace            #
# ------------------------------------------------------------------------------------------ #
@pytest.mark.parametrize("model", ["GCN", "GAT", "HGCN"])
def test_train_ea_trace_vs_reference(golden, device, model):
    """EAModel (encode/decode/get_neg/get_loss/backward/Adam) vs the reference's 3-epoch trace:
    same negatives (index-exact), losses and final outputs within fp32 tolerance."""
    from models.models_ea import EAModel
    from test_dropin_cpu import make_args
    from utils.eval_utils import get_hits
    g, T = golden("graph_cfg1"), golden("train_trace_cfg1")
    train, test = T["train"], T["test"]
    a = make_args(model)
    a.cuda, a.device = 0, device
    a.n_nodes, a.neg_num, a.data = int(g["N"]), 10, {"train": train, "test": test}
    torch.manual_seed(10086)
    m = EAModel(a).to(device)
    opt = torch.optim.SGD(params=m.parameters(), lr=2.0)  # as the fixture (see gen_golden.py)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=2000, gamma=0.5)
    adj = _adj(g, device)
    x = torch.from_numpy(g["X"]).to_sparse().to(device)
    losses = []
    for epoch in range(3):
        m.train()
        opt.zero_grad()
        outputs = m.decode(m.encode(x, adj), adj)
        if epoch % 50 == 0:
            m.neg_right = m.get_neg(train[:, 0], outputs, a.neg_num)
            m.neg2_left = m.get_neg(train[:, 1], outputs, a.neg_num)
            assert (m.neg_right == T[model + "_neg_right"]).all()
            assert (m.neg2_left == T[model + "_neg2_left"]).all()
        loss = m.get_loss(outputs, a.data, "train")
        loss.backward()
        if epoch == 0:
            # the reference's own fp32 gradients differ from its fp64 ones by up to 5e-4
            # norm-relative here (margin-loss sign sums cancel), so 3e-3 is the honest bound;
            # a gradient that is zero in exact arithmetic (the last bias: the L1 margin is
            # translation invariant) is rounding noise and is only bounded in absolute terms
            refs = {n: T["%s_grad0.%s" % (model, n)] for n, _ in m.named_parameters()}
            gmax = max(np.abs(r).max() for r in refs.values())
            for name, p in m.named_parameters():
                ref = refs[name]
                if np.abs(ref).max() < 1e-3 * gmax:
                    assert np.abs(p.grad.cpu().numpy()).max() < 1e-3 * gmax, name
                else:
                    assert rel_err(p.grad.cpu(), ref) < 3e-3, name
        opt.step()
        sched.step()
        losses.append(float(loss.detach()))
    np.testing.assert_allclose(losses, T[model + "_losses"], rtol=1e-4)
    m.eval()
    with torch.no_grad():
        outputs = m.decode(m.encode(x, adj), adj)
    # two updates through sign-valued margin gradients: the reference's own trained outputs move
    # by 6e-4 (GCN), 8e-3 (GAT), 1e-6 (HGCN) between two CPU runs with other thread counts
    tol = {"GCN": 3e-2, "GAT": 6e-2, "HGCN": 1e-3}[model]
    assert rel_err(outputs.cpu(), T[model + "_final_out"]) < tol
    hits = np.array(list(get_hits(outputs, test).values()))
    # the reference itself moves up to 3 of 500 ranks run to run (CPU thread order): near ties
    assert np.abs(hits - T[model + "_hits"]).max() <= 1.0


# ------------------------------------------------------------------------------------------ #
# §8f #3: GW / relaxed GW / FGW outer loops (device GEMMs + device Sinkhorn) vs the reference  #
# ------------------------------------------------------------------------------------------ #
@pytest.mark.parametrize("tag", ["a", "b"])
def test_gw_outer_loops_vs_reference(golden, device, tag):
    from SinkhornOT.iterative_projection import (fgw_iterative_1, gw_iterative_1,
                                                 rgw_iterative_1)
    f = golden("gw")
    C1 = torch.from_numpy(f[tag + "_C1"]).to(device)
    C2 = torch.from_numpy(f[tag + "_C2"]).to(device)
    M = torch.from_numpy(f[tag + "_M"]).to(device)
    I, J = C1.shape[0], C2.shape[0]
    mu = torch.full((I,), 1.0 / I, dtype=torch.float64, device=device)
    nu = torch.full((J,), 1.0 / J, dtype=torch.float64, device=device)
    runs = {"gw": lambda: gw_iterative_1(C1, C2, mu, nu, epsilon=0.01, max_iter=8),
            "rgw": lambda: rgw_iterative_1(C1, C2, mu, nu, max_iter=8, lambdda=1.0,
                                           epsilon=0.01),
            "fgw": lambda: fgw_iterative_1(M, C1, C2, mu, nu, alpha=0.5, p=2, max_iter=8,
                                           epsilon=0.01)}
    for name, run in runs.items():
        T, d = run()
        assert T.shape == f["%s_%s_T" % (tag, name)].shape
        assert rel_err(T.cpu(), f["%s_%s_T" % (tag, name)]) < 1e-8, name
        ref_d = float(f["%s_%s_d" % (tag, name)])
        assert abs(float(d) - ref_d) <= 1e-8 * abs(ref_d), name


def test_spmm_block_diagonal_launches(device, monkeypatch):
    """The two-KG adjacency is launched per diagonal block when X exceeds the Infinity Cache;
    per-row results are bit-identical to the single launch (same rows, same order)."""
    from gnnea import ops, synth
    from gnnea.graph import DeviceCSR
    n = 300000
    tr = synth.kg_pair_triples(n, 3 * n, 500, seed=4)
    r, c, v = synth.adjacency_coo(tr, 2 * n, reference_order=False)
    csr = DeviceCSR.from_coo(torch.from_numpy(r).to(device), torch.from_numpy(c).to(device),
                             torch.from_numpy(v).to(device), 2 * n, 2 * n)
    assert csr.row_blocks() == [(0, n), (n, 2 * n)]
    x = torch.randn(2 * n, 128, device=device)
    assert len(ops._blocks(csr, x)) == 2
    y_blocks = ops.spmm(csr, x, 1)
    heads, dh = 4, 75
    H = (torch.randn(2 * n, heads * dh, device=device) * 0.1).requires_grad_(True)
    a_all = (torch.randn(heads, 2 * dh, device=device) * 0.1).requires_grad_(True)
    dy = torch.randn(2 * n, heads * dh, device=device)

    # the row-major edge pass launched per block vs once (the sliced pass, which the default
    # cache size selects here, has its own tests in test_gpu_sliced.py)
    monkeypatch.setattr(ops, "GAT_SLICED", False)

    def gat_run():
        y = ops.GATFn.apply(H, a_all, csr, heads, dh, 0.2, 1, None)
        gH, ga = torch.autograd.grad(y, (H, a_all), dy)
        return y.detach(), gH, ga
    assert len(ops._blocks(csr, H)) == 2
    g_blocks = gat_run()
    monkeypatch.setattr(ops, "INFINITY_CACHE_BYTES", 1 << 40)
    assert len(ops._blocks(csr, x)) == 1
    y_one = ops.spmm(csr, x, 1)
    assert torch.equal(y_blocks, y_one)
    for u, w in zip(g_blocks, gat_run()):
        assert torch.equal(u, w)
    # a graph with an edge across the KGs has no split
    r2 = np.concatenate([r, [5]])
    c2 = np.concatenate([c, [2 * n - 1]])
    v2 = np.concatenate([v, [0.5]]).astype(np.float32)
    csr2 = DeviceCSR.from_coo(torch.from_numpy(r2).to(device), torch.from_numpy(c2).to(device),
                              torch.from_numpy(v2).to(device), 2 * n, 2 * n)
    assert csr2.row_blocks() == [(0, 2 * n)]


@pytest.mark.parametrize("mode_name", ["STAB", "RELAX", "KNOPP"])
def test_sinkhorn_batch_one_launch_sequence(device, mode_name):
    """gnnea.sinkhorn.solve_batch ([bt, I, J] as one launch sequence, one status read-back per
    round) equals solving each problem alone with solve(): same kernels, same stops."""
    from gnnea import _lib
    from gnnea.sinkhorn import solve, solve_batch
    mode = getattr(_lib, "GNNEA_SK_" + mode_name)
    g = torch.Generator().manual_seed(7)
    bt, I, J = 3, 70, 90
    C = torch.rand(bt, I, J, generator=g, dtype=torch.float64).to(device)
    C[1] *= 4.0  # different conditioning: the problems stop at different iterations
    a = torch.full((bt, I), 1.0 / I, dtype=torch.float64, device=device)
    b = torch.full((bt, J), 1.0 / J, dtype=torch.float64, device=device)
    eps, tol, it = (0.05, 1e-9, 200)
    p = 0.8 if mode_name == "RELAX" else 1.0
    res = solve_batch(mode, C, a, b, eps, tol, it, p=p)
    for k in range(bt):
        r1 = solve(mode, C[k], a[k], b[k], eps, tol, it, p=p)
        assert res[k].iters == r1.iters and res[k].reason == r1.reason
        assert torch.equal(res[k].plan, r1.plan)
        assert res[k].transport_new == r1.transport_new or mode_name == "KNOPP"
        assert res[k].loss == r1.loss or mode_name != "KNOPP"


def test_gemm_f64_vs_numpy(device):
    """gnnea_gemm_f64 (f64 MFMA) in all transpose forms with the fused alpha / beta * E epilogue
    (the GW products of SinkhornOT/cderivation.py:146-162) vs numpy fp64."""
    from gnnea import ops
    rng = np.random.default_rng(5)
    for (M, N, K) in [(1, 1, 1), (70, 90, 33), (128, 64, 300), (257, 130, 129)]:
        for ta in (0, 1):
            for tb in (0, 1):
                a = rng.standard_normal((K, M) if ta else (M, K))
                b = rng.standard_normal((N, K) if tb else (K, N))
                e = rng.standard_normal((M, N))
                out = ops.gemm_f64(torch.from_numpy(a).to(device), torch.from_numpy(b).to(device),
                                   bool(ta), bool(tb), alpha=-1.0,
                                   e=torch.from_numpy(e).to(device), beta=1.0).cpu().numpy()
                ref = e - (a.T if ta else a) @ (b.T if tb else b)
                assert rel_err(out, ref) < 1e-14, (M, N, K, ta, tb)


# reduced-precision legs of the GW / FGW outer loops: C1, C2, M rounded to fp32 / bf16, the
# cost GEMMs on gnnea's fp32 (x3) / bf16 kernels, each inner solve in fp64 and cast back
# (SinkhornOT/cderivation.py:160-162, iterative_projection.py:6-58).  The plan is exp(-2L/eps)
# at eps = 0.01, so a relative cost perturbation delta moves it by ~2|L|delta/eps: input rounding
# alone (fp32 6e-8, bf16 4e-3 relative, |L| <= 1) bounds the reachable agreement at ~1e-5 (fp32)
# and ~1 (bf16) — the stated tolerances: fp32 plan 1e-4 / distance 1e-5 against the reference's
# fp64 fixture; bf16 against the same reduced-precision loop run in fp64 on the bf16-rounded
# inputs (cost GEMM products exact, the one rounding of each product to bf16 is what differs):
# plan 5e-2 at eps = 0.1.
@pytest.mark.parametrize("tag", ["a", "b"])
def test_gw_outer_loops_fp32_vs_reference(golden, device, tag, record_property):
    from SinkhornOT.iterative_projection import fgw_iterative_1, gw_iterative_1
    f = golden("gw")
    C1 = torch.from_numpy(f[tag + "_C1"]).to(device).float()
    C2 = torch.from_numpy(f[tag + "_C2"]).to(device).float()
    M = torch.from_numpy(f[tag + "_M"]).to(device).float()
    I, J = C1.shape[0], C2.shape[0]
    mu = torch.full((I,), 1.0 / I, dtype=torch.float32, device=device)
    nu = torch.full((J,), 1.0 / J, dtype=torch.float32, device=device)
    errs = {}
    for name, run in (("gw", lambda: gw_iterative_1(C1, C2, mu, nu, epsilon=0.01, max_iter=8)),
                      ("fgw", lambda: fgw_iterative_1(M, C1, C2, mu, nu, alpha=0.5, p=2,
                                                      max_iter=8, epsilon=0.01))):
        T, d = run()
        assert T.dtype == torch.float32
        ref_d = float(f["%s_%s_d" % (tag, name)])
        errs[name] = (rel_err(T.cpu(), f["%s_%s_T" % (tag, name)]),
                      abs(float(d) - ref_d) / abs(ref_d))
    record_property("gw_fp32", errs)
    print("GW fp32 %s: %s" % (tag, errs))
    for name, (eT, ed) in errs.items():
        assert eT < 1e-4 and ed < 1e-5, (name, eT, ed)


@pytest.mark.parametrize("tag", ["a", "b"])
def test_gw_outer_loop_bf16(golden, device, tag, record_property):
    from SinkhornOT.iterative_projection import gw_iterative_1
    f = golden("gw")
    C1 = torch.from_numpy(f[tag + "_C1"]).to(device).bfloat16()
    C2 = torch.from_numpy(f[tag + "_C2"]).to(device).bfloat16()
    I, J = C1.shape[0], C2.shape[0]
    eps = 0.1
    mu = torch.full((I,), 1.0 / I, dtype=torch.float64, device=device)
    nu = torch.full((J,), 1.0 / J, dtype=torch.float64, device=device)
    Tb, db = gw_iterative_1(C1, C2, mu.bfloat16(), nu.bfloat16(), epsilon=eps, max_iter=8)
    assert Tb.dtype == torch.bfloat16
    T64, d64 = gw_iterative_1(C1.double(), C2.double(), mu, nu, epsilon=eps, max_iter=8)
    eT = rel_err(Tb.float().cpu(), T64.cpu())
    ed = abs(float(db) - float(d64)) / abs(float(d64))
    record_property("gw_bf16", (eT, ed))
    print("GW bf16 %s: plan %.2e, distance %.2e" % (tag, eT, ed))
    assert eT < 5e-2 and ed < 5e-2, (eT, ed)
