"""BASELINE configs[3] at its full size on one MI355X: 2 x 1M entities, 41,999,552 nnz, D = 300.

This is the production path with nothing monkeypatched: the projection on the x3 GEMM (M = 2M
rows), the hidden written slice-major (the table exceeds the Infinity Cache), one aggregation
launch per KG block, the fused sliced HighWay layer.  Checked against
  * the fp64 CPU oracle on sampled rows over their neighbourhoods (oracle/local.py): outputs and
    input gradients, norm-relative 1e-4;
  * a whole-graph fp64 restatement on the device (tests/fp64_ref.py) for the weight gradients,
    which sum over all 2M rows, 1e-4; and for one HGCN-EA training step (3 HighWay layers +
    EAModel.get_loss with t = 4500, k = 125): loss 1e-5, parameter gradients 3e-3 (the margin
    loss's sign sums cancel, as at cfg-1).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import fp64_ref
import scale_inputs as si
from conftest import rel_err

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]
TOL32 = 1e-4


@pytest.fixture(scope="module")
def cfg4(device):
    from gnnea import synth
    from oracle.local import LocalGraph
    cf = synth.CONFIGS["cfg4"]
    n = cf["n"]
    N = 2 * n
    tr = synth.kg_pair_triples(n, cf["t"], cf["n_rel"], seed=0)
    r, c, v = synth.adjacency_coo(tr, N, reference_order=False)
    del tr
    assert r.size == 41999552
    d = {"N": N, "n": n, "g": LocalGraph(r, c, v, N)}
    d["r"] = torch.from_numpy(r).to(device)
    d["c"] = torch.from_numpy(c).to(device)
    d["v"] = torch.from_numpy(v).to(device)
    d["adj"] = torch.sparse_coo_tensor(torch.stack([d["r"], d["c"]]), d["v"], (N, N))
    d["X"] = si.features(N)
    d["x"] = torch.from_numpy(d["X"]).to(device)
    d["Rn"] = si.upstream(N)
    d["R"] = torch.from_numpy(d["Rn"]).to(device)
    rows = si.sample_rows(N, 192, seed=41)
    d["rows"], d["grad_rows"] = rows, rows[::2]
    yield d
    d.clear()
    torch.cuda.empty_cache()


def _rows_of(t):
    t = t.detach()
    return lambda rows: t[torch.from_numpy(np.asarray(rows)).to(t.device)].float().cpu().numpy()


def test_cfg4_gcn_layer_vs_oracle(device, cfg4, relu_band):
    from layers.layers import GraphConvolution
    from oracle.local import sampled_input_grads, sampled_outputs
    d = cfg4
    torch.manual_seed(10086)
    layer = GraphConvolution(300, 300, 0.0, F.relu, True).to(device)
    xx = d["x"].clone().requires_grad_(True)
    out, _ = layer((xx, d["adj"]))
    assert type(out.grad_fn).__name__ == "GCNLayerFnBackward"  # the fused slice-major layer
    (out * d["R"]).sum().backward()
    W = layer.linear.weight.detach().cpu().double()
    b = layer.linear.bias.detach().cpu().double()
    S, o_ref = sampled_outputs("gcn", d["g"], d["X"], d["rows"], [W, b], "relu", _rows_of(out))
    assert rel_err(_rows_of(out.detach())(S), o_ref) < TOL32
    T, dx_ref = sampled_input_grads("gcn", d["g"], d["X"], d["Rn"], d["grad_rows"], [W, b],
                                    "relu", _rows_of(out))
    assert rel_err(_rows_of(xx.grad)(T), dx_ref) < TOL32
    x64 = d["x"].double()
    dW, db = fp64_ref.gcn_grads(d["r"], d["c"], d["v"].double(), x64, W.to(device),
                                b.to(device), d["R"].double(), out.detach().double())
    assert rel_err(layer.linear.weight.grad.cpu(), dW.cpu()) < TOL32
    assert rel_err(layer.linear.bias.grad.cpu(), db.cpu()) < TOL32


def test_cfg4_highway_layer_vs_oracle(device, cfg4, relu_band):
    from layers.layers import HighWayGraphConvolution
    from oracle.local import sampled_input_grads, sampled_outputs
    d = cfg4
    torch.manual_seed(10087)
    layer = HighWayGraphConvolution(300, 300, 0.0, F.relu, True, 0, device).to(device)
    xx = d["x"].clone().requires_grad_(True)
    out, _ = layer((xx, d["adj"]))
    assert type(out.grad_fn).__name__ == "HighwayLayerFnBackward"
    # relu's branch as the layer took it (for the rounding band): the forward keeps only the
    # sign of S = relu(A·hidden), bit (c % 4) of byte [row][16 (c // 64) + (c % 64) // 4]
    mask = out.grad_fn.saved_tensors[3]
    assert mask.dtype == torch.uint8 and mask.shape == (out.shape[0], 16 * 5)
    cols = torch.arange(out.shape[1], device=device)
    S_gpu = ((mask[:, 16 * (cols // 64) + (cols % 64) // 4] >> (cols % 4).to(torch.uint8)) & 1)
    S_gpu = S_gpu.to(torch.float32)
    del mask
    (out * d["R"]).sum().backward()
    W = layer.linear.weight.detach().cpu().double()
    b = layer.linear.bias.detach().cpu().double()
    Kg = layer.kernel_gate.detach().cpu().double()
    params = [W, b, Kg, None]
    S, o_ref = sampled_outputs("highway", d["g"], d["X"], d["rows"], params, "relu",
                               _rows_of(S_gpu))
    assert rel_err(_rows_of(out.detach())(S), o_ref) < TOL32
    T, dx_ref = sampled_input_grads("highway", d["g"], d["X"], d["Rn"], d["grad_rows"], params,
                                    "relu", _rows_of(S_gpu))
    assert rel_err(_rows_of(xx.grad)(T), dx_ref) < TOL32
    dW, db = fp64_ref.highway_grads(d["r"], d["c"], d["v"].double(), d["x"].double(),
                                    W.to(device), b.to(device), Kg.to(device), d["R"].double(),
                                    S_gpu.detach().double())
    assert rel_err(layer.linear.weight.grad.cpu(), dW.cpu()) < TOL32
    assert rel_err(layer.linear.bias.grad.cpu(), db.cpu()) < TOL32


def test_cfg4_hgcn_ea_step_vs_fp64(device, cfg4, relu_band, record_property):
    """One HGCN-EA training step (run/train_ea.py:55-66) on the full configs[3] graph, with the
    default projection GEMMs (the f16x2 form, GNNEA_X3W unset = 4): the loss against the fp64
    restatement's (1e-5), and EVERY parameter gradient against the fp64 restatement
    differentiated with the reference loss's cotangent at OUR outputs (1e-4; the margin loss's
    sign pattern is chaotic under rounding, so the fp64 step's own cotangent, whose gradients
    are recorded beside it, is not the bar)."""
    from models.models_ea import EAModel
    from test_dropin_cpu import make_args
    d = cfg4
    N, n = d["N"], d["n"]
    train = si.ea_pairs(n)
    t, k = train.shape[0], 125
    a = make_args("HGCN")
    a.cuda, a.device = 0, device
    a.n_nodes, a.neg_num, a.data = N, k, {"train": train}
    torch.manual_seed(10086)
    m = EAModel(a).to(device)
    m.train()
    enc_acts = []  # relu(S)'s sign of each encoder layer, as the layer took it (rounding band)
    for L in m.encoder.layers:
        L.register_forward_hook(lambda mod, i, o: enc_acts.append(
            fp64_ref.highway_s_sign(o[0] if isinstance(o, tuple) else o)))
    outputs = m.decode(m.encode(d["x"], d["adj"]), d["adj"])
    assert all(a_ is not None for a_ in enc_acts)
    m.neg_right = si.negatives(N, t, k, 31)
    m.neg2_left = si.negatives(N, t, k, 32)
    loss = m.get_loss(outputs, {"train": train}, "train")
    loss.backward()
    ix = [torch.from_numpy(np.asarray(z, dtype=np.int64)).to(device) for z in
          (train[:, 0], train[:, 1], m.neg_left, m.neg_right, m.neg2_left, m.neg2_right)]
    v64 = d["v"].double()
    # the same restatement in fp32 first (what any fp32 evaluation of these sums gets), then fp64
    g32, _ = fp64_ref.ea_step_grads(m, "HGCN", d["x"], d["r"], d["c"], v64, ix, t, k, outputs,
                                    enc_acts, [], dtype=torch.float32)
    g32 = {nm: g_.double() for nm, g_ in g32.items()}
    g64, h64 = fp64_ref.ea_step_grads(m, "HGCN", d["x"], d["r"], d["c"], v64, ix, t, k, outputs,
                                      enc_acts, [])
    with torch.no_grad():
        loss64 = fp64_ref.margin_loss(h64, *ix, t, k)
    loss_err = abs(float(loss) - float(loss64)) / abs(float(loss64))
    params = [(nm, p) for nm, p in m.named_parameters()]
    assert sorted(g64) == sorted(nm for nm, _ in params)
    gmax = max(float(g64[nm].abs().max()) for nm, _ in params)
    errs, errs32 = {"loss": loss_err}, {}
    for nm, p in params:
        ref = g64[nm]
        zero = float(ref.abs().max()) < 1e-3 * gmax
        for dst, got in ((errs, p.grad.double()), (errs32, g32[nm])):
            dst[nm] = float((got - ref).abs().max()) / gmax if zero else \
                rel_err(got.cpu(), ref.cpu())
    # reported: the fp64 step's own gradients (its cotangent at the fp64 outputs)
    h64r = h64.clone().requires_grad_(True)
    fp64_ref.margin_loss(h64r, *ix, t, k).backward()
    o64 = outputs.detach().double().requires_grad_(True)
    fp64_ref.margin_loss(o64, *ix, t, k).backward()
    cot_diff = rel_err(o64.grad.cpu(), h64r.grad.cpu())
    record_property("cfg4_hgcn_step_errs", {"vs_fp64_at_our_outputs": errs,
                                            "fp32_restatement_vs_fp64": errs32,
                                            "loss_cotangent_ours_vs_fp64_outputs": cot_diff})
    print("cfg4 HGCN-EA step vs the fp64 restatement at our outputs (loss rel; grads norm-rel; "
          "analytically-zero bias: max / largest gradient):", errs,
          "; the same restatement evaluated in fp32:", errs32,
          "; the loss cotangent at our outputs vs at the fp64 outputs: %.2e" % cot_diff)
    assert loss_err <= 1e-5
    # every parameter at 1e-4 (relu's branch in the rounding band follows the layers' own
    # signs: without that, a few near-zero S entries taking the other branch moved W1 to 1.3e-4)
    for nm, _ in params:
        assert errs[nm] < TOL32, (nm, errs[nm], errs32[nm])


def _coalesced(r, c, N):
    """Unique (row, col) pairs in row-major order (the edge set the GAT layer attends over,
    adj.coalesce().indices(), att_layers.py:31)."""
    key = torch.unique(r.long() * N + c.long())
    return key // N, key % N


def test_cfg4_gat_layer_vs_oracle(device, cfg4, monkeypatch, relu_band, record_property):
    """The fp32 4-head GAT layer (att_layers.py:29-61, 82-91) at full configs[3] size through
    the slice-major forward and backward (nothing monkeypatched but a spy): outputs and dx on
    sampled rows vs the fp64 neighbourhood oracle (1e-4), every head's W and a gradients vs the
    whole-graph fp64 restatement on the device (tests/fp64_ref.gat_layer, 1e-4)."""
    from gnnea import ops
    from layers.att_layers import GraphAttentionLayer
    from oracle.local import sampled_input_grads, sampled_outputs
    d = cfg4
    taken = []
    orig = ops._gat_sliced_applies
    monkeypatch.setattr(ops, "_gat_sliced_applies",
                        lambda *a, **k: (lambda v: (taken.append(v), v)[1])(orig(*a, **k)))
    torch.manual_seed(10089)
    layer = GraphAttentionLayer(300, 75, 0.0, F.relu, 0.2, 4, True).to(device)
    xx = d["x"].clone().requires_grad_(True)
    out, _ = layer((xx, d["adj"]))
    (out * d["R"]).sum().backward()
    assert taken == [True, True], taken  # sliced forward and sliced backward
    Ws = torch.stack([a.W.detach().cpu() for a in layer.attentions]).double()
    As = torch.stack([a.a.detach().cpu() for a in layer.attentions]).double()
    S, o_ref = sampled_outputs("gat", d["g"], d["X"], d["rows"], [Ws, As], "relu",
                               _rows_of(out))
    assert rel_err(_rows_of(out.detach())(S), o_ref) < TOL32
    T, dx_ref = sampled_input_grads("gat", d["g"], d["X"], d["Rn"], d["grad_rows"], [Ws, As],
                                    "relu", _rows_of(out))
    assert rel_err(_rows_of(xx.grad)(T), dx_ref) < TOL32
    r, c = _coalesced(d["r"], d["c"], d["N"])
    grads = {}
    for dt, store in ((torch.float64, None), (torch.float32, None),
                      ("f64_store32", fp64_ref.f32_store)):
        # the reference's op sequence (tests/fp64_ref.gat_layer: gathers, exp, index_add) in
        # fp64, in fp32 for the accumulation error any fp32 evaluation of these sums has, and in
        # fp64 with this path's fp32 storage points emulated (each head's projection H and the
        # output rounded to fp32, value and gradient): what is left there is our arithmetic
        cdt = torch.float64 if store is not None else dt
        Wd = Ws.to(device, cdt).requires_grad_(True)
        Ad = As.to(device, cdt).requires_grad_(True)
        yd = fp64_ref.gat_layer(d["x"].to(cdt), Wd, Ad, r, c, 0.2, True,
                                tested=out.detach().to(cdt), store=store)
        (yd * d["R"].to(cdt)).sum().backward()
        grads[dt] = (Wd.grad.double().cpu(), Ad.grad.double().cpu())
        del yd
    W64, A64 = grads[torch.float64]
    W32, A32 = grads[torch.float32]
    Ws32, As32 = grads["f64_store32"]
    # dW sums x_i (x) dH_i over 2M rows; da sums ds (x) H over every row, ds = sum of dz over the
    # row's 21 edges with dz = alpha (mask g.h_j - c_i) LeakyReLU', differences of nearby
    # products: far more cancellation, so fp32 accumulation alone lands further from fp64 there.
    # Each gradient must be within 1e-4 of fp64, or within twice the torch-fp32 evaluation's own
    # error, whichever is larger (the DBP15K tests' rule for the reference's fp32 step).
    # (The fp64 leg with this path's fp32 storage points emulated is reported: it does not close
    # the gap -- the a gradients' error is the fp32 arithmetic of the softmax backward's
    # differences G.H_j - c_i, which the torch fp32 evaluation shares.)
    errs = []
    for h, att in enumerate(layer.attentions):
        for ours, r64, r32, rst in ((att.W.grad, W64[h], W32[h], Ws32[h]),
                                    (att.a.grad, A64[h], A32[h], As32[h])):
            e, e32, est = rel_err(ours.cpu(), r64), rel_err(r32, r64), rel_err(ours.cpu(), rst)
            errs.append((e, e32, est))
            assert e < max(TOL32, 2.0 * e32), (h, e, e32)
    record_property("cfg4_gat_grad_errs", errs)
    print("cfg4 GAT layer grads (ours vs fp64, torch-fp32 vs fp64, ours vs fp64 with the fp32 "
          "storage points):", errs)
