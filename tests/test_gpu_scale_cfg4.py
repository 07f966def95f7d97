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


def test_cfg4_gcn_layer_vs_oracle(device, cfg4):
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


def test_cfg4_highway_layer_vs_oracle(device, cfg4):
    from layers.layers import HighWayGraphConvolution
    from oracle.local import sampled_input_grads, sampled_outputs
    d = cfg4
    torch.manual_seed(10087)
    layer = HighWayGraphConvolution(300, 300, 0.0, F.relu, True, 0, device).to(device)
    xx = d["x"].clone().requires_grad_(True)
    out, _ = layer((xx, d["adj"]))
    assert type(out.grad_fn).__name__ == "HighwayLayerFnBackward"
    S_gpu = out.grad_fn.saved_tensors[3]  # relu(A·hidden) as the layer computed it (branch band)
    assert S_gpu.shape == out.shape
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


def test_cfg4_hgcn_ea_step_vs_fp64(device, cfg4):
    """One HGCN-EA training step (run/train_ea.py:55-66) on the full configs[3] graph."""
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
    outputs = m.decode(m.encode(d["x"], d["adj"]), d["adj"])
    m.neg_right = si.negatives(N, t, k, 31)
    m.neg2_left = si.negatives(N, t, k, 32)
    loss = m.get_loss(outputs, {"train": train}, "train")
    loss.backward()
    # fp64 restatement with the same weights (encoder: 2 HighWay layers, relu; decoder: 1, identity)
    layers = list(m.encoder.layers) + [m.decoder.cls]
    ps = [(L.linear.weight.detach().double().requires_grad_(True),
           L.linear.bias.detach().double().requires_grad_(True),
           L.kernel_gate.detach().double()) for L in layers]
    v64 = d["v"].double()
    h = d["x"].double()
    for i, (W, b, Kg) in enumerate(ps):
        h = fp64_ref.highway_layer(h, W, b, Kg, d["r"], d["c"], v64, relu=i < 2)
    ix = [torch.from_numpy(np.asarray(z, dtype=np.int64)).to(device) for z in
          (train[:, 0], train[:, 1], m.neg_left, m.neg_right, m.neg2_left, m.neg2_right)]
    loss64 = fp64_ref.margin_loss(h, *ix, t, k)
    loss64.backward()
    assert abs(float(loss) - float(loss64)) <= 1e-5 * abs(float(loss64))
    got = [(L.linear.weight.grad, L.linear.bias.grad) for L in layers]
    gmax = max(float(p.grad.abs().max()) for trip in ps for p in trip[:2])
    for (gW, gb), (W, b, _) in zip(got, ps):
        for g_, p in ((gW, W), (gb, b)):
            ref = p.grad
            if float(ref.abs().max()) < 1e-3 * gmax:  # analytically zero (last bias)
                assert float(g_.abs().max()) < 1e-3 * gmax
            else:
                assert rel_err(g_.cpu(), ref.cpu()) < 3e-3
