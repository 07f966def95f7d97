"""BASELINE configs[4] shape on one MI355X: the 4-head GAT layer in bf16 storage on the
2 x 2M-entity / 2 x 20M-triple pair (~84M nnz) — the production bf16 path (bf16 MFMA projection,
all-heads edge pass per KG block, bf16 backward), nothing monkeypatched.

Checked against the fp64 CPU oracle over the sampled rows' neighbourhoods (oracle/local.py) on
the SAME bf16-rounded inputs and weights.  Stated bf16 tolerance: 1e-2
norm-relative on outputs (the projection H and the output are each rounded to bf16 once), 2e-2
on input gradients (bf16 dY·W and bf16 gradient storage), as tests/test_gpu_bf16.py.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import scale_inputs as si
from conftest import rel_err

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]
TOL_BF16 = 1e-2


@pytest.fixture(scope="module")
def cfg5(device):
    from gnnea import synth
    from oracle.local import LocalGraph
    cf = synth.CONFIGS["cfg5"]
    n = cf["n"]
    N = 2 * n
    tr = synth.kg_pair_triples(n, cf["t"], cf["n_rel"], seed=0)
    r, c, v = synth.adjacency_coo(tr, N, reference_order=False)
    del tr
    d = {"N": N, "nnz": int(r.size), "g": LocalGraph(r, c, v, N)}
    rt, ct = torch.from_numpy(r).to(device), torch.from_numpy(c).to(device)
    d["adj"] = torch.sparse_coo_tensor(torch.stack([rt, ct]), torch.from_numpy(v).to(device),
                                       (N, N))
    del r, c, v
    xb = torch.from_numpy(si.features(N)).to(device).bfloat16()
    d["xb"] = xb
    d["X"] = xb.float().cpu().numpy()  # the bf16 values the layer sees
    d["Rn"] = si.upstream(N)
    d["R"] = torch.from_numpy(d["Rn"]).to(device)
    rows = si.sample_rows(N, 128, seed=43)
    d["rows"], d["grad_rows"] = rows, rows[::2]
    yield d
    d.clear()
    torch.cuda.empty_cache()


def test_cfg5_gat_bf16_layer_vs_oracle(device, cfg5):
    from layers.att_layers import GraphAttentionLayer
    from oracle.local import sampled_input_grads, sampled_outputs
    d = cfg5
    assert d["nnz"] > 80_000_000
    torch.manual_seed(10088)
    layer = GraphAttentionLayer(300, 75, 0.0, F.relu, 0.2, 4, True).to(device).bfloat16()
    xx = d["xb"].clone().requires_grad_(True)
    out, _ = layer((xx, d["adj"]))
    assert out.dtype == torch.bfloat16
    (out.float() * d["R"]).sum().backward()
    assert xx.grad.dtype == torch.bfloat16
    Ws = torch.stack([a.W.detach().float().cpu() for a in layer.attentions]).double()
    As = torch.stack([a.a.detach().float().cpu() for a in layer.attentions]).double()

    def tested(t):
        return lambda rows: t[torch.from_numpy(np.asarray(rows)).to(t.device)].float().cpu().numpy()

    S, o_ref = sampled_outputs("gat", d["g"], d["X"], d["rows"], [Ws, As], "relu",
                               tested(out.detach()), tau=TOL_BF16)
    assert rel_err(tested(out.detach())(S), o_ref) < TOL_BF16
    T, dx_ref = sampled_input_grads("gat", d["g"], d["X"], d["Rn"], d["grad_rows"], [Ws, As],
                                    "relu", tested(out.detach()), tau=TOL_BF16)
    assert rel_err(tested(xx.grad)(T), dx_ref) < 2 * TOL_BF16
    for a in layer.attentions:
        assert torch.isfinite(a.W.grad.float()).all() and torch.isfinite(a.a.grad.float()).all()
