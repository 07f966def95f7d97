"""Drop-in modules on the host: reference signatures, RNG order / state_dict parity, and the
loud refusal to compute without a HIP device (no CPU fallback in the product path)."""
import hashlib

import numpy as np
import pytest
import torch
import torch.nn.functional as F


class Args:
    pass


def make_args(model):
    a = Args()
    a.model, a.num_layers, a.dim, a.act, a.dropout, a.bias = model, 3, 300, "relu", 0.0, 1
    a.n_heads, a.alpha, a.feat_dim, a.n_classes, a.cuda, a.device = 4, 0.2, 300, 300, -1, "cpu"
    return a


def digest(t):
    a = t.detach().contiguous().numpy()
    return "%s|%s|%s" % (a.dtype.str, "x".join(map(str, a.shape)),
                         hashlib.sha256(a.tobytes()).hexdigest())


@pytest.mark.parametrize("model", ["GCN", "GAT", "HGCN"])
def test_reference_init_bit_identical(golden, model):
    from models.decoders import model2decoder
    from models.encoders import model2encoder
    E = golden("encoders_cfg1")
    a = make_args(model)
    torch.manual_seed(10086)
    e = model2encoder[model](a)
    d = model2decoder[model](a)
    seen = 0
    for part, mod in (("enc", e), ("dec", d)):
        for k, v in mod.state_dict().items():
            assert str(E["%s_%s.%s" % (model, part, k)]) == digest(v), k
            seen += 1
    want = [k for k in E if k.startswith(model + "_") and "." in k and "kernel_gate" not in k]
    assert seen == len(want)
    if model == "HGCN":
        for i, layer in enumerate(e.layers):
            assert str(E["HGCN_enc_kernel_gate.%d" % i]) == digest(layer.kernel_gate)
        assert str(E["HGCN_dec_kernel_gate"]) == digest(d.cls.kernel_gate)


def test_layer_signatures_and_keys():
    from layers.att_layers import GraphAttentionLayer, SpGraphAttentionLayer
    from layers.layers import GraphConvolution, HighWayGraphConvolution, Linear
    gc = GraphConvolution(8, 6, 0.0, F.relu, True)
    assert set(gc.state_dict()) == {"linear.weight", "linear.bias"}
    hw = HighWayGraphConvolution(6, 6, 0.0, F.relu, True, -1, "cpu")
    assert set(hw.state_dict()) == {"linear.weight", "linear.bias"}  # gate is not a parameter
    assert hw.kernel_gate.shape == (6, 6) and not hw.kernel_gate.requires_grad
    ga = GraphAttentionLayer(8, 3, 0.0, F.relu, 0.2, 2, True)
    assert set(ga.state_dict()) == {"attention_0.W", "attention_0.a", "attention_1.W",
                                    "attention_1.a"}
    sp = SpGraphAttentionLayer(8, 3, 0.0, 0.2, F.relu)
    assert sp.W.shape == (8, 3) and sp.a.shape == (1, 6)
    assert set(Linear(4, 5, 0.0, F.relu, True).state_dict()) == {"linear.weight", "linear.bias"}


def test_no_cpu_fallback(golden):
    from gnnea import GnneaError
    from layers.layers import GraphConvolution
    g = golden("graph_small")
    adj = torch.sparse_coo_tensor(np.stack([g["row"], g["col"]]), g["val"], (8, 8))
    gc = GraphConvolution(4, 4, 0.0, F.relu, True)
    with pytest.raises(GnneaError):
        gc((torch.randn(8, 4), adj))


def test_sinkhorn_refuses_host_tensors():
    from gnnea import GnneaError
    from utils.ot_loss import sinkhorn
    with pytest.raises(GnneaError):
        sinkhorn(torch.ones(4), torch.ones(4), torch.rand(4, 4), 0.1)
