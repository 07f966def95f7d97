"""The oracle (CPU restatements) pinned against fixtures produced by the reference itself."""
import numpy as np
import pytest
import torch

from conftest import rel_err
from oracle import gnn, sinkhorn as osk
from oracle.adjacency import adjacency_loops

FP32_TOL = 1e-5  # oracle is fp64; the reference fixtures are fp32 (measured 1.8e-7 .. 4.1e-7)


def _graph(golden):
    g = golden("graph_cfg1")
    return g, torch.from_numpy(g["X"]).double()


def test_adjacency_loops_match_reference(golden):
    for name in ("graph_cfg1", "graph_small"):
        g = golden(name)
        r, c, v = adjacency_loops([tuple(t) for t in g["triples"].tolist()])
        assert np.array_equal(r, g["row"]) and np.array_equal(c, g["col"])
        assert np.array_equal(v.view(np.int32), g["val"].view(np.int32))


def _R():
    torch.manual_seed(7)
    return torch.randn(2000, 300).double()


def test_gcn_layer_oracle(golden):
    g, x = _graph(golden)
    L = golden("layers_cfg1")
    out, dx, (dW, db) = gnn.layer_with_grads(
        lambda xx, W, b: gnn.gcn_layer(xx, W, b, g["row"], g["col"], g["val"]),
        x, [L["gcn_W"], L["gcn_b"]], _R())
    assert rel_err(out, L["gcn_out"]) < FP32_TOL
    assert rel_err(dx, L["gcn_dx"]) < FP32_TOL
    assert rel_err(dW, L["gcn_dW"]) < FP32_TOL
    assert rel_err(db, L["gcn_db"]) < FP32_TOL


def test_highway_layer_oracle(golden):
    g, x = _graph(golden)
    L = golden("layers_cfg1")
    Kg = torch.from_numpy(L["hw_Kg"]).double()
    out, dx, (dW, db) = gnn.layer_with_grads(
        lambda xx, W, b: gnn.highway_layer(xx, W, b, Kg, g["row"], g["col"], g["val"]),
        x, [L["hw_W"], L["hw_b"]], _R())
    assert rel_err(out, L["hw_out"]) < FP32_TOL
    assert rel_err(dx, L["hw_dx"]) < FP32_TOL
    assert rel_err(dW, L["hw_dW"]) < FP32_TOL
    assert rel_err(db, L["hw_db"]) < FP32_TOL


def test_gat_layer_oracle(golden):
    g, x = _graph(golden)
    L = golden("layers_cfg1")
    out, dx, (dW, da) = gnn.layer_with_grads(
        lambda xx, W, a: gnn.gat_layer(xx, W, a, g["row"], g["col"], 0.2),
        x, [L["gat_W"], L["gat_a"]], _R())
    assert rel_err(out, L["gat_out"]) < FP32_TOL
    assert rel_err(dx, L["gat_dx"]) < FP32_TOL
    assert rel_err(dW, L["gat_dW"]) < FP32_TOL
    assert rel_err(da, L["gat_da"]) < 1e-4


@pytest.mark.parametrize("tag", ["s", "m"])
@pytest.mark.parametrize("reg", [0.05, 0.01])
def test_sinkhorn_oracles(golden, tag, reg):
    S = golden("sinkhorn")
    M = S["%s_M" % tag]
    I, J = M.shape
    key = "%s_r%g" % (tag, reg)
    P, loss, _, _ = osk.knopp(np.ones(I), np.ones(J), M.astype(np.float64), reg)
    assert rel_err(P, S[key + "_knopp_P"]) < 1e-12
    assert abs(loss - float(S[key + "_knopp_loss"])) <= 1e-12 * abs(loss)
    for mode in ("stab", "gen", "relax"):
        t, m1, m2, K = osk.stabilized(M, np.full(I, 1.0 / I), np.full(J, 1.0 / J), reg,
                                      mode=mode, lam=1.0,
                                      tol=1e-9 if mode == "stab" else 1e-6)
        assert abs(t - float(S["%s_%s_transport" % (key, mode)])) <= 1e-12 * abs(t)
        assert abs(m1 - float(S["%s_%s_m1" % (key, mode)])) <= 1e-10 * max(abs(m1), 1e-12)
        assert abs(m2 - float(S["%s_%s_m2" % (key, mode)])) <= 1e-10 * max(abs(m2), 1e-12)
        kk = "%s_%s_K" % (key, mode)
        if kk in S:
            assert rel_err(K, S[kk]) < 1e-12


def test_sinkhorn_underflow_break(golden):
    S = golden("sinkhorn")
    M = S["under_M"].astype(np.float64)
    P, loss, cpt, broke = osk.knopp(np.ones(M.shape[0]), np.ones(M.shape[1]), M, 0.01)
    assert broke and cpt == 0
    assert rel_err(P, S["under_P"]) < 1e-12


def test_sinkhorn_reference_test_config(golden):
    """SinkhornOT/test_Sinkhorn_OT.py:37-52 configuration (eps 1e-4, cosine costs)."""
    S = golden("sinkhorn")
    M = S["test_M"]
    t, m1, m2, K = osk.stabilized(M, np.full(100, 0.01), np.full(100, 0.01), 1e-4)
    assert abs(t - float(S["test_transport"])) <= 1e-10 * abs(t)
    assert rel_err(K, S["test_K"]) < 1e-10


def test_l1_search_oracle(golden):
    """oracle/l1.py vs the reference's get_neg / get_hits / eval_at_1 / generate_pairs."""
    from oracle import l1 as ol1
    f = golden("l1_search")
    vec, tr, te = f["vec"], f["train"], f["test"]
    assert (ol1.get_neg(tr[:, 0], vec, 25) == f["neg_right"]).all()
    assert (ol1.get_neg(tr[:, 1], vec, 25) == f["neg2_left"]).all()
    for split, pairs in (("train", tr), ("test", te)):
        m = ol1.get_hits(vec, pairs)
        assert list(m) == list(f["hits_%s_keys" % split])
        assert list(m.values()) == list(f["hits_%s_vals" % split])
    assert abs(ol1.eval_at_1(vec, te) - float(f["eval_at_1"])) < 1e-4  # reference: fp32 mean
    for key, bsz in (("gp_ILL", 200), ("gp_ILL30", 30)):
        assert (ol1.mutual_pairs(vec, f["gp_index1"], f["gp_index2"], bsz) == f[key]).all()


def test_margin_oracle(golden):
    """oracle/margin.py vs the reference's EAModel.get_loss (value and d loss / d outputs)."""
    from oracle import margin as om
    f = golden("l1_search")
    tr, k = f["train"], 25
    t = len(tr)
    nl = np.repeat(tr[:, 0], k)
    nr2 = np.repeat(tr[:, 1], k)
    loss, grad = om.margin_loss_and_grad(f["vec"], tr[:, 0], tr[:, 1], nl, f["neg_right"],
                                         f["neg2_left"], nr2, t, k)
    assert abs(loss - float(f["margin_loss"])) <= 1e-5 * abs(loss)
    assert rel_err(grad, f["margin_grad"]) < 1e-5


def test_l1_ties_oracle_vs_reference(golden):
    """Tie-heavy fixture (gen_golden.py gen_ties: duplicated rows, an all-equal block, a coarse
    grid): the stable-order oracle agrees with the reference's numpy-argsort results up to the
    order among exactly equal distances (tests/tie_rules.py), and does differ in that order on
    this input -- the documented deviation ("Ties")."""
    import tie_rules
    from oracle import l1
    f = golden("l1_ties")
    vec, train, test = f["vec"], f["train"], f["test"]
    differ = 0
    for col, key in ((0, "neg_right"), (1, "neg2_left")):
        got = l1.get_neg(train[:, col], vec, 25)
        differ += tie_rules.check_neg(vec, train[:, col], got, f[key], 25)
    assert differ > 0  # the fixture does exercise tie order
    for split, pairs in (("train", train), ("test", test)):
        tie_rules.check_hits(vec, pairs, l1.get_hits(vec, pairs), f["hits_%s_keys" % split],
                             f["hits_%s_vals" % split])
