"""Generate the golden fixtures in tests/golden/ by running the REFERENCE implementation.

Run in the build container only (it needs /root/reference, which never travels to the GPU box):

    python tests/golden/gen_golden.py

The reference is imported as-is from /root/reference.  Two third-party modules it imports at
module top but never uses on the paths exercised here are absent from the image and replaced by
empty placeholder modules before the import:
  * ``ot`` (POT)      — imported by SinkhornOT/sinkhorn_loss.py:9, used only in __main__/tests;
  * ``torchtext``     — imported by utils/data_utils.py:13, used only by load_data_nctext.
Everything written here is data (inputs and expected outputs), no reference source.
"""
import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"


def _placeholders():
    sys.modules.setdefault("ot", types.ModuleType("ot"))
    tt = types.ModuleType("torchtext")
    ttd = types.ModuleType("torchtext.data")
    for name in ("Dataset", "BucketIterator", "Field", "Example"):
        setattr(ttd, name, object)
    tt.data = ttd
    sys.modules.setdefault("torchtext", tt)
    sys.modules.setdefault("torchtext.data", ttd)


def _synth():
    # the synthetic generator lives in the product package (host logic, not reference code)
    sys.path.insert(0, os.path.join(REPO, "gnn-mtl_amd"))
    from gnnea import synth  # noqa: E402
    sys.path.pop(0)
    for k in [m for m in sys.modules if m == "gnnea" or m.startswith("gnnea.")]:
        del sys.modules[k]
    return synth


def _digest(t):
    import hashlib
    a = t.detach().contiguous().numpy()
    return "%s|%s|%s" % (a.dtype.str, "x".join(map(str, a.shape)), hashlib.sha256(a.tobytes()).hexdigest())


def main():
    synth = _synth()
    _placeholders()
    sys.path.insert(0, REF)
    import layers.layers as RL
    import layers.att_layers as RA
    import models.encoders as RE
    import models.decoders as RD
    import utils.data_utils as RDU
    import utils.ot_loss as ROT
    import SinkhornOT.sinkhorn_loss as RSK
    torch.set_num_threads(8)

    # ---------------- graph (cfg-1: 2 x 1k entities, 2 x 2.5k triples) ----------------
    n, t = 1000, 2500
    N = 2 * n
    triples = synth.kg_pair_triples(n, t, 1000, seed=0)
    KG = [tuple(x) for x in triples.tolist()]
    adj = RDU.sparse_mx_to_torch_sparse_tensor(RDU.get_sparse_tensor(N, KG))
    X = synth.features(N, 300, seed=1)
    idx = adj._indices().numpy()
    np.savez_compressed(os.path.join(HERE, "graph_cfg1.npz"), triples=triples, row=idx[0],
                        col=idx[1], val=adj._values().numpy(), X=X, N=np.int64(N))

    # tiny edge-case graph: self-loop triple, multi-edges, isolated entity
    tr_small = np.array([[0, 0, 0], [1, 5, 2], [1, 6, 2], [2, 1, 1], [3, 0, 3], [4, 2, 0],
                         [5, 1, 6]], dtype=np.int64)
    adj_s = RDU.sparse_mx_to_torch_sparse_tensor(
        RDU.get_sparse_tensor(8, [tuple(x) for x in tr_small.tolist()]))
    np.savez_compressed(os.path.join(HERE, "graph_small.npz"), triples=tr_small,
                        row=adj_s._indices().numpy()[0], col=adj_s._indices().numpy()[1],
                        val=adj_s._values().numpy(), N=np.int64(8))

    x = torch.from_numpy(X)
    torch.manual_seed(7)
    R = torch.randn(N, 300)

    def run_layer(layer, split_out):
        xx = x.clone().requires_grad_(True)
        out = layer((xx, adj))[0] if split_out else layer(xx, adj)
        (out * R[:, :out.shape[1]]).sum().backward()
        return out.detach().numpy(), xx.grad.numpy()

    data = {}
    # GraphConvolution(300, 300, dropout 0, relu, bias)  (layers/layers.py:19-42)
    torch.manual_seed(10086)
    gc = RL.GraphConvolution(300, 300, 0.0, F.relu, True)
    gc.train()
    out, dx = run_layer(gc, True)
    data.update(gcn_W=gc.linear.weight.detach().numpy(), gcn_b=gc.linear.bias.detach().numpy(),
                gcn_out=out, gcn_dx=dx, gcn_dW=gc.linear.weight.grad.numpy(),
                gcn_db=gc.linear.bias.grad.numpy())
    # HighWayGraphConvolution (layers/layers.py:45-80)
    torch.manual_seed(10087)
    hw = RL.HighWayGraphConvolution(300, 300, 0.0, F.relu, True, -1, "cpu")
    hw.train()
    out, dx = run_layer(hw, True)
    data.update(hw_W=hw.linear.weight.detach().numpy(), hw_b=hw.linear.bias.detach().numpy(),
                hw_Kg=hw.kernel_gate.numpy(), hw_out=out, hw_dx=dx,
                hw_dW=hw.linear.weight.grad.numpy(), hw_db=hw.linear.bias.grad.numpy())
    # GraphAttentionLayer, 4 heads x 75, concat (layers/att_layers.py:67-91)
    torch.manual_seed(10088)
    ga = RA.GraphAttentionLayer(300, 75, 0.0, F.relu, 0.2, 4, True)
    ga.train()
    out, dx = run_layer(ga, True)
    data.update(gat_W=np.stack([h.W.detach().numpy() for h in ga.attentions]),
                gat_a=np.stack([h.a.detach().numpy() for h in ga.attentions]),
                gat_out=out, gat_dx=dx,
                gat_dW=np.stack([h.W.grad.numpy() for h in ga.attentions]),
                gat_da=np.stack([h.a.grad.numpy() for h in ga.attentions]))
    np.savez_compressed(os.path.join(HERE, "layers_cfg1.npz"), **data)

    # ---------------- full encoder + decoder forward, reference init under seed 10086 ----------
    class Args:
        pass

    enc = {}
    for model in ("GCN", "GAT", "HGCN"):
        a = Args()
        a.model, a.num_layers, a.dim, a.act, a.dropout, a.bias = model, 3, 300, "relu", 0.0, 1
        a.n_heads, a.alpha, a.feat_dim, a.n_classes, a.cuda, a.device = 4, 0.2, 300, 300, -1, "cpu"
        torch.manual_seed(10086)
        e = RE.model2encoder[model](a)
        d = RD.model2decoder[model](a)
        e.eval()
        d.eval()
        xs = torch.from_numpy(X).to_sparse()
        with torch.no_grad():
            h = e.encode(xs, adj)
            o = d.decode(h, adj)
        enc[model + "_out"] = o.numpy()
        # weights are regenerated by the drop-in constructors under the same seed; the fixture
        # pins them bit-for-bit by digest (key order = state_dict order)
        for part, mod in (("enc", e), ("dec", d)):
            for k, v in mod.state_dict().items():
                enc["%s_%s.%s" % (model, part, k)] = np.array(_digest(v))
        if model == "HGCN":
            for i, layer in enumerate(e.layers):
                enc["HGCN_enc_kernel_gate.%d" % i] = np.array(_digest(layer.kernel_gate))
            enc["HGCN_dec_kernel_gate"] = np.array(_digest(d.cls.kernel_gate))
    np.savez_compressed(os.path.join(HERE, "encoders_cfg1.npz"), **enc)

    # ---------------- Sinkhorn family ----------------
    sk = {}
    rng = np.random.default_rng(5)
    for tag, (I, J) in {"s": (100, 120), "m": (300, 300)}.items():
        Xs = 0.05 * rng.standard_normal((I, 300))
        Ys = 0.05 * rng.standard_normal((J, 300))
        M = torch.cdist(torch.from_numpy(Xs).float(), torch.from_numpy(Ys).float(), p=2)
        M = M / M.max()
        sk["%s_M" % tag] = M.numpy()
        for reg in (0.05, 0.01):
            key = "%s_r%g" % (tag, reg)
            P, loss = ROT.sinkhorn(torch.ones(I), torch.ones(J), M, reg=reg)
            sk[key + "_knopp_P"] = P.numpy()
            sk[key + "_knopp_loss"] = loss.numpy()
            C = M.double().view(1, I, J)
            mu = torch.full((1, I, 1), 1.0 / I, dtype=torch.float64)
            nu = torch.full((1, 1, J), 1.0 / J, dtype=torch.float64)
            for name, fn in (("stab", lambda: RSK.sinkhorn_iteration(C, mu, nu, reg)),
                             ("gen", lambda: RSK.gsinkhorn_iteration(C, mu, nu, 1.0, reg)),
                             ("relax", lambda: RSK.forward_relax_sinkhorn_iteration(
                                 C, mu, nu, 1.0, reg))):
                tr_, m1, m2, K = fn()
                sk["%s_%s_transport" % (key, name)] = tr_.numpy()
                sk["%s_%s_m1" % (key, name)] = m1.numpy()
                sk["%s_%s_m2" % (key, name)] = m2.numpy()
                if tag == "s" or name == "stab":
                    sk["%s_%s_K" % (key, name)] = K.numpy()
    # underflow case: EA-like un-normalised distances, reg 0.01 -> K^T u == 0 break at it. 0
    Xu = rng.standard_normal((64, 300)) * 0.6
    Yu = rng.standard_normal((80, 300)) * 0.6
    Mu = torch.cdist(torch.from_numpy(Xu).float(), torch.from_numpy(Yu).float(), p=2)
    P, loss = ROT.sinkhorn(torch.ones(64), torch.ones(80), Mu, reg=0.01)
    sk.update(under_M=Mu.numpy(), under_P=P.numpy(), under_loss=loss.numpy())
    # the reference test's own configuration (SinkhornOT/test_Sinkhorn_OT.py:9-49): cosine
    # costs of uniform vectors, eps 1e-4, fp64, seeded here (the test leaves the seed unset)
    from SinkhornOT.cderivation import cos_dist_mat, get_inter_sim
    Va = torch.from_numpy(rng.uniform(size=(100, 100)))
    Vb = torch.from_numpy(rng.uniform(size=(100, 100)))
    Mt = get_inter_sim(Va, Vb, cos_dist_mat).double()
    at = torch.full((1, 100, 1), 0.01, dtype=torch.float64)
    bt = torch.full((1, 1, 100), 0.01, dtype=torch.float64)
    tr_, m1, m2, K = RSK.sinkhorn_iteration(Mt.view(1, 100, 100), at, bt, 1e-4)
    sk.update(test_M=Mt.numpy(), test_transport=tr_.numpy(), test_m1=m1.numpy(),
              test_m2=m2.numpy(), test_K=K.numpy())
    np.savez_compressed(os.path.join(HERE, "sinkhorn.npz"), **sk)
    print("golden fixtures written to", HERE)


def gen_l1():
    """§8f #1 fixtures: get_neg / get_hits / eval_at_1 / generate_pairs of the reference."""
    _synth()
    _placeholders()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import models.models_ea as RM
    import utils.eval_utils as REV
    rng = np.random.default_rng(11)
    n, D = 1000, 300
    left = (0.1 * rng.standard_normal((n, D))).astype(np.float32)
    # right entity = left + noise: mixed hit ranks (Hits@1 well below 100)
    right = (left + 0.3 * rng.standard_normal((n, D))).astype(np.float32)
    vec = np.concatenate([left, right])
    perm = rng.permutation(n)
    train = np.stack([perm[:150], perm[:150] + n], 1).astype(np.int64)
    test = np.stack([perm[150:550], perm[150:550] + n], 1).astype(np.int64)
    out = {"vec": vec, "train": train, "test": test}
    tv = torch.from_numpy(vec)
    out["neg_right"] = RM.BaseModel.get_neg(None, train[:, 0], tv, 25)
    out["neg2_left"] = RM.BaseModel.get_neg(None, train[:, 1], tv, 25)
    for split, pairs in (("train", train), ("test", test)):
        m = REV.get_hits(tv, pairs)
        out["hits_%s_keys" % split] = np.array(list(m.keys()))
        out["hits_%s_vals" % split] = np.array(list(m.values()), dtype=np.float64)
    out["eval_at_1"] = np.array(float(REV.eval_at_1(tv, {"test": test})))
    holder = types.SimpleNamespace(ILL=None)
    e1 = 700
    index1 = {i: int(x) for i, x in enumerate(rng.permutation(n)[:e1])}
    index2 = {i: int(x) + n for i, x in enumerate(rng.permutation(n)[:e1])}
    RM.UEAModel.generate_pairs(holder, tv, {"e1": e1, "e2": e1, "index1": index1,
                                            "index2": index2}, 200)
    out["gp_index1"] = np.array([index1[i] for i in range(e1)])
    out["gp_index2"] = np.array([index2[i] for i in range(e1)])
    out["gp_ILL"] = np.asarray(holder.ILL, dtype=np.int64)
    RM.UEAModel.generate_pairs(holder, tv, {"e1": e1, "e2": e1, "index1": index1,
                                            "index2": index2}, 30)
    out["gp_ILL30"] = np.asarray(holder.ILL, dtype=np.int64)
    # §8f #2 margin loss with those negatives (EAModel.get_loss), value and d loss / d outputs
    k = 25
    holder = types.SimpleNamespace(neg_num=k, neg_right=out["neg_right"],
                                   neg2_left=out["neg2_left"])
    holder.neg_left = (np.ones((len(train), k)) * train[:, 0:1]).reshape(-1)
    holder.neg2_right = (np.ones((len(train), k)) * train[:, 1:2]).reshape(-1)
    tg = tv.clone().requires_grad_(True)
    loss = RM.EAModel.get_loss(holder, tg, {"train": train}, "train")
    loss.backward()
    out["margin_loss"] = np.array(float(loss))
    out["margin_grad"] = tg.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "l1_search.npz"), **out)
    print("l1 fixtures written to", HERE)


def gen_ties():
    """Tie-heavy fixture for get_neg / get_hits: duplicated rows, an all-equal
    block and rows on a coarse grid, so many L1 distances are exactly equal.  The reference ranks
    with numpy's default argsort (models/models_ea.py:26, utils/eval_utils.py:78,85), whose order
    among equal keys is unspecified (introsort; SIMD-dispatched on some CPUs); the engine orders
    ties by index.  The fixture records what the reference returned here, with the numpy
    version, so the test can pin everything that does not depend on the tie order."""
    _synth()
    _placeholders()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import models.models_ea as RM
    import utils.eval_utils as REV
    rng = np.random.default_rng(17)
    n, D = 400, 64
    base = np.round(rng.standard_normal((n, D)) * 2) / 4  # coarse grid: exact, many equal sums
    base[40:80] = base[40]                                 # an all-equal block
    dup = rng.choice(n, 60, replace=False)
    base[dup[30:]] = base[dup[:30]]                         # 30 duplicated pairs
    vec = np.concatenate([base, base + (rng.random((n, D)) < 0.05) / 4]).astype(np.float32)
    perm = rng.permutation(n)
    train = np.stack([perm[:100], perm[:100] + n], 1).astype(np.int64)
    test = np.stack([perm[100:300], perm[100:300] + n], 1).astype(np.int64)
    tv = torch.from_numpy(vec)
    out = {"vec": vec, "train": train, "test": test, "numpy_version": np.array(np.__version__)}
    k = 25
    out["neg_right"] = RM.BaseModel.get_neg(None, train[:, 0], tv, k)
    out["neg2_left"] = RM.BaseModel.get_neg(None, train[:, 1], tv, k)
    for split, pairs in (("train", train), ("test", test)):
        m = REV.get_hits(tv, pairs)
        out["hits_%s_keys" % split] = np.array(list(m.keys()))
        out["hits_%s_vals" % split] = np.array(list(m.values()), dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "l1_ties.npz"), **out)
    print("tie fixtures written to", HERE)


def gen_train_trace():
    """run/train_ea.py:53-67 loop (3 epochs) of the reference EAModel on the cfg-1 graph."""
    _synth()
    _placeholders()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import models.models_ea as RM
    import utils.eval_utils as REV
    torch.set_num_threads(8)
    g = dict(np.load(os.path.join(HERE, "graph_cfg1.npz")))
    N = int(g["N"])
    adj = torch.sparse_coo_tensor(np.stack([g["row"], g["col"]]), g["val"], (N, N))
    x = torch.from_numpy(g["X"]).to_sparse()
    rng = np.random.default_rng(21)
    perm = rng.permutation(N // 2)
    train = np.stack([perm[:300], perm[:300] + N // 2], 1).astype(np.int64)
    test = np.stack([perm[300:800], perm[300:800] + N // 2], 1).astype(np.int64)
    out = {"train": train, "test": test}

    class Args:
        pass

    for model in ("GCN", "GAT", "HGCN"):
        a = Args()
        a.model, a.num_layers, a.dim, a.act, a.dropout, a.bias = model, 3, 300, "relu", 0.0, 1
        a.n_heads, a.alpha, a.feat_dim, a.n_classes, a.cuda, a.device = 4, 0.2, 300, 300, -1, "cpu"
        a.n_nodes, a.neg_num, a.data = N, 10, {"train": train, "test": test}
        torch.manual_seed(10086)
        m = RM.EAModel(a)
        # plain SGD: Adam's first steps are +-lr for every weight whatever the gradient's size,
        # so rounding-level gradient differences would turn into lr-sized weight differences
        opt = torch.optim.SGD(params=m.parameters(), lr=2.0)
        sched = torch.optim.lr_scheduler.StepLR(opt, step_size=2000, gamma=0.5)
        losses = []
        for epoch in range(3):
            m.train()
            opt.zero_grad()
            outputs = m.decode(m.encode(x, adj), adj)
            if epoch % 50 == 0:
                m.neg_right = m.get_neg(train[:, 0], outputs, a.neg_num)
                m.neg2_left = m.get_neg(train[:, 1], outputs, a.neg_num)
                out[model + "_neg_right"] = m.neg_right
                out[model + "_neg2_left"] = m.neg2_left
            loss = m.get_loss(outputs, a.data, "train")
            loss.backward()
            if epoch == 0:  # parameter gradients of the first step (before Adam moves anything)
                for name, p in m.named_parameters():
                    out["%s_grad0.%s" % (model, name)] = p.grad.numpy().copy()
            opt.step()
            sched.step()
            losses.append(float(loss))
        m.eval()
        with torch.no_grad():
            outputs = m.decode(m.encode(x, adj), adj)
        met = REV.get_hits(outputs, test)
        out[model + "_losses"] = np.array(losses)
        out[model + "_hits"] = np.array(list(met.values()))
        out[model + "_final_out"] = outputs.numpy()
    np.savez_compressed(os.path.join(HERE, "train_trace_cfg1.npz"), **out)
    print("train trace written to", HERE)


def gen_gw():
    """§8f #3: the reference's GW / relaxed GW / FGW outer loops on small fp64 problems."""
    _synth()
    _placeholders()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import SinkhornOT.iterative_projection as RIP
    from SinkhornOT.cderivation import cos_dist_mat
    torch.set_num_threads(8)
    rng = np.random.default_rng(13)
    out = {}
    for tag, (I, J) in {"a": (60, 60), "b": (90, 70)}.items():
        X = torch.from_numpy(rng.uniform(size=(I, 16)))
        Y = torch.from_numpy(rng.uniform(size=(J, 16)))
        C1, C2 = cos_dist_mat(X, X), cos_dist_mat(Y, Y)
        M = cos_dist_mat(X, Y)
        mu = torch.full((I,), 1.0 / I, dtype=torch.float64)
        nu = torch.full((J,), 1.0 / J, dtype=torch.float64)
        out.update({tag + "_C1": C1.numpy(), tag + "_C2": C2.numpy(), tag + "_M": M.numpy()})
        T, d = RIP.gw_iterative_1(C1, C2, mu, nu, epsilon=0.01, max_iter=8)
        out.update({tag + "_gw_T": T.numpy(), tag + "_gw_d": np.array(float(d))})
        T, d = RIP.rgw_iterative_1(C1, C2, mu, nu, max_iter=8, lambdda=1.0, epsilon=0.01)
        out.update({tag + "_rgw_T": T.numpy(), tag + "_rgw_d": np.array(float(d))})
        T, d = RIP.fgw_iterative_1(M, C1, C2, mu, nu, alpha=0.5, p=2, max_iter=8, epsilon=0.01)
        out.update({tag + "_fgw_T": T.numpy(), tag + "_fgw_d": np.array(float(d))})
    np.savez_compressed(os.path.join(HERE, "gw.npz"), **out)
    print("gw fixtures written to", HERE)


def gen_ingest():
    """§8f #4: the reference's load_data_ea / load_seperate_data_ea on a small DBP15K-format
    dataset written by tests/data/make_dbp15k_like.py."""
    import tempfile
    import types as _t
    _synth()
    _placeholders()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REPO, "tests", "data"))
    import make_dbp15k_like
    import utils.data_utils as RDU
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as root:
        lang = make_dbp15k_like.write(root)
        os.chdir(root)
        try:
            np.random.seed(7)
            data = RDU.load_data_ea(_t.SimpleNamespace(dataset=lang, model="GCN"))
            np.random.seed(8)
            sep = RDU.load_seperate_data_ea(_t.SimpleNamespace(dataset=lang))
        finally:
            os.chdir(cwd)
    np.savez_compressed(os.path.join(HERE, "ingest.npz"), **make_dbp15k_like.flatten(data, sep))
    print("ingest fixtures written to", HERE)


def _scale_inputs():
    """tests/scale_inputs.py (needs the product package's synthetic generator on the path)."""
    sys.path.insert(0, os.path.join(REPO, "gnn-mtl_amd"))
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import scale_inputs
    sys.path.pop(0)
    sys.path.pop(0)
    for k in [m for m in sys.modules if m == "gnnea" or m.startswith("gnnea.")]:
        del sys.modules[k]
    return scale_inputs


class _Args:
    pass


def _ea_args(model, N, data, neg_num):
    a = _Args()
    a.model, a.num_layers, a.dim, a.act, a.dropout, a.bias = model, 3, 300, "relu", 0.0, 1
    a.n_heads, a.alpha, a.feat_dim, a.n_classes, a.cuda, a.device = 4, 0.2, 300, 300, -1, "cpu"
    a.n_nodes, a.neg_num, a.data = N, neg_num, data
    return a


def gen_dbp15k():
    """BASELINE configs[1] / configs[2] (DBP15K-scale pair, 2 x 15k entities): the reference's
    layers (GCN, HighWay, 4-head GAT: outputs and input gradients on a row sample, full weight
    gradients), GCN-EA / GAT-EA / HGCN-EA training steps (loss, parameter gradients, sampled
    outputs) with seeded negatives.  Inputs are rebuilt from seeds by tests/scale_inputs.py."""
    si = _scale_inputs()
    _placeholders()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import layers.layers as RL
    import layers.att_layers as RA
    import models.models_ea as RM
    import utils.data_utils as RDU
    torch.set_num_threads(8)
    tr, N, r, c, v = si.dbp15k_graph()
    n = N // 2
    adj = RDU.sparse_mx_to_torch_sparse_tensor(
        RDU.get_sparse_tensor(N, [tuple(x) for x in tr.tolist()]))
    idx = adj._indices().numpy()
    # the vectorised builder the tests use must equal the reference's COO here as well
    assert np.array_equal(idx[0], r) and np.array_equal(idx[1], c)
    assert np.array_equal(adj._values().numpy(), v)
    import hashlib
    out = {"adj_sha256": np.array(hashlib.sha256(idx.astype(np.int64).tobytes() +
                                                 adj._values().numpy().tobytes()).hexdigest()),
           "nnz": np.int64(idx.shape[1])}
    X = si.features(N)
    R = torch.from_numpy(si.upstream(N))
    rows = si.sample_rows(N, 512)
    out["rows"] = rows
    x = torch.from_numpy(X)

    def run_layer(layer):
        xx = x.clone().requires_grad_(True)
        o = layer((xx, adj))[0]
        (o * R[:, :o.shape[1]]).sum().backward()
        return o.detach().numpy()[rows], xx.grad.numpy()[rows]

    torch.manual_seed(10086)
    gc = RL.GraphConvolution(300, 300, 0.0, F.relu, True)
    o, dx = run_layer(gc)
    out.update(gcn_out=o, gcn_dx=dx, gcn_dW=gc.linear.weight.grad.numpy(),
               gcn_db=gc.linear.bias.grad.numpy())
    torch.manual_seed(10087)
    hw = RL.HighWayGraphConvolution(300, 300, 0.0, F.relu, True, -1, "cpu")
    o, dx = run_layer(hw)
    out.update(hw_out=o, hw_dx=dx, hw_dW=hw.linear.weight.grad.numpy(),
               hw_db=hw.linear.bias.grad.numpy())
    torch.manual_seed(10088)
    ga = RA.GraphAttentionLayer(300, 75, 0.0, F.relu, 0.2, 4, True)
    o, dx = run_layer(ga)
    out.update(gat_out=o, gat_dx=dx,
               gat_dW=np.stack([h.W.grad.numpy() for h in ga.attentions]),
               gat_da=np.stack([h.a.grad.numpy() for h in ga.attentions]))

    # one training step of run/train_ea.py:55-66 per model, negatives from seeds (k = 125)
    train = si.ea_pairs(n)
    t, k = train.shape[0], 125
    out["train"] = train
    xs = torch.from_numpy(X).to_sparse()
    for model in ("GCN", "GAT", "HGCN"):
        torch.manual_seed(10086)
        m = RM.EAModel(_ea_args(model, N, {"train": train}, k))
        m.train()
        outputs = m.decode(m.encode(xs, adj), adj)
        m.neg_right = si.negatives(N, t, k, 31)
        m.neg2_left = si.negatives(N, t, k, 32)
        loss = m.get_loss(outputs, {"train": train}, "train")
        loss.backward()
        out[model + "_loss"] = np.array(float(loss))
        out[model + "_out"] = outputs.detach().numpy()[rows]
        for name, p in m.named_parameters():
            out["%s_grad.%s" % (model, name)] = p.grad.numpy().copy()
        print(model, "EA step done, loss", float(loss), flush=True)
        # the same step in fp64 (same init: built in fp32 under the seed, then widened; the
        # HighWay gates are plain tensors, widened by hand; torch.ones in att_layers.py:45 follows
        # the default dtype).  The margin loss's sign sums make fp32 parameter gradients
        # rounding-sensitive, so the GPU test measures both fp32 runs against this one.
        torch.manual_seed(10086)
        m = RM.EAModel(_ea_args(model, N, {"train": train}, k))
        m.double()
        for mod in m.modules():
            if hasattr(mod, "kernel_gate"):
                mod.kernel_gate = mod.kernel_gate.double()
                mod.bias_gate = mod.bias_gate.double()
        m.train()
        torch.set_default_dtype(torch.float64)
        try:
            outputs = m.decode(m.encode(xs.double(), adj.double()), adj.double())
            m.neg_right = si.negatives(N, t, k, 31)
            m.neg2_left = si.negatives(N, t, k, 32)
            loss = m.get_loss(outputs, {"train": train}, "train")
            loss.backward()
        finally:
            torch.set_default_dtype(torch.float32)
        out[model + "_loss64"] = np.array(float(loss))
        for name, p in m.named_parameters():
            out["%s_grad64.%s" % (model, name)] = p.grad.numpy().copy()
        print(model, "fp64 EA step done, loss", float(loss), flush=True)
    np.savez_compressed(os.path.join(HERE, "dbp15k.npz"), **out)
    print("dbp15k fixtures written to", HERE)


def gen_sinkhorn_scale():
    """§8d Sinkhorn batches B = 3000 and 15000 (utils/ot_loss.py:5-76 as models_ea.py:217 calls
    it, a = b = ones, reg 0.01; sinkhorn_iteration at B = 3000): plans on a row sample, their
    marginals, losses / transports.  The costs come from tests/scale_inputs.sinkhorn_cost."""
    si = _scale_inputs()
    _placeholders()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import utils.ot_loss as ROT
    import SinkhornOT.sinkhorn_loss as RSK
    torch.set_num_threads(8)
    out = {}
    for B in (3000, 15000):
        M = si.sinkhorn_cost(B)
        rows = si.sample_rows(B, 32, seed=3)
        P, loss = ROT.sinkhorn(torch.ones(B), torch.ones(B), M, reg=0.01)
        out.update({"B%d_rows" % B: rows, "B%d_knopp_P" % B: P.numpy()[rows],
                    "B%d_knopp_rowsum" % B: P.sum(1).numpy(),
                    "B%d_knopp_colsum" % B: P.sum(0).numpy(),
                    "B%d_knopp_loss" % B: loss.numpy()})
        del P
        if B == 3000:
            C = M.double().view(1, B, B)
            mu = torch.full((1, B, 1), 1.0 / B, dtype=torch.float64)
            nu = torch.full((1, 1, B), 1.0 / B, dtype=torch.float64)
            tr_, m1, m2, K = RSK.sinkhorn_iteration(C, mu, nu, 0.01)
            out.update({"B%d_stab_transport" % B: tr_.numpy(), "B%d_stab_m1" % B: m1.numpy(),
                        "B%d_stab_m2" % B: m2.numpy(), "B%d_stab_K" % B: K[0].numpy()[rows],
                        "B%d_stab_Kcolsum" % B: K[0].sum(0).numpy()})
        print("sinkhorn B =", B, "done", flush=True)
    np.savez_compressed(os.path.join(HERE, "sinkhorn_scale.npz"), **out)
    print("sinkhorn scale fixtures written to", HERE)


if __name__ == "__main__":
    sections = {"l1": gen_l1, "ties": gen_ties, "train": gen_train_trace, "gw": gen_gw, "ingest": gen_ingest,
                "dbp15k": gen_dbp15k, "sinkhorn_scale": gen_sinkhorn_scale}
    if sys.argv[1:]:
        for name in sys.argv[1:]:
            sections[name]()
    else:
        main()
        gen_l1()
        gen_ties()
        gen_train_trace()
        gen_gw()
        gen_ingest()
        gen_dbp15k()
        gen_sinkhorn_scale()
