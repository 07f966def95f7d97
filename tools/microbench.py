"""Per-kernel timings of the hot path at the cfg-4 scale (HIP events, median of reps).

    python tools/microbench.py [--n 1000000] [--reps 10] [--out gpurun_out/microbench.json]

Reports ms and the roofline-relevant rate of: CSR SpMM (gather model GB/s), HighWay SpMM
epilogue, MFMA f32 projection GEMM (TFLOP/s), GAT forward / backward (4 heads x 75), a GCN layer
forward+backward through the drop-in module, and Sinkhorn per-iteration time.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))
sys.path.insert(0, ROOT)

from gnnea import _lib, ops, synth  # noqa: E402
from gnnea.graph import DeviceCSR  # noqa: E402


def timeit(fn, reps, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1000000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "microbench.json"))
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n = args.n
    t = 10 * n
    t0 = time.time()
    tr = synth.kg_pair_triples(n, t, 3000)
    r, c, v = synth.adjacency_coo(tr, 2 * n, reference_order=False)
    N = 2 * n
    csr = DeviceCSR.from_coo(torch.from_numpy(r.astype(np.int32)).to(dev),
                             torch.from_numpy(c.astype(np.int32)).to(dev),
                             torch.from_numpy(v).to(dev), N, N)
    E = csr.nnz
    csr.transpose()
    print("graph N=%d E=%d built in %.1fs" % (N, E, time.time() - t0), file=sys.stderr)
    D = 300
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(N, D, device=dev, generator=g)
    X /= X.norm(dim=1, keepdim=True)
    res = {"N": N, "E": E, "D": D}
    only = set(args.only.split(",")) if args.only else None

    def want(k):
        return only is None or k in only

    gather = 4 * (N + 1) + 8 * E + 4 * E * D + 4 * N * D
    if want("spmm"):
        Y = torch.empty_like(X)
        ms = timeit(lambda: ops.spmm(csr, X, _lib.GNNEA_ACT_RELU, out=Y), args.reps)
        res["spmm_relu"] = {"ms": ms, "GBps_gather_model": gather / ms / 1e6,
                            "edges_per_s": E / ms * 1e3}
    if want("spmm_bf16"):
        # cfg-5 storage: bf16 rows gathered, fp32 accumulate, bf16 out (per-KG launches as ops)
        Xb = X.to(torch.bfloat16)
        Yb = torch.empty_like(Xb)
        ms = timeit(lambda: ops.spmm(csr, Xb, _lib.GNNEA_ACT_RELU, out=Yb), args.reps)
        gb = 4 * (N + 1) + 8 * E + 2 * E * D + 2 * N * D
        res["spmm_relu_bf16"] = {"ms": ms, "GBps_gather_model": gb / ms / 1e6,
                                 "edges_per_s": E / ms * 1e3}
        del Xb, Yb
    if want("spmm_split"):
        # the same SpMM as two launches, one per KG block of rows (block-diagonal adjacency)
        Y = torch.empty_like(X)
        L = _lib.lib()
        st = _lib.stream_of(dev)

        def two():
            for k in range(2):
                _lib.check(L.gnnea_spmm_csr_f32(
                    _lib.ctypes.c_void_p(csr.rowptr.data_ptr() + 4 * k * n), _lib.ptr(csr.col),
                    _lib.ptr(csr.val), n, D, _lib.ptr(X), D,
                    _lib.ctypes.c_void_p(Y.data_ptr() + 4 * k * n * D), D, 1, st))
        ms = timeit(two, args.reps)
        res["spmm_relu_two_launches"] = {"ms": ms, "GBps_gather_model": gather / ms / 1e6,
                                         "edges_per_s": E / ms * 1e3}
    if want("spmm_slices"):
        # per-rank work of the multi-GPU feature partition: one KG's rows (n of 2n), a column
        # slice of width Dl (world 2: 300, world 4: 152 / 148, world 8: 76 / 72)
        m = r < n
        csr1 = DeviceCSR.from_coo(torch.from_numpy(r[m].astype(np.int32)).to(dev),
                                  torch.from_numpy(c[m].astype(np.int32)).to(dev),
                                  torch.from_numpy(v[m]).to(dev), n, n)
        for Dl in (300, 152, 148, 76, 72):
            Xs = X[:n, :Dl].contiguous()
            Ys = torch.empty_like(Xs)
            ms = timeit(lambda: ops.spmm(csr1, Xs, _lib.GNNEA_ACT_RELU, out=Ys), args.reps)
            gb = 4 * (n + 1) + 8 * csr1.nnz + 4 * csr1.nnz * Dl + 4 * n * Dl
            res["spmm_kg_D%d" % Dl] = {"ms": ms, "GBps_gather_model": gb / ms / 1e6,
                                      "edges_per_s": csr1.nnz / ms * 1e3}
    if want("highway"):
        G = torch.randn(N, D, device=dev, generator=g)
        Wg = torch.zeros(D, device=dev)
        csr_obj = csr

        def hw():
            return ops.HighwayFn.apply(X, G, X, Wg, csr_obj, _lib.GNNEA_ACT_RELU)
        ms = timeit(hw, args.reps)
        b = gather + 2 * 4 * N * D + 2 * 4 * N * D  # + gate, resid reads, S/g saves
        res["highway_fwd"] = {"ms": ms, "GBps_model": b / ms / 1e6}
    if want("gemm"):
        W = torch.randn(D, D, device=dev, generator=g) * 0.05
        bvec = torch.zeros(D, device=dev)
        ms = timeit(lambda: ops.gemm(X, W, trans_b=True, bias=bvec), args.reps)
        res["gemm_xWt"] = {"ms": ms, "TFLOPs": 2.0 * N * D * D / ms / 1e9}
        dY = torch.randn(N, D, device=dev, generator=g)
        ms = timeit(lambda: ops.gemm(dY, X, trans_a=True), args.reps)
        res["gemm_dW_splitK"] = {"ms": ms, "TFLOPs": 2.0 * N * D * D / ms / 1e9}
        ms = timeit(lambda: torch.mm(X, W.t()), args.reps)
        res["torch_mm_xWt_hipblaslt"] = {"ms": ms, "TFLOPs": 2.0 * N * D * D / ms / 1e9}
    if want("gemm_bf16"):
        Xb = X.to(torch.bfloat16)
        Wb = (torch.randn(D, D, device=dev, generator=g) * 0.05).to(torch.bfloat16)
        bvec = torch.zeros(D, device=dev)
        io = 2 * (2 * N * D + D * D)  # read X, write Y (bf16), W
        ms = timeit(lambda: ops.gemm(Xb, Wb, trans_b=True, bias=bvec), args.reps)
        res["gemm_bf16_xWt"] = {"ms": ms, "TFLOPs": 2.0 * N * D * D / ms / 1e9,
                                "GBps_io": io / ms / 1e6}
        dYb = torch.randn(N, D, device=dev, generator=g).to(torch.bfloat16)
        ms = timeit(lambda: ops.gemm(dYb, Xb, trans_a=True), args.reps)
        res["gemm_bf16_dW_splitK"] = {"ms": ms, "TFLOPs": 2.0 * N * D * D / ms / 1e9}
        ms = timeit(lambda: ops.gemm(dYb, Wb), args.reps)
        res["gemm_bf16_dX"] = {"ms": ms, "TFLOPs": 2.0 * N * D * D / ms / 1e9}
        ms = timeit(lambda: torch.mm(Xb, Wb.t()), args.reps)
        res["torch_mm_bf16_xWt_hipblaslt"] = {"ms": ms, "TFLOPs": 2.0 * N * D * D / ms / 1e9}
        del Xb, dYb
    if want("gat"):
        heads, dh = 4, 75
        a_all = torch.randn(heads, 2 * dh, device=dev, generator=g) * 0.1
        H = X.clone().requires_grad_(True)
        a_all.requires_grad_(True)
        adj_csr = csr

        def fwd():
            return ops.GATFn.apply(H, a_all, adj_csr, heads, dh, 0.2, _lib.GNNEA_ACT_RELU, None)
        ms = timeit(fwd, args.reps)
        b = 4 * (N + 1) + E * (4 + 4 * D + 4 * heads) + N * (4 * D + 8 * heads)
        res["gat_fwd"] = {"ms": ms, "GBps_model": b / ms / 1e6, "head_edges_per_s":
                          heads * E / ms * 1e3}
        y = fwd()
        dy = torch.randn_like(y)
        ms = timeit(lambda: torch.autograd.grad(y, (H, a_all), dy, retain_graph=True),
                    max(3, args.reps // 2), warm=1)
        res["gat_bwd"] = {"ms": ms}
    if want("gat_bf16"):
        heads, dh = 4, 75
        a_all = (torch.randn(heads, 2 * dh, device=dev, generator=g) * 0.1).requires_grad_(True)
        Hb = X.to(torch.bfloat16).requires_grad_(True)

        def fwdb():
            return ops.GATFn.apply(Hb, a_all, csr, heads, dh, 0.2, _lib.GNNEA_ACT_RELU, None)
        ms = timeit(fwdb, args.reps)
        b = 4 * (N + 1) + E * (4 + 2 * D + 4 * heads) + N * (2 * D + 8 * heads)
        res["gat_fwd_bf16"] = {"ms": ms, "GBps_model": b / ms / 1e6,
                               "head_edges_per_s": heads * E / ms * 1e3}
        yb = fwdb()
        dyb = torch.randn_like(yb)
        ms = timeit(lambda: torch.autograd.grad(yb, (Hb, a_all), dyb, retain_graph=True),
                    max(3, args.reps // 2), warm=1)
        res["gat_bwd_bf16"] = {"ms": ms}
        del Hb, yb, dyb
    if want("gcn_layer"):
        from layers.layers import GraphConvolution
        idx = torch.stack([torch.from_numpy(r), torch.from_numpy(c)]).to(dev)
        adj = torch.sparse_coo_tensor(idx, torch.from_numpy(v).to(dev), (N, N))
        torch.manual_seed(0)
        layer = GraphConvolution(D, D, 0.0, F.relu, True).to(dev)
        xg = X.clone().requires_grad_(True)

        def fb():
            out, _ = layer((xg, adj))
            out.backward(torch.ones_like(out))
        ms = timeit(fb, max(3, args.reps // 2), warm=1)
        res["gcn_layer_fwd_bwd"] = {"ms": ms}
    if want("sinkhorn"):
        from gnnea.sinkhorn import solve
        B = int(os.environ.get("SK_B", "3000"))
        M = torch.rand(B, B, device=dev, generator=g)
        la = torch.ones(B, dtype=torch.float64, device=dev)
        variants = [int(v) for v in os.environ.get("SK_VARIANTS", "0").split(",")]
        for name, mode, C in (("knopp_f32C", _lib.GNNEA_SK_KNOPP, M),
                              ("stab_f64C", _lib.GNNEA_SK_STAB, M.double())):
            for var in variants:
                best = []
                for rnd in range(3):  # interleaved rounds, median
                    ts = []
                    for it in (50, 550):
                        torch.cuda.synchronize()
                        s = time.perf_counter()
                        solve(mode, C, la, la, 0.01, -1.0, it, want_plan=False, batch=100,
                              variant=var)
                        torch.cuda.synchronize()
                        ts.append(time.perf_counter() - s)
                    best.append((ts[1] - ts[0]) / 500 * 1e6)
                key = "sinkhorn_" + name + ("" if var == 0 else "_v%d" % var) + \
                    ("" if B == 3000 else "_B%d" % B)
                res[key] = {"us_per_iter": float(np.median(best))}
    if want("l1"):
        # DBP15K-sized searches: get_neg of 4500 train entities over 30k, get_hits of 10.5k pairs
        from gnnea import l1
        V = torch.randn(30000, D, device=dev, generator=g) * 0.1
        Qn = V[:4500].contiguous()
        ms = timeit(lambda: l1.keys(Qn, V), args.reps)
        pd = 4500 * 30000 * D
        res["l1_keys_4500x30000"] = {"ms": ms, "Gpairdims_per_s": pd / ms / 1e6}
        ms = timeit(lambda: l1.topk(Qn, V, 126, 1), args.reps)
        res["get_neg_4500x30000_k125"] = {"ms": ms}
        Lh, Rh = V[:10500].contiguous(), V[10500:21000].contiguous()
        ms = timeit(lambda: l1.hits_ranks(Lh, Rh), args.reps)
        res["get_hits_10500"] = {"ms": ms, "Gpairdims_per_s": 2 * 10500 ** 2 * D / ms / 1e6}
    if want("margin"):
        # DBP15K-sized margin loss: t = 4500 train pairs, k = 125 negatives, 30k x 300 outputs
        from gnnea.margin import margin_loss
        Nm, tm, km = 30000, 4500, 125
        V = (torch.randn(Nm, D, device=dev, generator=g) * 0.05).requires_grad_(True)
        li = torch.randint(0, Nm, (tm,), device=dev, generator=g)
        ri = torch.randint(0, Nm, (tm,), device=dev, generator=g)
        n1 = torch.randint(0, Nm, (tm * km,), device=dev, generator=g)
        n2 = torch.randint(0, Nm, (tm * km,), device=dev, generator=g)
        nl, nr = li.repeat_interleave(km), ri.repeat_interleave(km)
        args_m = (li, ri, nl, n1, n2, nr, tm, km)

        def fused():
            loss = margin_loss(V, *args_m, checked=True)
            loss.backward()

        def torch_ops():  # the reference's op sequence on the device
            A = torch.sum(torch.abs(V[li] - V[ri]), 1).reshape(tm, 1) + 1.0
            B1 = torch.sum(torch.abs(V[nl] - V[n1]), 1).reshape(tm, km)
            B2 = torch.sum(torch.abs(V[n2] - V[nr]), 1).reshape(tm, km)
            loss = (F.relu(A - B1).sum() + F.relu(A - B2).sum()) / (2.0 * tm * km)
            loss.backward()
        res["margin_fwd_bwd_fused"] = {"ms": timeit(fused, args.reps)}
        res["margin_fwd_bwd_torch_ops"] = {"ms": timeit(torch_ops, args.reps)}
    if want("epoch"):
        # one run/train_ea.py epoch at DBP15K scale (2 x 15k entities, 2 x 50k triples, 4500
        # train pairs, 125 negatives): encode + decode + get_loss + backward + Adam, plus the
        # every-50-epochs get_neg and the eval get_hits (10.5k test pairs)
        from models.models_ea import EAModel
        from utils.eval_utils import get_hits

        class A:
            pass
        n15 = 15000
        tr15 = synth.kg_pair_triples(n15, 50000, 1000)
        r5, c5, v5 = synth.adjacency_coo(tr15, 2 * n15, reference_order=False)
        adj15 = torch.sparse_coo_tensor(torch.from_numpy(np.stack([r5, c5])),
                                        torch.from_numpy(v5), (2 * n15, 2 * n15)).to(dev)
        x15 = torch.from_numpy(synth.features(2 * n15, D)).to_sparse().to(dev)
        perm = np.random.default_rng(0).permutation(n15)
        train = np.stack([perm[:4500], perm[:4500] + n15], 1)
        test = np.stack([perm[4500:], perm[4500:] + n15], 1)
        for model in ("GCN", "HGCN", "GAT"):
            a = A()
            a.model, a.num_layers, a.dim, a.act, a.dropout, a.bias = model, 3, D, "relu", 0.0, 1
            a.n_heads, a.alpha, a.feat_dim, a.n_classes = 4, 0.2, D, D
            a.cuda, a.device, a.n_nodes, a.neg_num = 0, dev, 2 * n15, 125
            a.data = {"train": train, "test": test}
            torch.manual_seed(10086)
            mdl = EAModel(a).to(dev)
            opt = torch.optim.Adam(params=mdl.parameters(), lr=0.001)
            with torch.no_grad():
                o0 = mdl.decode(mdl.encode(x15, adj15), adj15)
            mdl.neg_right = mdl.get_neg(train[:, 0], o0, 125)
            mdl.neg2_left = mdl.get_neg(train[:, 1], o0, 125)

            def epoch():
                opt.zero_grad()
                o = mdl.decode(mdl.encode(x15, adj15), adj15)
                loss = mdl.get_loss(o, a.data, "train")
                loss.backward()
                opt.step()
            ms = timeit(epoch, args.reps)
            ms_neg = timeit(lambda: (mdl.get_neg(train[:, 0], o0, 125),
                                     mdl.get_neg(train[:, 1], o0, 125)), 3, warm=1)
            ms_hits = timeit(lambda: get_hits(o0, test), 3, warm=1)
            res["epoch_dbp15k_" + model] = {"ms_train_step": ms, "ms_get_neg_x2": ms_neg,
                                            "ms_get_hits": ms_hits}
    print(json.dumps(res, indent=1))
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
