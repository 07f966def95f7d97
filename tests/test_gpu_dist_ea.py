"""The drop-in EAModel (models/models_ea.py:88-124) on a row-sharded graph, as run/train_ea.py
drives it (encode, decode, get_neg x 2 every 50 epochs, get_loss, backward, compute_metrics),
rehearsed at world 2 / 4 on ONE MI355X (gloo, exchanges staged through host memory, HIP kernels):

* get_neg / compute_metrics on the rank's output rows take the sharded search
  (gnnea.dist_search: query all-reduce, per-rank top-k merged by (distance, index), per-rank
  pair-rank counts summed) and must equal the single-GPU search on the GATHERED output index for
  index / count for count;
* get_loss on the rank's rows takes the column-sharded loss (gnnea.dist_loss); loss and the
  all-reduced parameter gradients vs the same model in one process on the whole graph (fp32
  kernels on both sides; gradients relative to the model's largest gradient entry, 1e-4: the
  sharded loss sums its distances in fp64, the one-process margin kernel in fp32 — a hinge
  decision differing between them would show here).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N_KG, T_KG, D = 64, 240, 132


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, model_name, q, dtype="f32"):
    import sys
    import types
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "gnn-mtl_amd"))
    from gnnea import synth
    from gnnea.dist_graph import DistAdj, allreduce_grads
    from models.models_ea import EAModel
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        tr = synth.kg_pair_triples(N_KG, T_KG, 20)
        R, C, V = synth.adjacency_coo(tr, 2 * N_KG, reference_order=False)
        adj_full = torch.sparse_coo_tensor(torch.from_numpy(np.stack([R, C])).long(),
                                           torch.from_numpy(V), (2 * N_KG, 2 * N_KG)).to(dev)
        X = torch.from_numpy(synth.features(2 * N_KG, D, seed=5)).float().to(dev)
        rng = np.random.default_rng(4)
        left = rng.choice(N_KG, 12, replace=False)
        pairs = np.stack([left, left + N_KG], 1).astype(np.int64)
        k = 5
        args = types.SimpleNamespace(model=model_name, num_layers=2, dim=D, act="relu",
                                     dropout=0.0, bias=1, n_heads=4, alpha=0.2, feat_dim=D,
                                     n_classes=D, cuda=0, device=dev, n_nodes=2 * N_KG,
                                     neg_num=k, data={"train": pairs, "test": pairs})
        data = {"train": pairs, "test": pairs}
        dt = torch.bfloat16 if dtype == "bf16" else torch.float32
        X = X.to(dt)
        torch.manual_seed(10086)
        ref = EAModel(args).to(dev, dt)
        torch.manual_seed(10086)
        mdl = EAModel(args).to(dev, dt)
        dadj = DistAdj.from_triples(tr, N_KG, T_KG, rank, world, dev)
        p0, nr = dadj.part.global_row0, dadj.part.n_rows
        # sharded forward; the search on the rank's rows vs the one-GPU search on the gathered rows
        enc = mdl.encode(X[p0:p0 + nr], dadj)
        enc.retain_grad()
        out = mdl.decode(enc, dadj)
        full = dadj.gather_rows(out).detach()
        res = {}
        for name, ill in (("neg_right", pairs[:, 0]), ("neg2_left", pairs[:, 1])):
            got = mdl.get_neg(ill, out, k)
            want = EAModel.get_neg(None, ill, full, k)
            res[name] = bool((got == want).all())
            setattr(mdl, name, got)
            setattr(ref, name, got)
        res["hits"] = mdl.compute_metrics(out, data, "train") == \
            EAModel.compute_metrics(None, full, data, "train")
        # the sharded loss and gradients vs the one-process model on the whole graph
        loss = mdl.get_loss(out, data, "train")
        loss.backward()
        # each rank's partial of every parameter gradient, rounded to the parameter dtype: for a
        # gradient that is analytically zero (the last Linear's bias: the L1 loss is translation
        # invariant) the partials cancel across ranks and what is left is their rounding, at
        # most half an ulp of each -- the bound that gradient is held to
        ulp = 2.0 ** -8 if dt == torch.bfloat16 else 2.0 ** -24
        bounds = {n: (p.grad.detach().float().abs() * ulp).cpu() for n, p in mdl.named_parameters()
                  if p.grad is not None}
        for b_ in bounds.values():
            dist.all_reduce(b_)
        allreduce_grads(list(mdl.parameters()))
        enc_r = ref.encode(X, adj_full)
        enc_r.retain_grad()
        out_r = ref.decode(enc_r, adj_full)
        loss_r = ref.get_loss(out_r, data, "train")
        loss_r.backward()

        def rel(a, b):
            a, b = a.detach().double().cpu(), b.detach().double().cpu()
            return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))
        res["out"] = rel(full, out_r)
        res["loss"] = abs(float(loss.detach()) - float(loss_r.detach())) / abs(float(loss_r.detach()))
        # each parameter's error against the largest gradient entry of the model: the last
        # Linear's bias gradient is a sum of +-c sign(x_a - x_b) pairs that cancels exactly (L1
        # distances are translation invariant), so its own scale is rounding noise
        gmax = max(float(pr.grad.abs().max()) for pr in ref.parameters() if pr.grad is not None)
        res["grad_errs"], res["zero_grads"] = {}, {}
        for (n, p), pr in zip(mdl.named_parameters(), ref.parameters()):
            if pr.grad is None:
                continue
            diff = (p.grad.double() - pr.grad.double()).abs().cpu()
            if float(pr.grad.abs().max()) < 1e-3 * gmax:  # analytically zero: the rounding bound
                res["zero_grads"][n] = float((diff - bounds[n].double()
                                              - pr.grad.double().abs().cpu()).max()) / gmax
            else:
                res["grad_errs"][n] = float(diff.max()) / gmax
        res["grads"] = max(res["grad_errs"].values())
        res["enc_grad"] = rel(enc.grad, enc_r.grad[p0:p0 + nr])
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("model_name,dtype", [("GCN", "f32"), ("HGCN", "f32"), ("GAT", "f32"),
                                              ("GAT", "bf16")])
def test_eamodel_sharded_rehearsal(device, world, model_name, dtype):
    """GAT / bf16: configs[4]'s model and storage dtype (two 4-head GAT layers, the MLP decoder,
    bf16 projections, halo and -- world 4, staged -- the bf16 GAT slice tables); bf16 judged at
    the storage tolerances of tests/test_gpu_scale_cfg5.py (outputs 1e-2, gradients 2e-2 of the
    largest, loss 1e-2), the searches index-exact as in fp32 (both run on the same output)."""
    import queue
    import time
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, model_name, q, dtype))
             for r in range(world)]
    for p in procs:
        p.start()
    out, t0 = [], time.time()
    while len(out) < world:
        try:
            out.append(q.get(timeout=1))
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs) or time.time() - t0 > 240:
                for p in procs:
                    p.kill()
                raise AssertionError("rank failed: %s" % [p.exitcode for p in procs])
    for p in procs:
        p.join(60)
    for rank, r in out:
        assert r["neg_right"] and r["neg2_left"] and r["hits"], (rank, r)
        t_out, t_loss, t_grad = (1e-2, 1e-2, 2e-2) if dtype == "bf16" else (1e-4, 1e-5, 1e-4)
        bad = {k: v for k, v in r["grad_errs"].items() if v >= t_grad}
        print(model_name, dtype, world, rank, "out %.2e loss %.2e grads %.2e enc_grad %.2e"
              % (r["out"], r["loss"], r["grads"], r["enc_grad"]), "zero-gradient excess over "
              "the partials' rounding bound:", r["zero_grads"])
        assert all(v <= 1e-6 for v in r["zero_grads"].values()), (rank, r["zero_grads"])
        assert r["out"] < t_out and r["loss"] < t_loss and r["grads"] < t_grad, \
            (rank, r["out"], r["loss"], r["enc_grad"], bad)
