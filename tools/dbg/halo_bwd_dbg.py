"""Debug: the unstaged HaloAggregateFn backward at scale, step by step, 4-rank gloo rehearsal.
    python tools/dbg/halo_bwd_dbg.py [entities]"""
import json
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max())


def worker(rank, world, port, n, order, q):
    from gnnea import _lib, exchange, synth
    from gnnea.dist_graph import DistAdj, HaloAggregateFn
    from gnnea.dist import shard_coo
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    t = 10 * n
    tr = synth.kg_pair_triples(n, t, 3000)
    dadj = DistAdj.from_triples(tr, n, t, rank, world, dev)
    part = dadj.part
    g = torch.Generator(device=dev).manual_seed(0)
    Hall = torch.randn(2 * n, 300, device=dev, generator=g)
    p0, nr = part.global_row0, part.n_rows
    R, C, V = synth.adjacency_coo(tr, 2 * n, reference_order=False)
    A = torch.sparse_coo_tensor(torch.from_numpy(np.stack([R, C])).long(),
                                torch.from_numpy(V).double(), (2 * n, 2 * n)).coalesce()
    y64 = torch.relu(torch.sparse.mm(A, Hall.double().cpu()))
    gx = torch.sparse.mm(A.t().coalesce(), (y64 > 0).double())
    out = {"rank": rank, "order": order}
    if order == "manual_first":
        exchange.STAGED = False
        full, _ = dadj.halo(Hall[p0:p0 + nr])
        y = dadj.engine.spmm(dadj.csr, full, _lib.GNNEA_ACT_RELU)
        out["y"] = rel(y, y64[p0:p0 + nr])
        P = dadj.engine.act_spmm_t(dadj.csr, torch.ones_like(y), y, _lib.GNNEA_ACT_RELU)
        r, c, v = shard_coo(tr, n, t, part)
        As = torch.sparse_coo_tensor(torch.from_numpy(np.stack([r, c])).long(),
                                     torch.from_numpy(v).double(), (nr, n)).coalesce()
        out["P"] = rel(P, torch.sparse.mm(As.t().coalesce(), (y.double().cpu() > 0).double()))
        dx = dadj.reduce_scatter(P)
        out["dx_manual"] = rel(dx, gx[p0:p0 + nr])
    exchange.STAGED = False
    x = Hall[p0:p0 + nr].clone().requires_grad_()
    y = HaloAggregateFn.apply(x, dadj, _lib.GNNEA_ACT_RELU)
    y.backward(torch.ones_like(y))
    torch.cuda.synchronize()
    out["dx_autograd"] = rel(x.grad, gx[p0:p0 + nr])
    q.put(out)
    dist.destroy_process_group()


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    for order in ("autograd_first", "manual_first"):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        ps = [ctx.Process(target=worker, args=(r, 4, port, n, order, q)) for r in range(4)]
        for p in ps:
            p.start()
        outs = [q.get(timeout=600) for _ in range(4)]
        for p in ps:
            p.join(60)
        for o in sorted(outs, key=lambda o: o["rank"]):
            print(json.dumps(o), flush=True)
