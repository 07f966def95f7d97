"""Debug: the unstaged reduce-scatter (exchange.reduce_scatter) vs the per-slice one vs a host sum,
4-rank gloo rehearsal on one device at scale; and HipEngine.act_spmm_t vs fp64.
    python tools/dbg/rs_dbg.py [entities] [D]"""
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


def worker(rank, world, port, n, D, q):
    from gnnea import _lib, exchange, synth
    from gnnea.dist_graph import DistAdj
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    t = 10 * n
    tr = synth.kg_pair_triples(n, t, 3000)
    dadj = DistAdj.from_triples(tr, n, t, rank, world, dev)
    part = dadj.part
    g = torch.Generator(device=dev).manual_seed(rank)
    P = torch.randn(n, D, device=dev, generator=g)
    out = {"rank": rank}
    # host reference: every rank's P, summed in rank order over the group
    allP = [torch.empty(n, D) for _ in range(world)]
    dist.all_gather(allP, P.cpu())
    grp = part.group_ranks(part.kg)
    ref = sum(allP[r].double() for r in grp)[part.row0:part.row0 + part.n_rows]
    out["unstaged_rs"] = rel(dadj.reduce_scatter(P), ref)
    ranks, li, other = dadj._peers()
    o2 = torch.empty(part.n_rows, D, device=dev)
    pend = []
    for c0 in range(0, D, 64):
        c1 = min(D, c0 + 64)
        pend.append(exchange.reduce_scatter_start(P[:, c0:c1].contiguous(), dadj.group, ranks, li,
                                                  other, out=o2[:, c0:c1]))
    for p_ in pend:
        p_.finish()
    out["staged_rs"] = rel(o2, ref)
    # act_spmm_t vs fp64
    y = torch.randn(part.n_rows, D, device=dev, generator=g)
    dy = torch.randn(part.n_rows, D, device=dev, generator=g)
    gt = dadj.engine.act_spmm_t(dadj.csr, dy, y, _lib.GNNEA_ACT_RELU)
    from gnnea.dist import shard_coo
    r, c, v = shard_coo(tr, n, t, part)
    A = torch.sparse_coo_tensor(torch.from_numpy(np.stack([r, c])).long(),
                                torch.from_numpy(v).double(), (part.n_rows, n)).coalesce()
    g64 = (dy.double() * (y > 0).double()).cpu()
    out["act_spmm_t"] = rel(gt, torch.sparse.mm(A.t().coalesce(), g64))
    q.put(out)
    dist.destroy_process_group()


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    D = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ps = [ctx.Process(target=worker, args=(r, 4, port, n, D, q)) for r in range(4)]
    for p in ps:
        p.start()
    outs = [q.get(timeout=600) for _ in range(4)]
    for p in ps:
        p.join(60)
    for o in sorted(outs, key=lambda o: o["rank"]):
        print(json.dumps(o), flush=True)
