"""Debug: which side of halo_ab is wrong at scale?  (1) kernels alone on one process: the shard's
aggregation row-major vs slice-major whole vs per-slice column blocks, forward and transposed;
(2) a 4-rank gloo rehearsal: each rank's staged and unstaged GCN aggregation against the
one-process result over the whole KG.
    python tools/dbg/halo_ab_dbg.py [entities]"""
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
sys.path.insert(0, ROOT)


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max())


def kernels(n):
    from gnnea import _lib, ops, synth
    from gnnea.dist import Partition, shard_coo
    from gnnea.dist_graph import HipEngine
    dev = torch.device("cuda", 0)
    t = 10 * n
    tr = synth.kg_pair_triples(n, t, 3000)
    part = Partition(n, 0, 4, "rows")
    r, c, v = shard_coo(tr, n, t, part)
    csr = HipEngine().csr(r, c, v, part.n_rows, part.n_cols, dev)
    g = torch.Generator(device=dev).manual_seed(0)
    H = torch.randn(n, 300, device=dev, generator=g)
    relu = _lib.GNNEA_ACT_RELU
    y_row = ops.spmm(csr, H, relu)
    hs = ops.slice_pack(H)
    y_sl = ops.spmm_sliced(csr, hs, 300, relu)
    y_blk = torch.empty_like(y_row)
    for q in range(hs.shape[0]):
        c0, c1 = 64 * q, min(300, 64 * q + 64)
        ops.spmm_sliced(csr, hs[q].unsqueeze(0), c1 - c0, relu, out=y_blk[:, c0:c1])
    G = torch.randn(part.n_rows, 300, device=dev, generator=g)
    csrT = csr.transpose()
    p_row = ops.spmm(csrT, G)
    gs = ops.slice_pack(G)
    p_blk = torch.empty((n, 300), device=dev)
    for q in range(gs.shape[0]):
        c0, c1 = 64 * q, min(300, 64 * q + 64)
        p_blk[:, c0:c1] = ops.spmm_sliced(csrT, gs[q].unsqueeze(0), c1 - c0)
    # the reference: torch sparse on the host in fp64
    A = torch.sparse_coo_tensor(torch.from_numpy(np.stack([r, c])).long(),
                                torch.from_numpy(v).double(), (part.n_rows, n)).coalesce()
    y64 = torch.relu(torch.sparse.mm(A, H.double().cpu()))
    p64 = torch.sparse.mm(A.t().coalesce(), G.double().cpu())
    return {"y_row_vs_64": rel(y_row.cpu(), y64), "y_sl_vs_64": rel(y_sl.cpu(), y64),
            "y_blk_vs_64": rel(y_blk.cpu(), y64), "p_row_vs_64": rel(p_row.cpu(), p64),
            "p_blk_vs_64": rel(p_blk.cpu(), p64), "n_rows": part.n_rows, "nnz": int(r.size)}


def worker(rank, world, port, n, q):
    from gnnea import exchange, synth
    from gnnea.dist_graph import DistAdj
    import torch.nn.functional as F
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    t = 10 * n
    tr = synth.kg_pair_triples(n, t, 3000)
    dadj = DistAdj.from_triples(tr, n, t, rank, world, dev)
    g = torch.Generator(device=dev).manual_seed(0)
    Hall = torch.randn(2 * n, 300, device=dev, generator=g)
    p0, nr = dadj.part.global_row0, dadj.part.n_rows
    res = {}
    for mode in (False, True):
        exchange.STAGED = mode
        x = Hall[p0:p0 + nr].clone().requires_grad_()
        y = dadj.aggregate(x, F.relu)
        y.backward(torch.ones_like(y))
        res[mode] = (y.detach().cpu(), x.grad.cpu())
    # one-process reference on the whole graph (fp64 host)
    R, C, V = synth.adjacency_coo(tr, 2 * n, reference_order=False)
    A = torch.sparse_coo_tensor(torch.from_numpy(np.stack([R, C])).long(),
                                torch.from_numpy(V).double(), (2 * n, 2 * n)).coalesce()
    Hd = Hall.double().cpu()
    y64 = torch.relu(torch.sparse.mm(A, Hd))
    gy = (y64 > 0).double()
    gx = torch.sparse.mm(A.t().coalesce(), gy)
    out = {"rank": rank}
    for mode in (False, True):
        y, gxx = res[mode]
        out["staged" if mode else "unstaged"] = {"y": rel(y, y64[p0:p0 + nr]),
                                                 "dx": rel(gxx, gx[p0:p0 + nr])}
    q.put(out)
    dist.destroy_process_group()


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    print(json.dumps({"kernels": kernels(n)}), flush=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ps = [ctx.Process(target=worker, args=(r, 4, port, n, q)) for r in range(4)]
    for p in ps:
        p.start()
    outs = [q.get(timeout=600) for _ in range(4)]
    for p in ps:
        p.join(60)
    for o in sorted(outs, key=lambda o: o["rank"]):
        print(json.dumps(o), flush=True)
