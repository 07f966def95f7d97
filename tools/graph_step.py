"""A whole EA training iteration captured as ONE HIP graph (torch.cuda.CUDAGraph over the drop-in
modules): encode + decode + the EA margin loss + backward + the Adam update of
run/train_ea.py:55-66, replayed with a single launch per step.

At DBP15K scale (2 x 15k entities, BASELINE configs[1] / [2]) a step is ~150 small kernels and
the eager step is bound by their launches from Python (each libgnnea launch goes through ctypes);
the graph replays the same kernels, in the same order, on the same buffers.  The tool checks
that: from one snapshot of weights and optimizer state it runs one eager step and one graph
replay and compares the losses, every gradient and every updated weight (the kernels are the
same, so the difference is expected to be exactly zero), then times eager steps against replays
(HIP events, median).

    python tools/graph_step.py [--model GCN|HGCN|GAT] [--entities 15000] [--steps 50]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))
sys.path.insert(0, ROOT)

from gnnea import synth  # noqa: E402
from gnnea.dist_graph import DistAdj  # noqa: E402
from gnnea.margin import margin_loss  # noqa: E402
from tools.dist_step import loss_indices  # noqa: E402


def build(model, n, t, dev, seed=10086):
    import types
    from models.decoders import model2decoder
    from models.encoders import model2encoder
    a = types.SimpleNamespace(model=model, num_layers=3, dim=300, act="relu", dropout=0.0,
                              bias=1, n_heads=4, alpha=0.2, feat_dim=300, n_classes=300,
                              cuda=0, device=dev)
    torch.manual_seed(seed)
    enc = model2encoder[model](a).to(dev)
    dec = model2decoder[model](a).to(dev)
    tr = synth.kg_pair_triples(n, t, synth.CONFIGS["dbp15k"]["n_rel"])
    return enc, dec, DistAdj.from_triples(tr, n, t, 0, 1, dev)


def wall_ms(fn, reps):
    """Host wall clock per step over reps back-to-back steps (synchronized at both ends): what a
    training loop sees when the host, not the device, is the bottleneck."""
    import time
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def median_ms(fn, reps):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(reps)]
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in evs]))


def run(model, n, t, steps, dev):
    enc, dec, dadj = build(model, n, t, dev)
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(2 * n, 300, device=dev, generator=g)
    x /= x.norm(dim=1, keepdim=True)
    idx, t_, k_ = loss_indices(n)
    params = list(enc.parameters()) + list(dec.parameters())
    # (capturable: the step counter and the bias corrections stay on the device)
    opt = torch.optim.Adam(params, lr=0.005, capturable=True)

    def step():
        out = dec.decode(enc.encode(x, dadj), dadj)
        loss = margin_loss(out, *idx, t_, k_)
        loss.backward()
        opt.step()
        return loss

    def eager():
        opt.zero_grad(set_to_none=False)
        return step()

    # warm-up on a side stream (first-use allocations, the CSR transposes and the margin-loss
    # incidence are built and cached here, outside the capture)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(3):
            eager()
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()

    graph = torch.cuda.CUDAGraph()
    opt.zero_grad(set_to_none=False)
    with torch.cuda.graph(graph):
        static_loss = step()

    def replay():
        opt.zero_grad(set_to_none=False)
        graph.replay()

    # parity: one eager step and one replay from the same snapshot (weights + Adam state)
    snap_p = [p.detach().clone() for p in params]
    snap_s = {id(p): {k: v.clone() for k, v in opt.state[p].items()} for p in params}

    def restore():
        with torch.no_grad():
            for p, v in zip(params, snap_p):
                p.copy_(v)
            for p in params:
                for k, v in snap_s[id(p)].items():
                    opt.state[p][k].copy_(v)

    restore()
    le = eager().detach().clone()
    ge = [p.grad.detach().clone() for p in params]
    pe = [p.detach().clone() for p in params]
    restore()
    replay()
    torch.cuda.synchronize()
    lg = static_loss.detach().clone()
    gg = [p.grad.detach().clone() for p in params]
    pg = [p.detach().clone() for p in params]

    def rel(a, b):
        d = float((a.double() - b.double()).abs().max())
        m = float(b.double().abs().max())
        return d / m if m > 0 else d
    parity = {"loss_eager": float(le), "loss_graph": float(lg), "loss_rel": rel(lg, le),
              "grad_max_rel": max(rel(a, b) for a, b in zip(gg, ge)),
              "param_max_rel": max(rel(a, b) for a, b in zip(pg, pe))}

    eager_ms = median_ms(eager, steps)
    graph_ms = median_ms(replay, steps)
    eager_wall = wall_ms(eager, steps)
    graph_wall = wall_ms(replay, steps)
    return {"model": model + "-EA", "graph": "2x%d entities, %d triples per KG, %d nnz"
            % (n, t, dadj.nnz), "step": "encode + decode + margin loss (t=%d, k=%d) + backward "
            "+ Adam (capturable)" % (t_, k_), "steps": steps,
            "eager_ms": round(eager_ms, 4), "graph_ms": round(graph_ms, 4),
            "speedup": round(eager_ms / graph_ms, 3),
            "eager_wall_ms": round(eager_wall, 4), "graph_wall_ms": round(graph_wall, 4),
            "speedup_wall": round(eager_wall / graph_wall, 3), "parity": parity,
            "timing": "median of per-step HIP events (device timeline); *_wall: host wall clock "
                      "per step over the same number of back-to-back steps"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="all", choices=("all", "GCN", "HGCN", "GAT"))
    ap.add_argument("--entities", type=int, default=synth.CONFIGS["dbp15k"]["n"])
    ap.add_argument("--triples", type=int, default=synth.CONFIGS["dbp15k"]["t"])
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    models = ("GCN", "HGCN", "GAT") if args.model == "all" else (args.model,)
    for m in models:
        print(json.dumps(run(m, args.entities, args.triples, args.steps, dev)), flush=True)


if __name__ == "__main__":
    main()
