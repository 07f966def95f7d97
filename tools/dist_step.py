"""Row-sharded EA encoder training step (BASELINE.json configs[3]: HGCN-EA on the 2 x 1M-entity
synthetic KG pair, node-sharded with the RCCL halo exchange).

    python tools/dist_step.py [--model HGCN|GCN|GAT] [--steps 10] [--warmup 2] [--entities 1000000]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/dist_step.py

A step = the drop-in Encoder.encode + Decoder.decode (models/encoders.py, models/decoders.py;
HGCN: three HighWay graph convolutions; GCN: two graph convolutions + the 3-layer MLP decoder;
GAT: two 4-head graph attention layers + the MLP decoder, models/decoders.py:76-81) forward
on this rank's rows with a DistAdj, the EA margin loss (models/models_ea.py:103-123; t = 4500
synthetic train pairs, k = 125 negatives per side, fixed as the reference keeps them for 50
epochs) -- on one GPU the fused margin kernels on the output, on N > 1 the column-sharded loss
(gnnea/dist_loss.py: all-to-all to column blocks, one all-reduce of the per-term partials) --
its backward, and the one-bucket RCCL all-reduce of the weight gradients.  Prints one JSON line
on rank 0: the median per-step time, plus (after the timed steps) per-kernel-class GPU time of
attributed steps (gnnea/profile.py), the all-reduce time and the GFX clock during the timed steps.
"""
import argparse
import json
import os
import sys
import time
import types

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))

from gnnea import synth  # noqa: E402
from gnnea.dist_graph import DistAdj, allreduce_grads  # noqa: E402


def build(model, n, rank, world, device, seed=10086, dtype=torch.float32):
    from models.decoders import model2decoder
    from models.encoders import model2encoder
    a = types.SimpleNamespace(model=model, num_layers=3, dim=300, act="relu", dropout=0.0,
                              bias=1, n_heads=4, alpha=0.2, feat_dim=300, n_classes=300,
                              cuda=0, device=device)
    torch.manual_seed(seed)  # replicated weights on every rank (run/train_ea.py:10)
    enc = model2encoder[model](a).to(device=device, dtype=dtype)
    dec = model2decoder[model](a).to(device=device, dtype=dtype)
    t = synth.CONFIGS["cfg4"]["t"] if n == synth.CONFIGS["cfg4"]["n"] else 10 * n
    tr = synth.kg_pair_triples(n, t, synth.CONFIGS["cfg4"]["n_rel"])
    dadj = DistAdj.from_triples(tr, n, t, rank, world, device)
    return enc, dec, dadj


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="HGCN", choices=("HGCN", "GCN", "GAT"))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--entities", type=int, default=synth.CONFIGS["cfg4"]["n"])
    ap.add_argument("--dtype", default="f32", choices=("f32", "bf16"),
                    help="feature / weight storage (bf16: configs[4]'s dtype, fp32 arithmetic)")
    ap.add_argument("--attribute", type=int, default=3,
                    help="steps run after the timed ones with HIP events around every launch "
                         "(the per-class kernel times); 0 for profiler runs")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import datetime
        dist.init_process_group("nccl", device_id=dev, timeout=datetime.timedelta(
            seconds=float(os.environ.get("GNNEA_PG_TIMEOUT_S", "300"))))
    res = measure(args.model, args.entities, rank, world, dev, args.steps, args.warmup,
                  torch.bfloat16 if args.dtype == "bf16" else torch.float32,
                  attribute=args.attribute)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def loss_indices(n, t=4500, k=125, seed=7):
    """Synthetic EA supervision on the cfg pair: t aligned pairs (left in KG1, right = left + n in
    KG2: gnnea.synth gives both KGs the same generator) and k negatives per side, in the layout
    EAModel keeps (models/models_ea.py:80-92): neg_left = left repeated, neg2_right = right
    repeated, neg_right / neg2_left drawn from all entities."""
    import numpy as np
    rng = np.random.default_rng(seed)
    t = min(t, n)
    left = rng.choice(n, t, replace=False).astype(np.int64)
    right = left + n
    return ([left, right, np.repeat(left, k), rng.integers(0, 2 * n, t * k),
             rng.integers(0, 2 * n, t * k), np.repeat(right, k)], t, k)


def measure(model, n, rank, world, dev, steps, warmup, dtype=torch.float32, attribute=3,
            min_steps=21, min_warmup=3):
    """Time `steps` sharded training steps (after `warmup`), max over ranks; returns the summary
    (the same dict on every rank).  Every rank runs the same collective sequence.  SURVEY.md §8d
    timing asks for >= 3 warm-ups and >= 21 timed steps (min_warmup / min_steps; lower only for
    the one-device rehearsal, where the rate means nothing)."""
    from gnnea.profile import ClockSampler, KernelClassTimer
    t0 = time.time()
    enc, dec, dadj = build(model, n, rank, world, dev, dtype=dtype)
    part = dadj.part
    g = torch.Generator(device=dev).manual_seed(1 + rank)
    x = torch.randn(part.n_rows, 300, device=dev, generator=g)
    x /= x.norm(dim=1, keepdim=True)
    x = x.to(dtype)
    idx, t_, k_ = loss_indices(n)
    params = list(enc.parameters()) + list(dec.parameters())
    print("rank %d: %d rows, %d nnz, setup %.1fs" % (rank, part.n_rows, dadj.nnz,
                                                     time.time() - t0), file=sys.stderr)
    if world > 1:
        from gnnea.dist_loss import sharded_margin_loss

        def loss_of(out):
            return sharded_margin_loss(out, dadj, *idx, t_, k_)
    else:
        from gnnea.margin import margin_loss

        def loss_of(out):
            return margin_loss(out, *idx, t_, k_)  # (bf16 rows read as bf16)
    ar = []

    def step(ar_events=False):
        for p in params:
            p.grad = None
        out = dec.decode(enc.encode(x, dadj), dadj)
        loss_of(out).backward()
        if world > 1:
            if ar_events:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                allreduce_grads(params)
                b.record()
                ar.append((a, b))
            else:
                allreduce_grads(params)

    # SURVEY.md §8d timing: >= 3 warm-ups, then per-step HIP events on the launching stream,
    # median of >= 21 steps (max over ranks step by step); the wall-clock mean is kept beside it
    warmup, steps = max(min_warmup, warmup), max(min_steps, steps)
    wev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(warmup)]
    for a, b in wev:  # timed too: first-use costs (allocator growth, lazy transposes) show here
        a.record()
        step()
        b.record()
    torch.cuda.synchronize()
    warm_ms = [round(a.elapsed_time(b), 2) for a, b in wev]
    if world > 1:
        dist.barrier()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(steps)]
    with ClockSampler(dev) as clk:
        t1 = time.perf_counter()
        for a, b in evs:
            a.record()
            step()
            b.record()
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    # (host tensors under gloo: the one-device rehearsal)
    red_dev = "cpu" if world > 1 and dist.get_backend() == "gloo" else dev
    per = torch.tensor([a.elapsed_time(b) for a, b in evs] + [(time.perf_counter() - t1) * 1e3],
                       dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(per, op=dist.ReduceOp.MAX)
    per = per.cpu()
    wall_ms = float(per[-1]) / steps
    per = per[:-1]
    ms = float(per.median())
    if rank == 0:
        print("warm-up ms: %s; per-step ms: %s" % (warm_ms, " ".join("%.2f" % v
                                                                  for v in per.tolist())),
              file=sys.stderr)
    # attribution (after the timed steps): libgnnea kernel classes + the gradient all-reduce
    attrib = None
    if attribute > 0:
        sev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(attribute)]
        with KernelClassTimer() as kt:
            for a, b in sev:
                a.record()
                step(ar_events=True)
                b.record()
            cls = kt.totals_ms()
        st_ms = sum(a.elapsed_time(b) for a, b in sev) / attribute
        attrib = {k: round(v / attribute, 3) for k, v in sorted(cls.items())}
        if ar:
            attrib["allreduce"] = round(sum(a.elapsed_time(b) for a, b in ar) / attribute, 3)
        attrib["step_ms_attributed"] = round(st_ms, 3)
        attrib["other_ms"] = round(st_ms - sum(v for k, v in attrib.items()
                                               if k not in ("step_ms_attributed",)), 3)
        attrib["note"] = ("HIP events around every libgnnea launch of %d steps after the timed "
                          "ones (rank 0); other = torch elementwise kernels, copies, the loss's "
                          "and the halo's collectives, gaps" % attribute)
    nnz = torch.tensor([float(dadj.nnz)], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(nnz)  # row shards: every edge of the graph once
    layers = {"HGCN": "3 HighWay graph convolutions",
              "GCN": "2 graph convolutions + 3-layer MLP decoder",
              "GAT": "2 four-head graph attention layers + 3-layer MLP decoder"}[model]
    return {"metric": "EA encoder training steps/s", "model": model + "-EA (encode + decode, "
            "%s, EA margin loss t=%d k=%d, fwd + bwd + gradient all-reduce)" % (layers, t_, k_),
            "graph": "2x%d entities, %d nnz" % (n, int(nnz)),
            "dtype": "bf16 storage, f32 arithmetic" if dtype == torch.bfloat16 else "f32",
            "n_gpus": world, "steps": steps, "warmup": warmup, "ms_per_step": round(ms, 3),
            "timing": "median of per-step HIP events (max over ranks)",
            "ms_min_max": [round(float(per.min()), 3), round(float(per.max()), 3)],
            "ms_wall_mean": round(wall_ms, 3), "ms_warmup_steps_rank0": warm_ms,
            "steps_per_s": round(1e3 / ms, 2),
            # 3 aggregations forward + 3 transposed aggregations backward per step
            "edges_per_s_fwd_bwd": round(6 * float(nnz) / ms * 1e3, 1),
            "kernel_classes_ms_per_step": attrib, "gfx_clock_timed_steps_rank0": clk.summary(),
            "loss": "margin loss on the output (gnnea.margin)" if world == 1 else
            "column-sharded margin loss (gnnea.dist_loss)",
            "partition": "single GPU" if world == 1 else
            "rows: 2 KG groups of %d GPUs, RCCL halo all-gather (fwd) + reduce-scatter (bwd) "
            "per layer, one-bucket gradient all-reduce" % part.g}


if __name__ == "__main__":
    main()
