"""Per-rank aggregation time of the multi-GPU partitions, measured on ONE MI355X.

    python tools/scale_probe.py [--n 1000000] [--reps 10] [--out gpurun_out/scale_probe.json]

For world sizes W = 1, 2, 4, 8 this builds the shard that rank r of W would own
(gnnea.dist.KGShard, feature-column partition: no exchange in the aggregation) and times its
SpMM alone on the one device (the slice-major table where bench.py uses it, else row-major).  Ranks of the feature partition are independent, so the slowest
rank's time bounds the W-GPU step: predicted value = nnz(A) / max_r t_r.  This is a prediction
for the driver's 1/2/4/8-GPU run, not a measurement of it (8-GPU runs are the driver's).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))

from gnnea import _lib, ops, synth  # noqa: E402
from gnnea.dist import KGShard  # noqa: E402


def timeit(fn, reps, warm=3):
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
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--dtype", default="f32", choices=("f32", "bf16"))
    ap.add_argument("--kind", default="tiles", choices=("tiles", "features"),
                    help="exchange-free partition inside a KG group (bench.py --partition)")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "scale_probe.json"))
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n, t = args.n, 10 * args.n
    D = 300
    dt = torch.float32 if args.dtype == "f32" else torch.bfloat16
    res = {"n": n, "D": D, "dtype": args.dtype, "partition": args.kind, "worlds": {}}
    for W in [int(w) for w in args.worlds.split(",")]:
        # ranks of one KG group differ only in their column slice; probe the first and last
        ranks = [0] if W <= 2 else [0, W // 2 - 1]
        per = []
        for rank in ranks:
            sh = KGShard(n, t, 3000, rank, W, dev, kind=args.kind, D=D)
            Dl = sh.part.col1 - sh.part.col0
            g = torch.Generator(device=dev).manual_seed(1 + rank)
            h = torch.randn(sh.n_cols, Dl, device=dev, generator=g).to(dt)
            y = torch.empty(sh.n_rows, Dl, device=dev, dtype=dt)
            es = 2 if dt == torch.bfloat16 else 4
            byt = 4 * (sh.n_rows + 1) + 8 * sh.nnz + es * sh.nnz * Dl + es * sh.n_rows * Dl
            ent = {"rank": rank, "rows": sh.n_rows, "nnz": sh.nnz, "cols": Dl,
                   "launches": len(ops._blocks(sh.csr, h))}
            ms = timeit(lambda: ops.spmm(sh.csr, h, _lib.GNNEA_ACT_RELU, out=y), args.reps)
            ent["auto"] = {"ms": round(ms, 4), "GBps_gather_model": round(byt / ms / 1e6, 1)}
            ent["ms"] = ent["auto"]["ms"]
            if ops.use_sliced(sh.n_cols, Dl, dt):  # what bench.py runs: the slice-major table
                hs = ops.slice_pack(h)
                ms = timeit(lambda: ops.spmm_sliced(sh.csr, hs, Dl, _lib.GNNEA_ACT_RELU, out=y),
                            args.reps)
                ent["sliced"] = {"ms": round(ms, 4),
                                 "GBps_gather_model": round(byt / ms / 1e6, 1)}
                ent["ms"] = ent["sliced"]["ms"]
                del hs
            per.append(ent)
            print(W, per[-1], flush=True)
            del sh, h, y
            torch.cuda.empty_cache()
        E = 41999552 if n == 1000000 else None
        tmax = max(p["ms"] for p in per)
        total_units = E if E else per[0]["nnz"] * (2 if W > 1 else 1)
        res["worlds"][W] = {"ranks": per, "predicted_edges_per_s": round(total_units / tmax * 1e3, 1)}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
