"""fp32 GEMM shapes of the EA training step (cfg-4, 2M rows): gnnea.ops.gemm on the f32 MFMA and
through the three-way bf16 split (x3) vs hipBLASLt
(torch.mm) on the same operands; HIP events, median of reps.

    python tools/gemm_bench.py [--rows 2000000] [--reps 10] [--out gpurun_out/gemm_bench.json]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))

from gnnea import ops  # noqa: E402


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
    ap.add_argument("--rows", type=int, default=2000000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "gemm_bench.json"))
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    N, D = args.rows, 300
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(N, D, device=dev, generator=g)
    X2 = torch.randn(N, 2 * D, device=dev, generator=g)
    W = torch.randn(D, D, device=dev, generator=g)
    W2 = torch.randn(D, 2 * D, device=dev, generator=g)
    W3 = torch.randn(2 * D, D, device=dev, generator=g)
    b = torch.randn(D, device=dev, generator=g)
    cases = {
        "NT x.W^T+b [N,300]x[300,300]": (lambda x3: ops.gemm(X, W, trans_b=True, bias=b, x3=x3),
                                         lambda: torch.addmm(b, X, W.t()), 2.0 * N * D * D),
        "NN x.W [N,300]x[300,300]": (lambda x3: ops.gemm(X, W, x3=x3), lambda: torch.mm(X, W),
                                     2.0 * N * D * D),
        "NN x.[W^T|Kg] [N,300]x[300,600]": (lambda x3: ops.gemm(X, W2, x3=x3),
                                            lambda: torch.mm(X, W2), 4.0 * N * D * D),
        "NN [dh|dg].[W;Kg^T] [N,600]x[600,300]": (lambda x3: ops.gemm(X2, W3, x3=x3),
                                                  lambda: torch.mm(X2, W3), 4.0 * N * D * D),
        "TN dW = dY^T.X [300,N]x[N,300]": (lambda x3: ops.gemm(X, X, trans_a=True, x3=x3),
                                           lambda: torch.mm(X.t(), X), 2.0 * N * D * D),
    }
    res = {"rows": N}
    for name, (ours, ref, flop) in cases.items():
        t3 = timeit(lambda: ours(True), args.reps)
        t0 = timeit(lambda: ours(False), args.reps)
        t1 = timeit(ref, args.reps)
        r = ref().double()
        e0 = float((ours(False).double() - r).abs().max() / r.abs().max())
        e3 = float((ours(True).double() - r).abs().max() / r.abs().max())
        res[name] = {"x3_ms": round(t3, 4), "x3_TFLOPs": round(flop / t3 / 1e9, 1),
                     "f32mfma_ms": round(t0, 4), "f32mfma_TFLOPs": round(flop / t0 / 1e9, 1),
                     "hipblaslt_ms": round(t1, 4), "hipblaslt_TFLOPs": round(flop / t1 / 1e9, 1),
                     "rel_err_vs_hipblaslt": {"x3": e3, "f32mfma": e0}}
        print(name, res[name], flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
