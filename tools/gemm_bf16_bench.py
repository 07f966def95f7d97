"""bf16 projection GEMM of the cfg-5 GAT step (x·Wᵀ + b, [M, 300] x [300, 300], bf16 out):
gnnea.ops.gemm vs hipBLASLt (torch.nn.functional.linear); HIP events, median of reps; the
result checked against an fp32 product of the same bf16 operands.

    python tools/gemm_bf16_bench.py [--rows 4000000] [--reps 10]
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
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4000000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--k", type=int, default=300, help="inner dimension of the projection")
    ap.add_argument("--only-fwd", action="store_true", help="only x.W^T + b (mode sweeps)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    M, D, K = args.rows, 300, args.k
    X = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    W = (torch.randn(D, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(D, device=dev, generator=g) * 0.1
    Y = ops.gemm(X, W, trans_b=True, bias=b)
    ref = (X[:65536].float() @ W.float().t() + b)
    err = float(((Y[:65536].float() - ref).abs() / (ref.abs() + 1e-2)).max())
    io = 2 * (M * K + M * D + D * K)
    ms = timeit(lambda: ops.gemm(X, W, trans_b=True, bias=b), args.reps)
    if args.only_fwd:
        print(json.dumps({"rows": M, "K": K, "wres": os.environ.get("GNNEA_BF16_WRES", "1"),
                          "gnnea_ms": round(ms, 4), "gnnea_GBps_io": round(io / ms / 1e6, 1),
                          "max_rel_err_vs_fp32": err}))
        return
    bl = b.to(torch.bfloat16)
    ms_t = timeit(lambda: torch.nn.functional.linear(X, W, bl), args.reps)
    dY = torch.randn(M, D, device=dev, generator=g).to(torch.bfloat16)
    dW = ops.gemm(dY, X, trans_a=True)
    refw = dY[:65536].float().t() @ X[:65536].float()
    dW_part = ops.gemm(dY[:65536], X[:65536], trans_a=True)
    errw = float(((dW_part.float() - refw).abs() / (refw.abs() + 1e-1)).max())
    ms_w = timeit(lambda: ops.gemm(dY, X, trans_a=True), args.reps)
    ms_wt = timeit(lambda: torch.mm(dY.t(), X), args.reps)
    ms_x = timeit(lambda: ops.gemm(dY, W), args.reps)
    del dW
    print(json.dumps({"rows": M, "wres": os.environ.get("GNNEA_BF16_WRES", "1"),
                      "dW_ms": round(ms_w, 4), "dW_hipblaslt_ms": round(ms_wt, 4),
                      "dW_max_rel_err_vs_fp32": errw, "dX_ms": round(ms_x, 4),
                      "gnnea_ms": round(ms, 4), "gnnea_GBps_io": round(io / ms / 1e6, 1),
                      "gnnea_TFLOPs": round(2.0 * M * D * K / ms / 1e9, 1),
                      "hipblaslt_ms": round(ms_t, 4), "max_rel_err_vs_fp32": err}))


if __name__ == "__main__":
    main()
