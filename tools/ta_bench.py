"""Weight-gradient GEMM dW = Aᵀ·B at the EA-step shapes (gemm_ta.hip): fp32 2M x 300 x 300
(cfg-4) and bf16 4M x 300 x 300 (cfg-5); HIP events, median of reps, error vs fp64.

    python tools/ta_bench.py [--reps 21] [--out gpurun_out/ta_bench.json]
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
    ap.add_argument("--reps", type=int, default=21)
    ap.add_argument("--out", default=None)
    ap.add_argument("--wide", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    shapes = [("fp32 2M x 300 x 300", 2_000_000, 300, torch.float32),
              ("bf16 4M x 300 x 300", 4_000_000, 300, torch.bfloat16)]
    if args.wide:  # the 300- against the 600-wide dW on the same kernel, per-flop rate
        shapes += [("fp32 2M x 300 x 600", 2_000_000, 600, torch.float32),
                   ("fp32 4M x 300 x 300", 4_000_000, 300, torch.float32)]
    for name, K, N, dt in shapes:
        a = torch.randn(K, 300, device=dev, generator=g).to(dt)
        b = torch.randn(K, N, device=dev, generator=g).to(dt)
        ref = a.double().t() @ b.double()
        y = ops.gemm(a, b, trans_a=True, out_dtype=torch.float32)
        err = float((y.double() - ref).norm() / ref.norm())
        ms = timeit(lambda: ops.gemm(a, b, trans_a=True, out_dtype=torch.float32), args.reps)
        byts = K * (300 + N) * a.element_size()
        res[name] = {"ms": round(ms, 4), "rel_err_vs_fp64": err,
                     "TBps_compulsory": round(byts / (ms * 1e-3) / 1e12, 3),
                     "TFLOPs_product": round(2.0 * K * 300 * N / (ms * 1e-3) / 1e12, 1)}
        del a, b, ref, y
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)
    if args.out:
        with open(args.out, "a") as f:
            f.write(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
