"""A/B of the fp32 projection GEMMs of the EA steps (2M rows, K = 300): x·Wᵀ + b (300 wide,
row-major) and the HighWay layer's x·[Wᵀ | 0 | K_g] (620 wide, slice-major) through
gnnea.ops with whichever libgnnea build GNNEA_LIB_FILE names; median of HIP-event timings and
the norm-relative error against the fp64 product of the same operands.

    GNNEA_LIB_FILE=libgnnea_base.so python tools/dbg/gemm_as_ab.py
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))
from gnnea import ops  # noqa: E402


def timed(fn, reps=15):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in ev)[reps // 2]


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    M = 2_000_000
    x = torch.randn(M, 300, device=dev, generator=g)
    x /= x.norm(dim=1, keepdim=True)
    out = {"lib": os.environ.get("GNNEA_LIB_FILE", "libgnnea.so")}
    for name, N, sliced in (("x_Wt_b_300", 300, False), ("x_WtKg_620_sliced", 620, True)):
        W = torch.randn(N, 300, device=dev, generator=g) / 300 ** 0.5
        b = torch.randn(N, device=dev, generator=g) * 0.1
        if sliced:
            fn = lambda: ops.gemm_sliced(x, W, b)  # noqa: E731
        else:
            fn = lambda: ops.gemm(x, W, trans_b=True, bias=b)  # noqa: E731
        ms = timed(fn)
        y = fn()
        if sliced:
            S = y.shape[0]
            y = y.permute(1, 0, 2).reshape(M, S * 64)[:, :N]
        ref = x[:200000].double() @ W.double().t() + b.double()
        err = float((y[:200000].double() - ref).abs().max() / ref.abs().max())
        out[name] = {"ms": round(ms, 4), "TFLOPs_3products": round(3 * 2 * M * N * 300 / ms / 1e9, 1),
                     "norm_rel_err": err}
        del y
    print(json.dumps(out))


if __name__ == "__main__":
    main()
