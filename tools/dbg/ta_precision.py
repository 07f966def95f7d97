"""Where the cfg-4 weight / attention gradient errors come from (VERDICT r05 "do this" #2).

The product alone on identical fp32 inputs: dW = dhᵀ·x over K = 2M rows (k_gemm_ta_x3d, split-K
partials reduced in fp32 in split order) and da = sum_i ds_i (x) H_i (k_gat_da_part / _final)
against the fp64 product of the SAME fp32 operands, beside torch's fp32 product (hipBLASLt).
If the kernels are at ~1e-6 here, the 1e-4-level errors of the full-size tests come from the
fp32 intermediates upstream (H, Y, dh stored in fp32), not from the reductions.

    python tools/dbg/ta_precision.py
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))
from gnnea import ops  # noqa: E402


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max())


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    K, D = 2_000_000, 300
    x = torch.randn(K, D, device=dev, generator=g)
    x /= x.norm(dim=1, keepdim=True)
    out = {}
    # dense upstream gradient; the EA loss's: nonzero on ~1 % of rows, spread by one hop
    cases = {"dense": torch.randn(K, D, device=dev, generator=g) * 1e-3}
    m = (torch.rand(K, device=dev, generator=g) < 0.01).float()[:, None]
    cases["sparse_rows"] = torch.sign(torch.randn(K, D, device=dev, generator=g)) * m * 1e-4
    # a gradient correlated with x (the margin loss's sign sums are): strong cancellation
    cases["correlated"] = (x + 1e-3 * torch.randn(K, D, device=dev, generator=g)) * \
        torch.sign(torch.randn(K, 1, device=dev, generator=g))
    for name, dh in cases.items():
        ref = dh.double().t() @ x.double()
        ours = ops.gemm(dh, x, trans_a=True)
        t32 = dh.t() @ x
        out["dW_" + name] = {"ours": rel(ours, ref), "torch_fp32": rel(t32, ref)}
    H = torch.randn(K, D, device=dev, generator=g) * 0.1
    ds = torch.randn(K, 4, device=dev, generator=g) * 1e-3
    ref = (ds.double()[:, :, None] * H.double().view(K, 4, 75)).sum(0).reshape(-1)
    ours = ops.gat_da(H, ds, 4, 75)
    t32 = (ds[:, :, None] * H.view(K, 4, 75)).sum(0).reshape(-1)
    out["da"] = {"ours": rel(ours, ref), "torch_fp32": rel(t32, ref)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
