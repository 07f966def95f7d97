"""One fp32 (x3) GEMM shape of the EA step, a few launches (for rocprofv3 --pmc passes):
python tools/dbg/gemm_one.py {proj|proj600|dx|dw} [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))
from gnnea import ops  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
N, D = 2000000, 300
shape = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
if shape == "proj":
    X, W, b = (torch.randn(N, D, device=dev, generator=g), torch.randn(D, D, device=dev, generator=g),
               torch.randn(D, device=dev, generator=g))
    fn = lambda: ops.gemm(X, W, trans_b=True, bias=b, x3=True)  # noqa: E731
elif shape == "proj600":
    X, W = torch.randn(N, D, device=dev, generator=g), torch.randn(D, 2 * D, device=dev, generator=g)
    fn = lambda: ops.gemm(X, W, x3=True)  # noqa: E731
elif shape == "dx":
    X, W = torch.randn(N, 2 * D, device=dev, generator=g), torch.randn(2 * D, D, device=dev, generator=g)
    fn = lambda: ops.gemm(X, W, x3=True)  # noqa: E731
else:
    X = torch.randn(N, D, device=dev, generator=g)
    fn = lambda: ops.gemm(X, X, trans_a=True, x3=True)  # noqa: E731
for _ in range(reps):
    fn()
torch.cuda.synchronize()
print("done", shape)
