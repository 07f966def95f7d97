"""Time the x3p projection GEMM (cfg-4 shape) in the current GNNEA_X3P_MODE (debug tool)."""
import os
import sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))
from gnnea import ops  # noqa

dev = torch.device("cuda:0")
X = torch.randn(2000000, 300, device=dev)
W = torch.randn(300, 300, device=dev)
for _ in range(3):
    ops.gemm(X, W, trans_b=True, x3=True)
torch.cuda.synchronize()
ts = []
for _ in range(10):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    ops.gemm(X, W, trans_b=True, x3=True)
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
print("mode", os.environ.get("GNNEA_X3P_MODE", "0"), "ms %.3f" % sorted(ts)[5])
