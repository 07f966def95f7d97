"""Time the TA (weight-gradient) x3 GEMM dW = dY^T X at cfg-4 shape under GNNEA_X3TA_WGS."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))
import torch  # noqa: E402
from gnnea import ops  # noqa: E402
dev = torch.device("cuda:0")
X = torch.randn(2000000, 300, device=dev)
G = torch.randn(2000000, 300, device=dev)
for _ in range(3):
    ops.gemm(G, X, trans_a=True, x3=True)
torch.cuda.synchronize()
ts = []
for _ in range(10):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    ops.gemm(G, X, trans_a=True, x3=True)
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
print("wgs", os.environ.get("GNNEA_X3TA_WGS", "512"), "ms %.3f" % sorted(ts)[5])
