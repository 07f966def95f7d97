"""Run the x3 projection GEMM (cfg-4 shape) a few times: a short program for rocprofv3 --pmc.
GNNEA_X3_PIPE=0 selects the register-staged k_gemm_x3 instead of k_gemm_x3p."""
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
print("done")
