"""STAB (sinkhorn_iteration) at B = 15000 through the scaling form: 100 iterations (profiling)."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "gnn-mtl_amd")]
import torch
from gnnea import _lib
from gnnea.sinkhorn import solve
dev = torch.device("cuda:0")
B = 15000
g = torch.Generator(device="cpu").manual_seed(0)
M = torch.rand(B, B, generator=g, dtype=torch.float64).to(dev)
a = torch.full((B,), 1.0 / B, dtype=torch.float64, device=dev)
for _ in range(2):
    solve(_lib.GNNEA_SK_STAB, M, a, a, 0.01, -1.0, 100, want_plan=False, batch=100, variant=0)
torch.cuda.synchronize()
print("done")
