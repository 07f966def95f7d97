"""One Sinkhorn solve (for kernel traces): python tools/sk_one.py B variant iters [mode]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-mtl_amd"))
import torch  # noqa: E402
from gnnea import _lib  # noqa: E402
from gnnea.sinkhorn import solve  # noqa: E402

B, variant, n = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
mode = _lib.GNNEA_SK_STAB if len(sys.argv) > 4 and sys.argv[4] == "stab" else _lib.GNNEA_SK_KNOPP
dev = torch.device("cuda", 0)
g = torch.Generator(device="cpu").manual_seed(0)
M = torch.cdist(0.05 * torch.randn(B, 300, generator=g), 0.05 * torch.randn(B, 300, generator=g))
M = (M / M.max()).to(dev)
w = torch.full((B,), 1.0 if mode == _lib.GNNEA_SK_KNOPP else 1.0 / B, dtype=torch.float64,
               device=dev)
for _ in range(2):
    r = solve(mode, M if mode == _lib.GNNEA_SK_KNOPP else M.double(), w, w, 0.01, -1.0, n,
              want_plan=False, batch=100, variant=variant)
torch.cuda.synchronize()
print("iters", r.iters)
