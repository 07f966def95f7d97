"""Per-iteration time of the row-sharded Sinkhorn driven on one device (W shards emulated)
against the unsharded log-domain solve, B = 15000 (bench.sinkhorn_large's problem)."""
import sys, os, time
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "gnn-mtl_amd"),
                os.path.join(os.path.dirname(__file__), "..", "..")]
import torch
from gnnea import _lib
from gnnea.sinkhorn import solve, solve_row_blocks
dev = torch.device("cuda:0")
B = 15000
g = torch.Generator(device="cpu").manual_seed(0)
X = (0.05 * torch.randn(B, 300, generator=g)).to(dev)
Y = (0.05 * torch.randn(B, 300, generator=g)).to(dev)
M = torch.cdist(X, Y)
M = (M / M.max()).contiguous()
a = torch.ones(B, dtype=torch.float64, device=dev)


def t(fn):
    fn(20)
    torch.cuda.synchronize()
    ts = []
    for n in (20, 120):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(n)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return (ts[1] - ts[0]) / 100 * 1e3


print("unsharded ms/iter %.3f" % t(lambda n: solve(_lib.GNNEA_SK_KNOPP, M, a, a, 0.01, -1.0, n,
                                                     want_plan=False, variant=1)))
for W in (1, 2, 8):
    splits = [B * k // W for k in range(1, W)]
    print("W=%d emulated ms/iter %.3f" % (W, t(lambda n: solve_row_blocks(
        M, a, a, 0.01, -1.0, n, splits, want_plan=False))), flush=True)
# one eighth of the rows alone: the per-rank work of an 8-GPU run (exchange excluded)
M8 = M[:B // 8].contiguous()
a8 = a[:B // 8]
print("rows/8 alone (W=1 driver) ms/iter %.3f" % t(lambda n: solve_row_blocks(
    M8, a8, a, 0.01, -1.0, n, [], want_plan=False)))
