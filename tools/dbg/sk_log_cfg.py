"""ms / iteration of the unsharded log-domain KNOPP at B = 15000 under GNNEA_SK_LOG_CFG."""
import sys, os, time
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "gnn-mtl_amd"),
                os.path.join(os.path.dirname(__file__), "..", "..")]
import torch
from gnnea import _lib
from gnnea.sinkhorn import solve
dev = torch.device("cuda:0")
B = int(os.environ.get("SKB", "15000"))
g = torch.Generator(device="cpu").manual_seed(0)
X = (0.05 * torch.randn(B, 300, generator=g)).to(dev)
Y = (0.05 * torch.randn(B, 300, generator=g)).to(dev)
M = torch.cdist(X, Y)
M = (M / M.max()).contiguous()
a = torch.ones(B, dtype=torch.float64, device=dev)
fn = lambda n: solve(_lib.GNNEA_SK_KNOPP, M, a, a, 0.01, -1.0, n, want_plan=False, variant=1)
fn(20)
ts = []
for n in (20, 120):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn(n)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
print("B %d cfg %s ms/iter %.3f" % (B, os.environ.get("GNNEA_SK_LOG_CFG", "0"),
                                    (ts[1] - ts[0]) / 100 * 1e3))
