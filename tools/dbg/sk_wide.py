"""B = 15000 KNOPP / STAB: scaling form (resident fp64 K, wide sweep) vs log-domain, ms per
iteration and agreement of the plans."""
import sys, os, time
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "gnn-mtl_amd"),
                os.path.join(os.path.dirname(__file__), "..", "..")]
import torch
from gnnea import _lib
from gnnea.sinkhorn import solve
dev = torch.device("cuda:0")
for B in (15000, 12000, 9000):
    g = torch.Generator(device="cpu").manual_seed(0)
    X = (0.05 * torch.randn(B, 300, generator=g)).to(dev)
    Y = (0.05 * torch.randn(B, 300, generator=g)).to(dev)
    M = torch.cdist(X, Y)
    M = (M / M.max()).contiguous()
    a = torch.ones(B, dtype=torch.float64, device=dev)
    for mode, name, w in ((_lib.GNNEA_SK_KNOPP, "knopp", 1.0), (_lib.GNNEA_SK_STAB, "stab", 1.0 / B)):
        aw = a * w
        C = M if mode == _lib.GNNEA_SK_KNOPP else M.double()
        out = {}
        for var in (0, 1):
            fn = lambda n: solve(mode, C, aw, aw, 0.01, -1.0, n, want_plan=False, batch=100,
                                 variant=var)
            fn(20)
            ts = []
            for n in (20, 120):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn(n)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            out[var] = (ts[1] - ts[0]) / 100 * 1e3
        r0 = solve(mode, C, aw, aw, 0.01, 1e-9, 200, variant=0)
        r1 = solve(mode, C, aw, aw, 0.01, 1e-9, 200, variant=1)
        d = ((r0.plan - r1.plan).abs().max() / r1.plan.abs().max()).item()
        print("B %d %s scaling %.3f ms  log %.3f ms  iters %d/%d  plan rel diff %.2e" % (
            B, name, out[0], out[1], r0.iters, r1.iters, d), flush=True)
        del r0, r1
