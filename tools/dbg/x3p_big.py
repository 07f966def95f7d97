"""x3p at 8-wave tile sizes (M >= 65536) vs fp64 on sampled rows: plain, bias, 600-wide, dual."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))
import torch  # noqa: E402
from gnnea import ops  # noqa: E402
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(3)
for (M, N, K, bias, tb) in [(300000, 300, 300, True, True), (262144, 300, 300, False, False),
                            (100003, 600, 300, False, False), (70000, 300, 600, True, True),
                            (65536, 96, 300, False, True)]:
    X = torch.randn(M, K, generator=g).to(dev)
    W = torch.randn(N, K, generator=g).to(dev) if tb else torch.randn(K, N, generator=g).to(dev)
    b = torch.randn(N, generator=g).to(dev) if bias else None
    Y = ops.gemm(X, W, trans_b=tb, bias=b, x3=True)
    rows = torch.randint(0, M, (4000,), generator=g).to(dev)
    ref = X[rows].double() @ (W.double().t() if tb else W.double())
    if bias:
        ref = ref + b.double()
    err = ((Y[rows].double() - ref).abs().max() / ref.abs().max()).item()
    print((M, N, K, bias, tb), "rel %.2e" % err, "OK" if err < 2e-6 else "BAD", flush=True)
