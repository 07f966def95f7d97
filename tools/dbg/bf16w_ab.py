"""Time the cfg-5 bf16 projection GEMM (4M x 300 x 300, weight-resident k_gemm_bf16w or its ring
form per GNNEA_BF16W_RING) and check it against fp64 (debug tool)."""
import os
import sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))
from gnnea import ops  # noqa

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(4000000, 300, device=dev, generator=g).to(torch.bfloat16)
W = torch.randn(300, 300, device=dev, generator=g).to(torch.bfloat16)
b = torch.randn(300, device=dev, generator=g)
res = {}
for name, fn in (("NT+b", lambda: ops.gemm(X, W, trans_b=True, bias=b)),
                 ("NN", lambda: ops.gemm(X, W))):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(21):
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(e))
    res[name] = round(float(np.median(ts)), 4)
y = ops.gemm(X[:200000], W, trans_b=True, bias=b, out_dtype=torch.float32)
ref = X[:200000].double() @ W.double().t() + b.double()
res["rel_err"] = float((y.double() - ref).norm() / ref.norm())
print(os.environ.get("GNNEA_BF16W_RING", "1"), res, flush=True)
