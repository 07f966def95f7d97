"""A/B timing of the x3p projection GEMM (cfg-4 shape) from an alternative build of the library
(debug tool): python tools/dbg/x3_ab.py <libname.so>"""
import os
import sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))
from gnnea import _lib  # noqa
_lib.LIB_PATH = os.path.join(os.path.dirname(_lib.LIB_PATH), sys.argv[1])
from gnnea import ops  # noqa

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(2000000, 300, device=dev, generator=g)
W = torch.randn(300, 300, device=dev, generator=g)
b = torch.randn(300, device=dev, generator=g)
res = {}
for name, fn in (("NT+b", lambda: ops.gemm(X, W, trans_b=True, bias=b, x3=True)),
                 ("NN", lambda: ops.gemm(X, W, x3=True))):
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
y = ops.gemm(X[:100000], W, trans_b=True, bias=b, x3=True)
ref = X[:100000].double() @ W.double().t() + b.double()
res["rel_err"] = float((y.double() - ref).norm() / ref.norm())
print(sys.argv[1], res, flush=True)
