"""A/B timing of the fp32 (x3) GEMM shapes of the EA step from alternative builds of the library
(debug tool): python tools/dbg/gemm_ab.py libgnnea.so libgnnea_<variant>.so libgnnea.so:GNNEA_X3W=3
Each library (optionally with one environment setting) is loaded in its own child process;
median of 21 HIP-event timings per shape."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = r'''
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(%r, "gnn-mtl_amd"))
from gnnea import _lib
_lib.LIB_PATH = os.path.join(os.path.dirname(_lib.LIB_PATH), sys.argv[1])
from gnnea import ops
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
N, D = 2000000, 300
X = torch.randn(N, D, device=dev, generator=g)
X2 = torch.randn(N, 2 * D, device=dev, generator=g)
W = torch.randn(D, D, device=dev, generator=g)
W2 = torch.randn(D, 2 * D, device=dev, generator=g)
W3 = torch.randn(2 * D, D, device=dev, generator=g)
b = torch.randn(D, device=dev, generator=g)
C0 = torch.randn(N, D, device=dev, generator=g)
Cb = torch.empty_like(C0)
def run(fn):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(21):
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); e.record(); torch.cuda.synchronize(); ts.append(a.elapsed_time(e))
    return round(float(np.median(ts)), 4)
res = {}
res["proj x.W^T+b 300"] = run(lambda: ops.gemm(X, W, trans_b=True, bias=b, x3=True))
res["proj x.[W^T|Kg] 600"] = run(lambda: ops.gemm(X, W2, x3=True))
res["dX [dh|dg].[W;Kg^T] K600 +C"] = run(lambda: ops.gemm(X2, W3, out=Cb.copy_(C0), beta=1.0, x3=True))
res["dW X^T.X"] = run(lambda: ops.gemm(X, X, trans_a=True, x3=True))
W80 = W[:80].contiguous()
res["proj x.W80^T 80 (one column tile)"] = run(lambda: ops.gemm(X, W80, trans_b=True, x3=True))
# accuracy on a row sample (fp64 reference)
y = ops.gemm(X2[:200000], W3, x3=True); r = X2[:200000].double() @ W3.double()
res["err dX K600"] = float((y.double() - r).abs().max() / r.abs().max())
y = ops.gemm(X[:200000], W, trans_b=True, bias=b, x3=True); r = X[:200000].double() @ W.double().t() + b.double()
res["err proj"] = float((y.double() - r).abs().max() / r.abs().max())
cb = Cb[:200000].copy_(C0[:200000]); ops.gemm(X2[:200000], W3, out=cb, beta=1.0, x3=True)
r = C0[:200000].double() + X2[:200000].double() @ W3.double()
res["err dX +C"] = float((cb.double() - r).abs().max() / r.abs().max())
y = ops.gemm(X[:200000], X[:200000], trans_a=True, x3=True); r = X[:200000].double().t() @ X[:200000].double()
res["err dW"] = float((y.double() - r).abs().max() / r.abs().max())
print(json.dumps({sys.argv[1]: res}), flush=True)
''' % ROOT

out = {}
for spec in sys.argv[1:]:
    lib, _, kv = spec.partition(":")
    env = dict(os.environ)
    if kv:
        k, v = kv.split("=", 1)
        env[k] = v
    r = subprocess.run([sys.executable, "-c", CHILD, lib], capture_output=True, text=True,
                       timeout=300, env=env)
    sys.stderr.write(r.stderr[-2000:])
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    # the child keys its result by the library file; keyed here by the whole spec
    out[spec] = next(iter(json.loads(line[-1]).values())) if line else {"rc": r.returncode}
    print(json.dumps({spec: out[spec]}), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "gemm_ab.json"), "w"), indent=1)
