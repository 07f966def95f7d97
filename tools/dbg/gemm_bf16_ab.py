"""A/B timing of the bf16 projection GEMM of the cfg-5 step (k_gemm_bf16w: 2M x 300 x 300,
bf16 in and out, the GAT / Linear projections) from alternative builds (debug tool):
python tools/dbg/gemm_bf16_ab.py libgnnea.so libgnnea_<variant>.so ...
Each library in its own child process; median of 21 HIP-event timings per shape."""
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
X = torch.randn(N, D, device=dev, generator=g).bfloat16()
W = torch.randn(D, D, device=dev, generator=g).bfloat16()
b = torch.randn(D, device=dev, generator=g)
def run(fn):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(21):
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); e.record(); torch.cuda.synchronize(); ts.append(a.elapsed_time(e))
    return round(float(np.median(ts)), 4)
res = {}
res["bf16 x.W^T+b 300 (bf16 out)"] = run(lambda: ops.gemm(X, W, trans_b=True, bias=b))
res["bf16 x.W 300 (bf16 out)"] = run(lambda: ops.gemm(X, W))
res["bf16 relu(x.W^T+b) 300"] = run(lambda: ops.gemm(X, W, trans_b=True, bias=b, act=1))
res["bf16 x.W^T+b 300 (fp32 out)"] = run(lambda: ops.gemm(X, W, trans_b=True, bias=b,
                                                          out_dtype=torch.float32))
y = ops.gemm(X[:100000], W, trans_b=True, bias=b).float()
r = X[:100000].float() @ W.float().t() + b
res["err x.W^T+b (norm-rel, bf16 out)"] = float((y - r).norm() / r.norm())
y = ops.gemm(X[:100000], W).float()
r = X[:100000].float() @ W.float()
res["err x.W (norm-rel, bf16 out)"] = float((y - r).norm() / r.norm())
print(json.dumps({sys.argv[1]: res}), flush=True)
''' % ROOT

out = {}
for lib in sys.argv[1:]:
    r = subprocess.run([sys.executable, "-c", CHILD, lib], capture_output=True, text=True,
                       timeout=300)
    sys.stderr.write(r.stderr[-2000:])
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    out[lib] = next(iter(json.loads(line[-1]).values())) if line else {"rc": r.returncode}
    print(json.dumps({lib: out[lib]}), flush=True)
