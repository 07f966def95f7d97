"""Host-side cost per gnnea op call on tiny inputs (GPU work negligible): wall time / call."""
import os
import sys
import time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))
from gnnea import ops  # noqa
from gnnea.graph import DeviceCSR  # noqa

dev = torch.device("cuda:0")
n = 64
r = torch.arange(n, device=dev)
csr = DeviceCSR.from_coo(r, r, torch.ones(n, device=dev), n, n)
x = torch.randn(n, 300, device=dev)
w = torch.randn(300, 300, device=dev)
y = torch.empty(n, 300, device=dev)


def bench(name, fn, k=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print("%-28s host %.2f us/call" % (name, (t1 - t0) / k * 1e6), flush=True)


bench("torch.relu (reference)", lambda: torch.relu(x))
bench("ops.spmm", lambda: ops.spmm(csr, x, 1, out=y))
bench("ops.gemm", lambda: ops.gemm(x, w, trans_b=True))
bench("ops.act_bwd", lambda: ops.act_bwd(x, x, 1))
bench("current_stream", lambda: torch.cuda.current_stream(dev).cuda_stream)
bench("raw stream", lambda: torch._C._cuda_getCurrentRawStream(0))
bench("with device", lambda: torch.cuda.device(dev).__enter__())
