"""The fp32 projection GEMM's split forms over a wide dynamic range (gemm_x3w.hip): the x3
bf16 ring and the f16x2 ring (two fp16 pieces per operand, every activation row and weight
column scaled by a power of two into fp16's range) against fp64, element by element relative
to sum_k |a_ik||w_kj| (the bound an fp32 GEMM's own rounding is stated in).

Rows of x are scaled by 10^U(-20, 20), columns of W by 10^U(-10, 10), one row is all zeros, one
row holds values 2^30 apart (the small ones fall to fp16 subnormals after scaling, inside the
bound), and K = 300 / 292 / 320 (tail quads) and 600 / 584 (the f16x2 form's two k-chunks, each with
its own row scale)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
TOL = 4e-6  # of sum_k |a||w|; fp32 accumulation alone reaches ~K 2^-24 = 1.8e-5 worst case


def _case(device, M, K, N, seed):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((M, K)) * 10.0 ** rng.uniform(-20, 20, (M, 1))
    W = rng.standard_normal((N, K)) * 10.0 ** rng.uniform(-10, 10, (N, 1))
    x[5] = 0.0
    x[7] = rng.standard_normal(K)
    x[7, ::3] *= 2.0 ** -30
    b = rng.standard_normal(N)
    return x, W, b


@pytest.mark.parametrize("mode", ["2", "4"])
@pytest.mark.parametrize("M,K,N", [(70000, 300, 300), (70000, 292, 600), (66000, 320, 96),
                                   (70000, 600, 300), (66000, 584, 132)])
def test_gemm_split_range_vs_fp64(device, mode, M, K, N):
    import subprocess
    import sys
    import os
    # the mode is read once per process: run the case in a child with GNNEA_X3W set
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = r'''
import sys, os, numpy as np, torch
sys.path.insert(0, os.path.join(%r, "gnn-mtl_amd")); sys.path.insert(0, %r)
sys.path.insert(0, os.path.join(%r, "tests"))
from test_gpu_gemm_range import _case
from gnnea import ops
M, K, N = %d, %d, %d
x, W, b = _case(None, M, K, N, M + K + N)
dev = torch.device("cuda:0")
xt = torch.from_numpy(x).float().to(dev); Wt = torch.from_numpy(W).float().to(dev)
bt = torch.from_numpy(b).float().to(dev)
y = ops.gemm(xt, Wt, trans_b=True, bias=bt, x3=True).double().cpu().numpy()
x32, W32 = xt.double().cpu().numpy(), Wt.double().cpu().numpy()
ref = x32 @ W32.T + bt.double().cpu().numpy()
bound = np.abs(x32) @ np.abs(W32).T + np.abs(bt.double().cpu().numpy())
e = np.abs(y - ref) / bound
print("MAXERR %%.3e" %% e.max(), "FINITE", bool(np.isfinite(y).all()))
''' % (root, root, root, M, K, N)
    env = dict(os.environ, GNNEA_X3W=mode)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("MAXERR")][-1].split()
    assert line[3] == "True"
    assert float(line[1]) < TOL, line
