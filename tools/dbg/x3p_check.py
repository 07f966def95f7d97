"""x3 GEMM (k_gemm_x3p / k_gemm_x3) vs fp64 on assorted shapes (debug tool, GPU)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gnnea import ops  # noqa: E402

dev = torch.device("cuda:0")
for (M, N, K) in [(70, 40, 12), (70, 40, 16), (70, 40, 32), (70, 64, 32), (70, 300, 32),
                  (70, 300, 12), (64, 64, 16), (64, 300, 300), (70, 128, 16), (70, 192, 16),
                  (70, 256, 16)]:
    rng = np.random.default_rng(0)
    a = rng.standard_normal((M, K)).astype(np.float32)
    b = rng.standard_normal((K, N)).astype(np.float32)
    y3 = ops.gemm(torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev), False, False,
                  x3=True).cpu().double().numpy()
    ref = a.astype(np.float64) @ b.astype(np.float64)
    err = np.abs(y3 - ref)
    bad = np.argwhere(err > 1e-4 * np.abs(ref).max())
    print((M, N, K), "rel %.2e" % (err.max() / np.abs(ref).max()), "bad", len(bad),
          "rows", sorted(set(bad[:, 0].tolist()))[:8], "cols", sorted(set(bad[:, 1].tolist()))[:8],
          flush=True)
