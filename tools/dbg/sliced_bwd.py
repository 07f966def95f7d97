"""Debug: sliced vs row-major AggregateFn backward on the two-KG test graph."""
import os
import sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))
from gnnea import ops, synth  # noqa
from gnnea.graph import DeviceCSR  # noqa

dev = torch.device("cuda:0")
n = 300000
tr = synth.kg_pair_triples(n, 3 * n, 500, seed=4)
r, c, v = synth.adjacency_coo(tr, 2 * n, reference_order=False)
csr = DeviceCSR.from_coo(torch.from_numpy(r).to(dev), torch.from_numpy(c).to(dev),
                         torch.from_numpy(v).to(dev), 2 * n, 2 * n)
h = torch.randn(2 * n, 128, device=dev)
dy = torch.randn(2 * n, 128, device=dev)
y = ops.spmm(csr, h, 1)
csrT = csr.transpose()
print("blocks", csr.row_blocks(), csrT.row_blocks(), csrT.n_rows, csrT.n_cols, csrT.nnz)
g = ops.act_bwd(dy, y, 1)
gs = ops.act_bwd_sliced(dy, y, 1)
un = gs.permute(1, 0, 2).reshape(2 * n, -1)[:, :128]
print("act_bwd_sliced == act_bwd:", torch.equal(un, g))
for trial in range(3):
    a = ops.spmm_sliced(csrT, gs, 128)
    b = ops.spmm(csrT, g)
    d = (a - b).abs()
    rows = torch.nonzero(d.max(dim=1).values > 1e-3 * b.abs().max()).flatten()
    print(trial, "maxdiff", float(d.max()), "bad rows", rows.numel(), rows[:10].tolist())
# symmetric A: A^T = A; compare with forward CSR too
a2 = ops.spmm_sliced(csr, gs, 128)
print("fwd csr vs T:", float((a2 - ops.spmm(csr, g)).abs().max()))
rp = csrT.rowptr.cpu().numpy()
print("csrT rowptr monotone", bool(np.all(np.diff(rp) >= 0)), rp[-1], int(csrT.col.max()), int(csrT.col.min()))
