"""Timed CPU baseline: the reference's own op on the host cores (bench.py cpu_baseline leg).

The GCN aggregation of the reference is ``torch.spmm(adj, hidden)`` on the uncoalesced
int64-index fp32 COO adjacency that utils/data_utils.py:325-336 / :51-57 builds
(layers/layers.py:35).  This module times exactly that call on a row-sample of the same graph.
"""
import time

import torch


def time_reference_spmm(row, col, val, n_rows, n_cols, H, sample_rows, reps=1, threads=None):
    """Edges/s of torch.spmm(COO[rows < sample_rows], H) on the host; returns (rate, nnz, s)."""
    if threads:
        torch.set_num_threads(int(threads))
    keep = row < sample_rows
    idx = torch.stack([torch.as_tensor(row[keep]), torch.as_tensor(col[keep])]).long()
    A = torch.sparse_coo_tensor(idx, torch.as_tensor(val[keep]), (int(sample_rows), n_cols))
    nnz = int(idx.shape[1])
    torch.spmm(A, H)  # warm-up (allocations, thread pool)
    t0 = time.perf_counter()
    for _ in range(reps):
        torch.spmm(A, H)
    dt = (time.perf_counter() - t0) / reps
    return nnz / dt, nnz, dt


def cpu_model():
    """The host CPU's model name (lscpu's 'Model name', read from /proc/cpuinfo)."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def time_reference_gat(row, col, val, n, x, W, a, sample_rows, alpha=0.2):
    """Head-edges/s of one SpGraphAttentionLayer head (layers/att_layers.py:29-61) as the
    reference computes it on the host: coalesced edges, h = x·W, edge logits from the
    concatenated endpoint rows, exp(-LeakyReLU), row sums and the weighted aggregation by
    torch.spmm, division, ReLU.  Destination rows < sample_rows only (their edges gather from
    the whole graph).  Returns (rate, edges, seconds)."""
    keep = row < sample_rows
    A = torch.sparse_coo_tensor(torch.stack([torch.as_tensor(row[keep]),
                                             torch.as_tensor(col[keep])]).long(),
                                torch.as_tensor(val[keep]), (int(sample_rows), n))

    def head():
        edge = A.coalesce().indices()
        h = torch.mm(x, W)
        edge_h = torch.cat((h[edge[0, :], :], h[edge[1, :], :]), dim=1).t()
        edge_e = torch.exp(-torch.nn.functional.leaky_relu(a.mm(edge_h).squeeze(), alpha))
        e_rowsum = torch.spmm(torch.sparse_coo_tensor(edge, edge_e, (int(sample_rows), n)),
                              torch.ones(n, 1))
        h_prime = torch.spmm(torch.sparse_coo_tensor(edge, edge_e, (int(sample_rows), n)), h)
        return torch.relu(h_prime.div(e_rowsum))

    head()
    t0 = time.perf_counter()
    head()
    dt = time.perf_counter() - t0
    e = int(keep.sum())
    return e / dt, e, dt


def time_reference_sinkhorn(M, reg, iters):
    """Iterations/s of the loop body of utils/ot_loss.py:50-66 (fp64, a = b = ones as
    models/models_ea.py:217 calls it, the every-10th error check included) on the host."""
    M = torch.as_tensor(M, dtype=torch.float64)
    I, J = M.shape
    a = torch.ones(I, dtype=torch.float64)
    b = torch.ones(J, dtype=torch.float64)
    u = torch.ones(I, 1, dtype=torch.float64) / I
    v = torch.ones(J, 1, dtype=torch.float64) / J
    K = torch.exp(M / -reg)
    Kp = (1 / a).reshape(-1, 1) * K
    t0 = time.perf_counter()
    for cpt in range(iters):
        KtranposeU = torch.mm(K.t(), u)
        v = b.reshape(-1, 1) / KtranposeU
        u = 1. / Kp.mm(v)
        if (torch.any(KtranposeU == 0) or torch.any(torch.isnan(u)) or torch.any(torch.isnan(v))
                or torch.any(torch.isinf(u)) or torch.any(torch.isinf(v))):
            break
        if cpt % 10 == 0:
            torch.norm(torch.einsum('ia,ij,jb->j', u, K, v) - b)
    dt = time.perf_counter() - t0
    return (cpt + 1) / dt, dt
