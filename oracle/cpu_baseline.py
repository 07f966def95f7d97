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
