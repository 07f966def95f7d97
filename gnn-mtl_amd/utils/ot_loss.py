"""Entropic OT (reference utils/ot_loss.py) on the HIP Sinkhorn (gnnea_sinkhorn_*, KNOPP).

``sinkhorn(a, b, M, reg, numItermax, stopThr, verbose) -> (P, loss)`` keeps the reference's
semantics and arithmetic (fp64, K = exp(M / -reg) built once on the device, u = 1/I and v = 1/J
start, err = ||v (K^T u) - b||_2 checked every 10th iteration, revert-and-break on K^T u == 0 /
inf / NaN); the loop runs on the device, the host only reads the stop flag between batches.

``sinkhorn_row_sharded(a_loc, b, M_loc, reg, ...)`` is the same solve with M's rows split over
the ranks of a torch.distributed group (consecutive row blocks in rank order):
one all-gather of the column log-sum-exp pairs per iteration, identical stop decisions on every
rank.  It returns this rank's plan rows and the loss of the whole plan.
"""
import torch

from gnnea import _lib
from gnnea.sinkhorn import solve, solve_row_sharded


def sinkhorn(a, b, M, reg, numItermax=1000, stopThr=1e-9, verbose=False):
    assert a.device == b.device and b.device == M.device, "a, b, M must be on the same device"
    _lib.require_device(M)
    I, J = M.shape
    a = a.double()
    b = b.double()
    if len(a) == 0:
        a = torch.ones(I, dtype=torch.float64, device=M.device) / I
    if len(b) == 0:
        b = torch.ones(J, dtype=torch.float64, device=M.device) / J
    assert len(a) == I and len(b) == J, "the dimension of weights and distance matrix don't match"
    # fp32 M is widened exactly inside the kernels (the reference casts M to fp64, :27)
    res = solve(_lib.GNNEA_SK_KNOPP, M, a, b, reg, stopThr, numItermax)
    if res.reason == 2:
        print("Warning: numerical errors at iteration ", res.iters)
    if verbose:
        print("{:5s}|{:5s}".format('It.', 'Err') + '\n' + '-' * 19)
        print("{:5d}|{:.6e}".format(res.iters, res.err))
    loss = torch.tensor(res.loss, dtype=torch.float64, device=M.device)
    return res.plan, loss


def sinkhorn_row_sharded(a_loc, b, M_loc, reg, numItermax=1000, stopThr=1e-9, verbose=False,
                         group=None):
    _lib.require_device(M_loc)
    a_loc = a_loc.double()
    b = b.double()
    assert len(a_loc) == M_loc.shape[0] and len(b) == M_loc.shape[1], \
        "the dimension of weights and distance matrix don't match"
    res = solve_row_sharded(M_loc, a_loc, b, reg, stopThr, numItermax, group=group)
    if res.reason == 2:
        print("Warning: numerical errors at iteration ", res.iters)
    if verbose:
        print("{:5d}|{:.6e}".format(res.iters, res.err))
    return res.plan, torch.tensor(res.loss, dtype=torch.float64, device=M_loc.device)
