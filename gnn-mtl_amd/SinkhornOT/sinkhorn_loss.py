"""Stabilised Sinkhorn solvers (reference SinkhornOT/sinkhorn_loss.py:159-356) on HIP.

``sinkhorn_iteration`` / ``gsinkhorn_iteration`` / ``forward_relax_sinkhorn_iteration`` keep
the reference signatures and return ``(transport, margin1, margin2, K)``.  The scaling-with-
absorption loop runs on the device in the reference's own form (fp64 K resident in HBM,
absorption schedule, 1e30 clamps, 1e20 trigger, relative-tolerance break).  A batch [bt, I, J]
runs as one launch sequence (gnnea.sinkhorn.solve_batch: every problem's iterations enqueued
round by round on one stream, one status read-back per round for the whole batch).
"""
import torch

from gnnea import _lib
from gnnea.sinkhorn import solve_batch

big = 1e20
huge = 1e30
small = 1e-7


def myclamp(x):
    return torch.clamp(x, 0, huge)


def kl_div(x, y):
    """KL term of two tensors (reference :20-30)."""
    div = torch.div(x, y + small)
    return torch.mul(y, div * torch.log(div + small) - div + 1)


def _run(mode, C, mu, nu, epsilon, numIterMax, tol, lambdda, debug, out_dtype, prev_transport):
    *lead, I, J = C.shape
    _, I1, _ = mu.shape
    *_, J1 = nu.shape
    if debug:
        assert I == I1
        assert J == J1
        assert len(C.shape) == len(mu.shape)
        assert len(C.shape) == len(nu.shape)
    _lib.require_device(C)
    p = lambdda / (lambdda + epsilon) if mode != _lib.GNNEA_SK_STAB else 1.0
    Cb = C.reshape(-1, I, J)
    bt = Cb.shape[0]
    mub = mu.reshape(-1, I).double()
    nub = nu.reshape(-1, J).double()
    mub = mub.expand(bt, I) if mub.shape[0] == 1 else mub
    nub = nub.expand(bt, J) if nub.shape[0] == 1 else nub
    if Cb.dtype not in (torch.float32, torch.float64):
        Cb = Cb.to(out_dtype)
    res = solve_batch(mode, Cb, mub, nub, epsilon, tol, numIterMax, p=p,
                      plan_dtype=torch.float64)
    Ks, trans, m1, m2 = [], [], [], []
    for k, r in enumerate(res):
        K = r.plan
        if debug:
            assert not torch.isnan(K).any()
        t = r.transport_prev if prev_transport else r.transport_new
        trans.append(torch.tensor(t, dtype=torch.float64, device=C.device))
        m1.append(kl_div(r.row_sum, mub[k]).sum())
        m2.append(kl_div(r.col_sum, nub[k]).sum())
        Ks.append(K)
    K = torch.stack(Ks).reshape(*lead, I, J).to(out_dtype)
    squeeze = lambda v: torch.stack(v).to(out_dtype).squeeze()  # noqa: E731
    return squeeze(trans), squeeze(m1), squeeze(m2), K


def sinkhorn_iteration(C, mu, nu, epsilon, numIterMax=100, tol=1e-9, debug=True):
    """Balanced stabilised Sinkhorn (:159-220): returns (transport_new, margin1, margin2, K)."""
    dt = torch.promote_types(torch.promote_types(mu.dtype, nu.dtype), C.dtype)
    return _run(_lib.GNNEA_SK_STAB, C, mu, nu, epsilon, numIterMax, tol, 0.0, debug, dt, False)


def gsinkhorn_iteration(C, mu, nu, lambdda, epsilon, numIterMax=100, tol=1e-6, debug=False):
    """Generalised (both marginals relaxed, exponent lambda/(lambda+eps)) Sinkhorn (:223-288)."""
    dt = torch.promote_types(torch.promote_types(mu.dtype, nu.dtype), C.dtype)
    return _run(_lib.GNNEA_SK_GEN, C, mu, nu, epsilon, numIterMax, tol, lambdda, debug, dt, True)


def forward_relax_sinkhorn_iteration(C, mu, nu, lambdda, epsilon, numIterMax=100, tol=1e-6,
                                     debug=False):
    """Target marginal relaxed only (:291-356); potentials in fp64 as in the reference."""
    return _run(_lib.GNNEA_SK_RELAX, C, mu, nu, epsilon, numIterMax, tol, lambdda, debug,
                torch.float64, True)
