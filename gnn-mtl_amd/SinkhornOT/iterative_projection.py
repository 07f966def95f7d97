"""GW / FGW iterative projection (drop-in for SinkhornOT/iterative_projection.py, §8f #3).

iterative_1 (iterative_projection.py:6-58): starting from the uniform plan, every outer
iteration rebuilds the GW (or FGW) linearised cost from the previous plan with two GEMMs
(cderivation.get_LT) and solves an entropic OT problem on 2·cost with the device Sinkhorn
(sinkhorn_iteration, or forward_relax_sinkhorn_iteration for the relaxed variants); it stops when
||T_old - T||_F < tol.  The plan, the costs and the Sinkhorn state stay on the device; the only
host synchronisation per outer iteration is the tolerance test (as in the reference).
"""
import torch

from .cderivation import FGW_cost_matrix, GW_cost_matrix, get_init_matrices
from .sinkhorn_loss import forward_relax_sinkhorn_iteration, sinkhorn_iteration


def iterative_1(C1, C2, mu, nu, epsilon, max_iter, log, tol=1e-9, g=True,
                cost_mat_func=GW_cost_matrix, lambdda=0):
    I, J = C1.shape[0], C2.shape[0]
    assert C1.device == C2.device
    dtype = C1.dtype
    mu = mu.view(1, I, 1)
    nu = nu.view(1, 1, J)
    T_old = (torch.ones(I, J) / (I * J)).to(C1.device).to(dtype)
    constC, hC1, hC2 = get_init_matrices(C1, C2, mu, nu)
    lt, _ = cost_mat_func(constC, hC1, hC2, T_old, epsilon)
    gw_dist = torch.sum(torch.mul(T_old, lt))
    rec = None
    if log:
        rec = {"constC": constC.cpu().numpy(), "hC1": hC1.cpu().numpy(),
               "hC2": hC2.cpu().numpy(), "err": [], "gwd": [], "D": [], "T": []}
    T = T_old
    for i_proj in range(max_iter):
        cost = 2 * lt.view(1, I, J)
        if g:
            gw_dist, *_, T = forward_relax_sinkhorn_iteration(cost, mu, nu, lambdda, epsilon)
        else:
            gw_dist, *_, T = sinkhorn_iteration(cost, mu, nu, epsilon)
        err = torch.norm(T_old - T)
        if rec is not None:
            rec["err"].append(err.cpu().numpy())
            rec["gwd"].append(gw_dist.cpu().numpy())
            rec["T"].append(T.cpu().numpy())
            rec["D"].append(2 * lt.cpu().numpy())
            print("Iteration:{} err:{} gwd:{}".format(i_proj, err.item(), gw_dist.item()))
        if err < tol:
            print("meet tol jump out GW iteration")
            break
        T_old = T
        # the reference rebuilds the next cost with GW_cost_matrix whatever cost_mat_func was
        # (iterative_projection.py:54): kept, FGW's fused cost only enters the first iteration
        lt, _ = GW_cost_matrix(constC, hC1, hC2, T_old, epsilon)
    if rec is not None:
        rec["gw_dist"] = gw_dist.cpu().numpy() / 2
        return T, rec
    return T, gw_dist


def gw_iterative_1(C1, C2, mu, nu, epsilon, max_iter, log=False, tol=1e-9):
    """iterative_projection.py:113-114"""
    return iterative_1(C1, C2, mu, nu, epsilon, max_iter, log, tol, False, GW_cost_matrix)


def rgw_iterative_1(C1, C2, mu, nu, max_iter, lambdda, epsilon, log=False, tol=1e-6):
    """iterative_projection.py:117-118"""
    return iterative_1(C1, C2, mu, nu, epsilon, max_iter, log, tol, True, GW_cost_matrix,
                       lambdda)


def fgw_iterative_1(D, C1, C2, mu, nu, alpha, p, max_iter, epsilon, log=False, tol=1e-6):
    """iterative_projection.py:121-124"""
    def cost(constC, hC1, hC2, T, eps):
        return FGW_cost_matrix(D, constC, hC1, hC2, T, alpha, eps, p)
    return iterative_1(C1, C2, mu, nu, epsilon, max_iter, log, tol, False, cost)


def rfgw_iterative_1(D, C1, C2, mu, nu, alpha, p, max_iter, lambdda, epsilon, log=False,
                     tol=1e-6):
    """iterative_projection.py:127-130"""
    def cost(constC, hC1, hC2, T, eps):
        return FGW_cost_matrix(D, constC, hC1, hC2, T, alpha, eps, p)
    return iterative_1(C1, C2, mu, nu, epsilon, max_iter, log, tol, True, cost, lambdda)
