"""Cost-matrix algebra of the GW / FGW outer loops (drop-in for SinkhornOT/cderivation.py, §8f #3).

Everything here is dense linear algebra on device tensors: the two products of get_LT
(C1 · T · C2^T, 2·I·J·(I+J) flops per outer iteration) go to the library GEMM (hipBLASLt through
torch.mm), elementwise work stays in torch.  The Sinkhorn inner solves that consume these costs
run on the gnnea kernels (SinkhornOT/sinkhorn_loss.py).  Distance helpers outside the GW path
(energy distances, ...) are taken from the reference module when GNNEA_UPSTREAM names its checkout.
"""
import math

import torch

big = 1e20
huge = 1e30
small = 1e-7


def p_norm_dist_mat(x, y, p=2):
    """cderivation.py:14-27: sum_d (x_d - y_d)^p for every pair, [n1, n2]."""
    assert x.shape[1] == y.shape[1]
    return torch.sum(torch.pow(x[:, None, :] - y[None, :, :], p), -1)


def norm_dist_mat(x, y, p=2):
    """cderivation.py:30-38"""
    return torch.pow(p_norm_dist_mat(x, y, p), 1 / p)


def cos_dist_mat(x, y):
    """cderivation.py:45-61: 1 - cosine similarity, [n1, n2] (row-chunked for large inputs)."""
    n1, d1 = x.shape
    n2, d2 = y.shape
    assert d1 == d2
    if n1 * n2 > 10000:
        sim = torch.cat([torch.cosine_similarity(x[i].view(1, 1, d1), y.view(1, n2, d2), -1)
                         for i in range(n1)], 0)
    else:
        sim = torch.cosine_similarity(x.view(n1, 1, d1), y.view(1, n2, d2), -1)
    return 1 - sim


def get_intra_sim(x, sim_func):
    """cderivation.py:136-138"""
    x = x.detach()
    return sim_func(x, x)


def get_inter_sim(x, y, sim_func):
    """cderivation.py:141-143"""
    return sim_func(x.detach(), y.detach())


def get_init_matrices(C1, C2, mu, nu, div_type="l2"):
    """cderivation.py:146-157: the T-independent part of the square-loss GW cost,
    constC_ij = 1/2 sum_k C1_ik^2 mu_k + 1/2 sum_l nu_l C2_jl^2 (each term a matrix product, as
    the reference forms them), and hC1 = C1, hC2 = C2."""
    I, J = C1.shape[0], C2.shape[0]
    mu_col = mu.reshape(I, 1)
    nu_row = nu.reshape(1, J)
    A = 0.5 * torch.matmul(C1 ** 2, mu_col.repeat(1, J))
    B = 0.5 * torch.matmul(nu_row.repeat(I, 1), C2.t() ** 2)
    return A + B, C1, C2


def get_LT(constC, hC1, hC2, T):
    """cderivation.py:160-162: L(C1, C2) (x) T = constC - C1 · T · C2^T."""
    return constC - torch.matmul(hC1, torch.matmul(T, hC2.t()))


def w2_cost_matrix(D, device):
    """cderivation.py:168-169"""
    return torch.pow(D, 2).to(device)


def wfr_cost_matrix(D, diameter, device):
    """cderivation.py:172-176"""
    half_pi = torch.tensor(math.pi / 2).to(device)
    return -2 * torch.log(torch.cos(torch.min(torch.div(D, diameter) * half_pi, half_pi)) + small)


def GW_cost_matrix(constC, hC1, hC2, T_old, epsilon):
    """cderivation.py:179-182: (lt, lt - eps log(T + small))."""
    lt = get_LT(constC, hC1, hC2, T_old)
    return lt, lt - epsilon * torch.log(T_old + small)


def FGW_cost_matrix(D, constC, hC1, hC2, T, alpha, epsilon, p):
    """cderivation.py:185-188: fused cost (1 - alpha) D^p + alpha L^p and its entropic form."""
    A = (1 - alpha) * D ** p + alpha * get_LT(constC, hC1, hC2, T) ** p
    return A, A - epsilon * torch.log(T)


def _merge_upstream():
    """Opt-in (GNNEA_UPSTREAM=<reference checkout>, gnnea/upstream.py): the reference module's
    remaining helpers."""
    from gnnea import upstream
    upstream.merge(globals(), "SinkhornOT/cderivation.py", "SinkhornOT._upstream_cderivation")


_merge_upstream()
