"""Cost-matrix algebra of the GW / FGW outer loops (drop-in for SinkhornOT/cderivation.py, §8f #3).

Everything here is dense linear algebra on device tensors.  The two products of get_LT
(C1 · T · C2^T, 2·I·J·(I+J) flops per outer iteration) run on gnnea's own matrix-core GEMMs:
fp64 (the reference path's dtype) on the f64 MFMA kernel gnnea_gemm_f64 with the subtraction
from constC fused into the second product's epilogue (L = constC - C1·X in one launch), fp32 /
bf16 on gnnea.ops.gemm.  get_init_matrices' two products are matrix-vector products in
disguise (every column of C1²·repeat(mu) is C1²·mu): they run as [I, 1] / [J, 1] GEMMs and
constC is their broadcast sum.  Elementwise work stays in torch.  The Sinkhorn inner solves
that consume these costs run on the gnnea kernels (SinkhornOT/sinkhorn_loss.py).  Distance helpers outside the GW path
(energy distances, ...) are out of scope.
"""
import math

import torch

from gnnea import _lib, ops

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


def _mm(a, b, trans_b=False):
    """a @ op(b) on the device GEMMs (fp64: gnnea_gemm_f64; fp32 / bf16: gnnea.ops.gemm)."""
    _lib.require_device(a, b)
    if a.dtype == torch.float64 or b.dtype == torch.float64:
        return ops.gemm_f64(a.double(), b.double(), trans_b=trans_b)
    return ops.gemm(a, b, trans_b=trans_b, out_dtype=torch.float32).to(a.dtype)


def get_init_matrices(C1, C2, mu, nu, div_type="l2"):
    """cderivation.py:146-157: the T-independent part of the square-loss GW cost,
    constC_ij = 1/2 sum_k C1_ik^2 mu_k + 1/2 sum_l nu_l C2_jl^2, and hC1 = C1, hC2 = C2.
    The reference forms both terms as [I, J] matrix products of repeated vectors; each is one
    [I, 1] / [J, 1] product here (the same exact products, summed in k order)."""
    I, J = C1.shape[0], C2.shape[0]
    a = _mm(C1 ** 2, mu.reshape(I, 1).to(C1.dtype))
    b = _mm(C2 ** 2, nu.reshape(J, 1).to(C2.dtype))
    return 0.5 * a + 0.5 * b.reshape(1, J), C1, C2


def get_LT(constC, hC1, hC2, T):
    """cderivation.py:160-162: L(C1, C2) (x) T = constC - C1 · (T · C2^T); in fp64 the
    subtraction is the second GEMM's epilogue (alpha = -1, beta = 1, E = constC)."""
    _lib.require_device(constC, hC1, hC2, T)
    if T.dim() > 2:  # a batch of plans (the Sinkhorn solvers return [bt, I, J]): as matmul
        lead = T.shape[:-2]
        Ts = T.reshape(-1, *T.shape[-2:])
        return torch.stack([get_LT(constC, hC1, hC2, t) for t in Ts]).reshape(
            *lead, *Ts.shape[-2:])
    if T.dtype == torch.float64:
        X = ops.gemm_f64(T, hC2.double(), trans_b=True)
        return ops.gemm_f64(hC1.double(), X, alpha=-1.0, e=constC.double(), beta=1.0)
    return constC - _mm(hC1, _mm(T, hC2, trans_b=True))


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
