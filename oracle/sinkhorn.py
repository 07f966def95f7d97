"""fp64 numpy restatement of the Sinkhorn solvers in their original scaling form.

  knopp      utils/ot_loss.py:5-76     u,v scaling; break on K^T u == 0 / inf / NaN (revert);
                                       err = ||v * (K^T u) - b||_2 at every 10th iteration
  stabilized SinkhornOT/sinkhorn_loss.py:159-356  (sinkhorn_iteration, gsinkhorn_iteration,
                                       forward_relax_sinkhorn_iteration): scaling a, b with
                                       clamps to 1e30, absorption into (u, v) every 10th
                                       iteration / when max(a|b) > 1e20 / at the last one,
                                       relative-tolerance test on sum(K*C) at each absorption
Independent of the HIP kernels, which run the same recursions in the log domain.
"""
import numpy as np

BIG, HUGE, SMALL = 1e20, 1e30, 1e-7


def knopp(a, b, M, reg, num_iter_max=1000, stop_thr=1e-9):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    M = np.asarray(M, np.float64)
    I, J = M.shape
    u = np.full(I, 1.0 / I)
    v = np.full(J, 1.0 / J)
    with np.errstate(all="ignore"):
        K = np.exp(M / -reg)
        Kp = K / a[:, None]
        cpt, err, broke = 0, 1.0, False
        while err > stop_thr and cpt < num_iter_max:
            u_prev, v_prev = u, v
            ktu = K.T @ u
            v = b / ktu
            u = 1.0 / (Kp @ v)
            if (np.any(ktu == 0) or np.any(np.isnan(u)) or np.any(np.isnan(v))
                    or np.any(np.isinf(u)) or np.any(np.isinf(v))):
                u, v = u_prev, v_prev
                broke = True
                break
            if cpt % 10 == 0:
                err = np.linalg.norm(v * (K.T @ u) - b)
            cpt += 1
        P = u[:, None] * K * v[None, :]
    return P, float(np.sum(P * M)), cpt, broke


def kl_div(x, y):
    d = x / (y + SMALL)
    return y * (d * np.log(d + SMALL) - d + 1)


def stabilized(C, mu, nu, eps, num_iter_max=100, tol=1e-9, mode="stab", lam=1.0):
    """mode: 'stab' (sinkhorn_iteration), 'gen' (gsinkhorn), 'relax' (forward_relax)."""
    C = np.asarray(C, np.float64)
    mu = np.asarray(mu, np.float64).reshape(-1, 1)
    nu = np.asarray(nu, np.float64).reshape(1, -1)
    p = lam / (lam + eps)
    pa = p if mode == "gen" else 1.0
    pb = p if mode in ("gen", "relax") else 1.0
    u = np.zeros_like(mu)
    v = np.zeros_like(nu)
    b = np.ones_like(nu)

    def kcalc():
        return np.clip(np.exp((u + v - C) / eps), 0, HUGE)

    with np.errstate(all="ignore"):
        K = kcalc()
        transport = np.float64(np.sum(K * C))
        transport_new = transport
        for ii in range(num_iter_max):
            a = np.clip((mu / np.sum(K * b, axis=1, keepdims=True)) ** pa, 0, HUGE)
            b = np.clip((nu / np.sum(K * a, axis=0, keepdims=True)) ** pb, 0, HUGE)
            if ii % 10 == 0 or a.max() > BIG or b.max() > BIG or ii == num_iter_max - 1:
                u = u + eps * np.log(a)
                v = v + eps * np.log(b)
                K = kcalc()
                b = np.ones_like(nu)
                transport_new = np.float64(np.sum(K * C))
                if abs(transport_new - transport) / abs(transport) < tol:
                    break
                transport = transport_new
        m1 = float(np.sum(kl_div(K.sum(axis=1, keepdims=True), mu)))
        m2 = float(np.sum(kl_div(K.sum(axis=0, keepdims=True), nu)))
    ret = transport_new if mode == "stab" else transport
    return float(ret), m1, m2, K
