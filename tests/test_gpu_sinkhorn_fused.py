"""The fused log-domain KNOPP sweep (csrc/sinkhorn_log.hip k_lsk_sweep + k_lsk_colfin: one pass
over C per iteration, one exponential per element) against the two-pass log-domain form
(flag GNNEA_SK_TWO_PASS), the scaling form and the fp64 oracle (utils/ot_loss.py:5-76 restated in
oracle/sinkhorn.py).  The fused path is what variant 1 runs for KNOPP at J <= 16384 (fp32 C;
8192 for fp64 C); every variant-1 fixture test (test_gpu_parity.py, test_gpu_scale_dbp15k.py)
runs through it as well.

Same stop iteration and reason as the two-pass form, plans at 1e-12 (the two sum in different
orders and take exponentials from different tables), the oracle at 1e-9; the column update's
exact recomputation (a column whose K^T u falls outside [2^-600, 2^600]) and the breaks
(an all-underflow column, an all-underflow row, NaN / -inf costs) exercised explicitly.
"""
import numpy as np
import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu
TOL64 = 1e-9


def _solve(two_pass, M, a, b, reg, tol=1e-9, iters=300, variant=1, flags=0):
    from gnnea import _lib
    from gnnea.sinkhorn import solve
    return solve(_lib.GNNEA_SK_KNOPP, M, a, b, reg, tol, iters, variant=variant,
                 flags=flags | (_lib.GNNEA_SK_TWO_PASS if two_pass else 0))


@pytest.mark.parametrize("I,J,reg,dtype", [(300, 200, 0.05, torch.float64),
                                           (1000, 1500, 0.01, torch.float32),
                                           (3000, 3000, 0.01, torch.float32),
                                           (777, 4100, 0.02, torch.float64),
                                           (2000, 9000, 0.02, torch.float32),
                                           (257, 16384, 0.05, torch.float32),
                                           (5000, 700, 0.005, torch.float32)])
def test_fused_matches_two_pass(device, monkeypatch, I, J, reg, dtype):
    rng = np.random.default_rng(I + 3 * J)
    M = rng.uniform(0, 1, (I, J))
    a = rng.uniform(0.5, 1.5, I)
    b = rng.uniform(0.5, 1.5, J)
    b *= a.sum() / b.sum()
    Mt = torch.from_numpy(M).to(device=device, dtype=dtype)
    at, bt = torch.from_numpy(a).to(device), torch.from_numpy(b).to(device)
    rf = _solve(False, Mt, at, bt, reg)
    r2 = _solve(True, Mt, at, bt, reg)
    assert rf.path == r2.path == "logdomain"
    assert (rf.iters, rf.reason) == (r2.iters, r2.reason), ((rf.iters, rf.reason),
                                                            (r2.iters, r2.reason))
    assert rel_err(rf.plan.cpu(), r2.plan.cpu()) < 1e-12
    assert abs(rf.loss - r2.loss) <= 1e-12 * abs(r2.loss)
    assert abs(rf.err - r2.err) <= 1e-9 * abs(r2.err) + 1e-12 * float(np.linalg.norm(b))
    if I * J <= 4_000_000:
        from oracle import sinkhorn as osk
        Mo = Mt.double().cpu().numpy()
        Po, lo, _, _ = osk.knopp(a, b, Mo, reg, 300)
        assert rel_err(rf.plan.cpu(), Po) < TOL64
        assert abs(rf.loss - lo) <= TOL64 * abs(lo)


def test_fused_matches_scaling_form(device, monkeypatch):
    """The fused sweep against the reference's own scaling form (variant 0, resident K)."""
    rng = np.random.default_rng(5)
    I, J, reg = 2500, 6000, 0.01
    M = torch.from_numpy(rng.uniform(0, 1, (I, J))).to(device=device, dtype=torch.float32)
    a = torch.ones(I, dtype=torch.float64, device=device)
    b = torch.full((J,), I / J, dtype=torch.float64, device=device)
    from gnnea import _lib
    rf = _solve(False, M, a, b, reg)
    rs = _solve(False, M, a, b, reg, variant=0, flags=_lib.GNNEA_SK_NO_ONCHIP)
    assert (rf.path, rs.path) == ("logdomain", "sweep")
    assert (rf.iters, rf.reason) == (rs.iters, rs.reason)
    assert rel_err(rf.plan.cpu(), rs.plan.cpu()) < 1e-11
    assert abs(rf.loss - rs.loss) <= 1e-11 * abs(rs.loss)


def test_fused_exact_column_recompute(device, monkeypatch):
    """Columns whose K^T u is tiny but not zero (K entries ~1e-300: k = -C / reg near -690):
    S_j falls below 2^-600, the column update recomputes the column exactly from C; the plan
    and the stop agree with the two-pass form and the oracle."""
    rng = np.random.default_rng(9)
    I, J, reg = 400, 300, 0.01
    M = rng.uniform(0, 1, (I, J))
    M[:, 17] = 6.9 + 0.001 * rng.uniform(0, 1, I)  # exp(-690) ~ 1e-300 per entry
    M[:, 230] = 7.2                                    # exp(-720) ~ 1e-313: subnormal K
    a, b = np.ones(I), np.ones(J) * I / J
    Mt, at, bt = (torch.from_numpy(x).to(device) for x in (M, a, b))
    rf = _solve(False, Mt, at, bt, reg, iters=200)
    r2 = _solve(True, Mt, at, bt, reg, iters=200)
    assert (rf.iters, rf.reason) == (r2.iters, r2.reason), ((rf.iters, rf.reason),
                                                            (r2.iters, r2.reason))
    f = torch.isfinite(r2.plan)
    assert torch.equal(torch.isfinite(rf.plan), f)
    assert rel_err(rf.plan[f].cpu(), r2.plan[f].cpu()) < 1e-12


@pytest.mark.parametrize("what", ["column", "row", "nan", "-inf"])
def test_fused_breaks(device, monkeypatch, what):
    """The breaks of ot_loss.py:57-62 through the fused sweep: an all-underflow column (K^T u
    == 0), an all-underflow row (Kp v == 0: u = inf), a NaN and a -inf cost; the same stop
    iteration, reason and reverted plan as the two-pass form."""
    rng = np.random.default_rng(13)
    I, J, reg = 500, 350, 0.05
    M = rng.uniform(0, 1, (I, J))
    if what == "column":
        M[:, 41] = 50.0
    elif what == "row":
        M[17] = 50.0
    elif what == "nan":
        M[7, 11] = float("nan")
    else:
        M[7, 11] = float("-inf")
    a, b = np.ones(I), np.ones(J) * I / J
    Mt, at, bt = (torch.from_numpy(x).to(device) for x in (M, a, b))
    rf = _solve(False, Mt, at, bt, reg, iters=50)
    r2 = _solve(True, Mt, at, bt, reg, iters=50)
    assert (rf.iters, rf.reason) == (r2.iters, r2.reason), ((rf.iters, rf.reason),
                                                            (r2.iters, r2.reason))
    assert rf.reason == 2
    f = torch.isfinite(r2.plan)
    assert torch.equal(torch.isfinite(rf.plan), f)
    assert rel_err(rf.plan[f].cpu(), r2.plan[f].cpu()) < 1e-12


def test_auto_routing(device, monkeypatch):
    """GNNEA_SK_AUTO (the default): KNOPP on chip where the blocks fit the CUs, else the fused
    log-domain sweep; the STAB family on the scaling form; fp64 C past the fused sweep's limit
    (J > 8192) on the scaling form too.  The fused result equals the explicit variant 1's."""
    from gnnea import _lib
    from gnnea.sinkhorn import solve
    rng = np.random.default_rng(21)

    def run(I, J, mode, dtype, variant=None):
        M = torch.from_numpy(rng.uniform(0, 1, (I, J))).to(device=device, dtype=dtype)
        a = torch.ones(I, dtype=torch.float64, device=device)
        b = torch.full((J,), I / J, dtype=torch.float64, device=device)
        if mode == _lib.GNNEA_SK_STAB:
            a, b = a / I, b / I
        return M, a, b, solve(mode, M, a, b, 0.02, 1e-9, 60, variant=variant)
    assert run(500, 400, _lib.GNNEA_SK_KNOPP, torch.float32)[3].path == "onchip"
    M, a, b, r = run(6000, 5000, _lib.GNNEA_SK_KNOPP, torch.float32)
    assert r.path == "logdomain"
    r1 = solve(_lib.GNNEA_SK_KNOPP, M, a, b, 0.02, 1e-9, 60, variant=1)
    assert (r.iters, r.reason) == (r1.iters, r1.reason) and torch.equal(r.plan, r1.plan)
    assert run(3000, 2000, _lib.GNNEA_SK_STAB, torch.float64)[3].path == "sweep"
    assert run(300, 9000, _lib.GNNEA_SK_KNOPP, torch.float64)[3].path in ("sweep", "onchip")
