"""The on-chip KNOPP kernel's timeout path on the device (csrc/sinkhorn.hip k_sk_res).

k_sk_res is a plain launch of at most one workgroup per CU whose workgroups hand row / column
partials to each other; nothing guarantees that they are all resident (an RCCL kernel on another
stream can hold CUs), so every inter-workgroup wait is bounded and a timed-out workgroup sets
GNNEA_SK_ST_TIMEOUT.  gnnea.sinkhorn then solves the problem again from the start on the sweep
path (utils/ot_loss.py:50-66 semantics either way).  The flag GNNEA_SK_DEBUG_SPIN gives every
wait a zero time budget, so a workgroup that finds a peer not yet arrived times out for real —
the kernel's own timeout, not a host-side fake (tests/test_sinkhorn_host.py covers the host
logic alone).
"""
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _problem(device, I=1000, J=900, seed=31):
    rng = np.random.default_rng(seed)
    M = torch.from_numpy(rng.uniform(0, 1, (I, J))).to(device)
    a = torch.ones(I, dtype=torch.float64, device=device)
    b = torch.full((J,), I / J, dtype=torch.float64, device=device)
    return M, a, b


def test_onchip_timeout_resolves_on_sweep(device):
    from gnnea import _lib
    from gnnea import sinkhorn as gsk
    M, a, b = _problem(device)
    K = _lib.GNNEA_SK_KNOPP
    ok = gsk.solve(K, M, a, b, 0.05, 1e-9, 200, variant=0)
    assert ok.path == "onchip" and ok.onchip_timeout is False
    sweep = gsk.solve(K, M, a, b, 0.05, 1e-9, 200, variant=0, flags=_lib.GNNEA_SK_NO_ONCHIP)
    assert sweep.path == "sweep"
    # the kernel itself reports the timeout through the status block ...
    with pytest.raises(gsk.SinkhornTimeout):
        gsk._solve(K, M, a, b, 0.05, 1e-9, 200, 1.0, torch.float64, True, 10, 0,
                   _lib.GNNEA_SK_DEBUG_SPIN)
    # ... and solve() re-solves on the sweep path: the sweep's result bit for bit, flagged
    t0 = time.perf_counter()
    to = gsk.solve(K, M, a, b, 0.05, 1e-9, 200, variant=0, flags=_lib.GNNEA_SK_DEBUG_SPIN)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert to.onchip_timeout is True and to.path == "sweep"
    assert (to.iters, to.reason) == (sweep.iters, sweep.reason)
    assert torch.equal(to.plan, sweep.plan)
    assert to.err == sweep.err and to.loss == sweep.loss
    assert torch.equal(to.row_sum, sweep.row_sum) and torch.equal(to.col_sum, sweep.col_sum)
    # the timed-out attempt ends at once (zero wait budget), not after a 250-ms spin per launch
    assert dt < 5.0, dt
    # the on-chip and sweep paths agree (both run the reference's scaling-form operations)
    assert (ok.iters, ok.reason) == (sweep.iters, sweep.reason)
    assert float((ok.plan - sweep.plan).abs().max() / sweep.plan.abs().max()) < 1e-12


def test_onchip_timeout_batch(device):
    """solve_batch (the GW / FGW inner solves): a timed-out batch is solved again on the sweep
    path as a whole; every problem flagged, each equal to its sweep solve bit for bit."""
    from gnnea import _lib
    from gnnea import sinkhorn as gsk
    Ms, As, Bs = zip(*[_problem(device, 700, 600, seed=s) for s in (1, 2, 3)])
    Cs, As, Bs = torch.stack(Ms), torch.stack(As), torch.stack(Bs)
    K = _lib.GNNEA_SK_KNOPP
    ref = gsk.solve_batch(K, Cs, As, Bs, 0.05, 1e-9, 120, variant=0,
                          flags=_lib.GNNEA_SK_NO_ONCHIP)
    got = gsk.solve_batch(K, Cs, As, Bs, 0.05, 1e-9, 120, variant=0,
                          flags=_lib.GNNEA_SK_DEBUG_SPIN)
    for r, g in zip(ref, got):
        assert g.onchip_timeout is True and r.onchip_timeout is False
        assert (g.iters, g.reason) == (r.iters, r.reason)
        assert torch.equal(g.plan, r.plan)
