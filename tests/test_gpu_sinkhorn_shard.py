"""§8e row-sharded KNOPP Sinkhorn (gnnea_sinkhorn_shard_*, csrc/sinkhorn_shard.hip).

The shards run on one device through gnnea.sinkhorn.solve_row_blocks: the same kernels and the
same rank-order merge of the gathered column pairs as solve_row_sharded over W ranks, with the
all-gather replaced by a stack.  Checked against the reference fixtures (tests/golden/
sinkhorn.npz, made from utils/ot_loss.py), the oracle restatement (oracle/sinkhorn.py:17-42) and
the unsharded device solve, including both numerical-error breaks (K^T u == 0 and an infinite
u, the latter detected one iteration late by the sharded loop and in the close step).
"""
import numpy as np
import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu

TOL64 = 1e-9


def _blocks(I, W):
    return [I * k // W for k in range(1, W)]


@pytest.fixture(params=[0, 1], ids=["scaling", "logdomain"])
def var(request):
    """Both sharded forms: the scaling form with each shard's fp64 K resident (variant 0) and the
    log-domain passes (variant 1)."""
    return request.param


@pytest.mark.parametrize("W", [2, 3])
@pytest.mark.parametrize("tag,reg", [("s", 0.05), ("m", 0.01), ("m", 0.05)])
def test_shard_vs_reference_fixture(golden, device, tag, reg, W, var):
    from gnnea.sinkhorn import solve_row_blocks
    S = golden("sinkhorn")
    M = torch.from_numpy(S["%s_M" % tag]).to(device)
    I, J = M.shape
    key = "%s_r%g" % (tag, reg)
    a = torch.ones(I, dtype=torch.float64, device=device)
    b = torch.ones(J, dtype=torch.float64, device=device)
    P, res = solve_row_blocks(M, a, b, reg, 1e-9, 1000, _blocks(I, W), variant=var)
    assert rel_err(P.cpu(), S[key + "_knopp_P"]) < TOL64
    ref_loss = float(S[key + "_knopp_loss"])
    assert abs(res.loss - ref_loss) <= TOL64 * abs(ref_loss)
    assert rel_err(res.col_sum.cpu(), P.sum(0).cpu()) < 1e-12


def test_shard_underflow_break(golden, device, var):
    from gnnea.sinkhorn import solve_row_blocks
    S = golden("sinkhorn")
    M = torch.from_numpy(S["under_M"]).to(device)
    I, J = M.shape
    a = torch.ones(I, dtype=torch.float64, device=device)
    b = torch.ones(J, dtype=torch.float64, device=device)
    for W in (2, 4):
        P, res = solve_row_blocks(M, a, b, 0.01, 1e-9, 1000, _blocks(I, W), variant=var)
        assert rel_err(P.cpu(), S["under_P"]) < TOL64
        assert res.reason == 2


@pytest.mark.parametrize("I,J,reg,W", [(50, 70, 0.1, 2), (257, 129, 0.02, 3), (1000, 1000, 0.01, 4),
                                       (3, 40, 0.05, 3)])
def test_shard_vs_oracle_and_unsharded(device, I, J, reg, W, var):
    from gnnea.sinkhorn import solve, solve_row_blocks
    from oracle import sinkhorn as osk
    import gnnea._lib as L
    rng = np.random.default_rng(I + J)
    M = rng.uniform(0, 1, (I, J))
    a = rng.uniform(0.5, 1.5, I)
    b = rng.uniform(0.5, 1.5, J)
    b *= a.sum() / b.sum()
    Md, ad, bd = (torch.from_numpy(x).to(device) for x in (M, a, b))
    P, res = solve_row_blocks(Md, ad, bd, reg, 1e-9, 300, _blocks(I, W), variant=var)
    Po, lo, cpt, broke = osk.knopp(a, b, M, reg, 300)
    assert rel_err(P.cpu(), Po) < TOL64
    assert abs(res.loss - lo) <= TOL64 * abs(lo)
    assert res.iters == cpt and (res.reason == 2) == broke
    ref = solve(L.GNNEA_SK_KNOPP, Md, ad, bd, reg, 1e-9, 300, variant=var)
    assert res.iters == ref.iters and res.reason == ref.reason
    assert rel_err(P.cpu(), ref.plan.cpu()) < 1e-11


def test_shard_tolerance_stop(device, var):
    """A loose stopThr ends the loop on the err test of an iterate 10n: same cpt as the
    reference loop (the sharded path evaluates it from the next iteration's gathered pairs)."""
    from gnnea.sinkhorn import solve_row_blocks
    from oracle import sinkhorn as osk
    rng = np.random.default_rng(5)
    I, J, reg = 300, 200, 0.05
    M = rng.uniform(0, 1, (I, J))
    a = np.full(I, 1.0 / I)
    b = np.full(J, 1.0 / J)
    for tol in (1e-3, 1e-6):
        P, res = solve_row_blocks(*(torch.from_numpy(x).to(device) for x in (M, a, b)), reg, tol,
                                  1000, _blocks(I, 3), variant=var)
        Po, lo, cpt, broke = osk.knopp(a, b, M, reg, 1000, tol)
        assert res.reason == 1 and res.iters == cpt and not broke, (tol, res.iters, cpt)
        assert rel_err(P.cpu(), Po) < TOL64


@pytest.mark.parametrize("max_iter", [1, 7, 300])
def test_shard_u_overflow_break(device, max_iter, var):
    """A row whose K is all zero (cost 100 at reg 0.1: exp(-1000) underflows) makes u infinite
    in iteration 0: the reference reverts to the initial scalings and stops with cpt = 0.  The
    sharded loop learns of it one iteration late (or in the close step when max_iter = 1)."""
    from gnnea.sinkhorn import solve, solve_row_blocks
    from oracle import sinkhorn as osk
    import gnnea._lib as L
    rng = np.random.default_rng(3)
    I, J, reg = 64, 48, 0.1
    M = rng.uniform(0, 1, (I, J))
    M[45] = 100.0
    a = np.full(I, 1.0 / I)
    b = np.full(J, 1.0 / J)
    Md, ad, bd = (torch.from_numpy(x).to(device) for x in (M, a, b))
    Po, lo, cpt, broke = osk.knopp(a, b, M, reg, max_iter)
    assert broke and cpt == 0
    P, res = solve_row_blocks(Md, ad, bd, reg, 1e-9, max_iter, _blocks(I, 2), variant=var)
    assert res.reason == 2 and res.iters == 0
    assert rel_err(P.cpu(), Po) < TOL64
    ref = solve(L.GNNEA_SK_KNOPP, Md, ad, bd, reg, 1e-9, max_iter, variant=var)
    assert ref.reason == 2 and ref.iters == 0
    assert rel_err(P.cpu(), ref.plan.cpu()) < 1e-12


def test_shard_b15000_vs_unsharded(device, var):
    """BASELINE's large Sinkhorn size (B = 15000), fp32 cost as ot_loss receives
    it: 4 row shards against the unsharded log-domain solve, 60 iterations, and the tolerance
    stop of the same problem (it converges in a few tens of iterations at stopThr 1e-9)."""
    from gnnea.sinkhorn import solve, solve_row_blocks
    import gnnea._lib as L
    g = torch.Generator(device=device).manual_seed(7)
    B = 15000
    M = torch.rand((B, B), generator=g, device=device, dtype=torch.float32)
    a = torch.full((B,), 1.0 / B, dtype=torch.float64, device=device)
    # stopThr < 0: the err test never passes, exactly 60 iterations run on both paths
    P, res = solve_row_blocks(M, a, a, 0.05, -1.0, 60, _blocks(B, 4), plan_dtype=torch.float32,
                              variant=var)
    ref = solve(L.GNNEA_SK_KNOPP, M, a, a, 0.05, -1.0, 60, plan_dtype=torch.float32,
                variant=var)
    assert res.iters == ref.iters == 60 and res.reason == ref.reason == 0
    d = (P - ref.plan).abs().max().item() / ref.plan.abs().max().item()
    assert d < 1e-6, d  # fp32 plan storage
    assert abs(res.loss - ref.loss) <= 1e-10 * abs(ref.loss)
    assert torch.allclose(res.col_sum, ref.col_sum, rtol=1e-10, atol=0)
    del P, ref
    _, res = solve_row_blocks(M, a, a, 0.05, 1e-9, 1000, _blocks(B, 4), want_plan=False,
                              variant=var)
    ref = solve(L.GNNEA_SK_KNOPP, M, a, a, 0.05, 1e-9, 1000, want_plan=False, variant=var)
    assert res.iters == ref.iters < 1000 and res.reason == ref.reason == 1
    assert abs(res.loss - ref.loss) <= 1e-10 * abs(ref.loss)


def _rank_worker(rank, world, port, q):
    import os
    import sys
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "gnn-mtl_amd"))
    sys.path.insert(0, root)
    from gnnea.sinkhorn import solve_row_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        rng = np.random.default_rng(21)
        I, J, reg = 401, 333, 0.02
        M = rng.uniform(0, 1, (I, J))
        a = rng.uniform(0.5, 1.5, I)
        b = np.full(J, a.sum() / J)
        r0, r1 = I * rank // world, I * (rank + 1) // world
        res = solve_row_sharded(torch.from_numpy(M[r0:r1]).to(dev),
                                torch.from_numpy(a[r0:r1]).to(dev), torch.from_numpy(b).to(dev),
                                reg, 1e-9, 500)
        q.put((rank, res.plan.cpu().numpy(), res.loss, res.iters, res.reason,
               res.col_sum.cpu().numpy()))
    finally:
        dist.destroy_process_group()


def test_shard_two_processes_gloo(device):
    """solve_row_sharded itself: 2 ranks (gloo, host-staged pair gather) on the one device."""
    import socket
    import torch.multiprocessing as mp
    from oracle import sinkhorn as osk
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 2
    procs = [ctx.Process(target=_rank_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(60)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    rng = np.random.default_rng(21)
    I, J, reg = 401, 333, 0.02
    M = rng.uniform(0, 1, (I, J))
    a = rng.uniform(0.5, 1.5, I)
    b = np.full(J, a.sum() / J)
    Po, lo, cpt, broke = osk.knopp(a, b, M, reg, 500)
    P = np.concatenate([o[1] for o in outs])
    assert rel_err(P, Po) < TOL64
    for o in outs:
        assert abs(o[2] - lo) <= TOL64 * abs(lo) and o[3] == cpt and (o[4] == 2) == broke
        assert rel_err(o[5], Po.sum(0)) < 1e-12
