"""Host logic of the Sinkhorn driver (no device): an on-chip solve whose inter-workgroup wait
timed out is solved again from the start with the on-chip path disabled (gnnea_sinkhorn.flags =
GNNEA_SK_NO_ONCHIP), once, and the result says so (onchip_timeout); a timeout on that path
propagates.  The device side of the same path: tests/test_gpu_sinkhorn_timeout.py."""
import types

import pytest

from gnnea import _lib, sinkhorn


@pytest.fixture(autouse=True)
def _fresh_timeout_state(monkeypatch):
    monkeypatch.setattr(sinkhorn, "_ONCHIP_TIMED_OUT", False)


def _fake(calls, fail_flags, batch=False):
    def f(*args):
        flags = args[-1]
        calls.append(flags)
        if flags in fail_flags:
            raise sinkhorn.SinkhornTimeout("timed out")
        r = types.SimpleNamespace(flags=flags)
        return [r, types.SimpleNamespace(flags=flags)] if batch else r
    return f


def test_solve_retries_on_the_sweep_path(monkeypatch):
    calls = []
    monkeypatch.setattr(sinkhorn, "_solve", _fake(calls, {0}))
    r = sinkhorn.solve(0, None, None, None, 0.01, 1e-9, 10)
    assert r.flags == _lib.GNNEA_SK_NO_ONCHIP and r.onchip_timeout is True
    assert calls == [0, _lib.GNNEA_SK_NO_ONCHIP]
    # the debug bit (zero wait budget) is dropped on the retry
    calls.clear()
    monkeypatch.setattr(sinkhorn, "_solve", _fake(calls, {_lib.GNNEA_SK_DEBUG_SPIN}))
    r = sinkhorn.solve(0, None, None, None, 0.01, 1e-9, 10, flags=_lib.GNNEA_SK_DEBUG_SPIN)
    assert calls == [_lib.GNNEA_SK_DEBUG_SPIN, _lib.GNNEA_SK_NO_ONCHIP]


def test_solve_batch_retries_and_second_timeout_propagates(monkeypatch):
    calls = []
    monkeypatch.setattr(sinkhorn, "_solve_batch", _fake(calls, {0}, batch=True))
    out = sinkhorn.solve_batch(0, None, None, None, 0.01, 1e-9, 10)
    assert [r.flags for r in out] == [_lib.GNNEA_SK_NO_ONCHIP] * 2
    assert all(r.onchip_timeout for r in out)
    calls.clear()
    monkeypatch.setattr(sinkhorn, "_ONCHIP_TIMED_OUT", False)  # (the timeout above is sticky)
    monkeypatch.setattr(sinkhorn, "_solve", _fake(calls, {0, _lib.GNNEA_SK_NO_ONCHIP}))
    with pytest.raises(sinkhorn.SinkhornTimeout):
        sinkhorn.solve(0, None, None, None, 0.01, 1e-9, 10)
    assert calls == [0, _lib.GNNEA_SK_NO_ONCHIP]


def test_problem_struct_carries_flags():
    p = _lib.SinkhornProblem(flags=_lib.GNNEA_SK_NO_ONCHIP)
    assert p.flags == 1
    names = [f[0] for f in _lib.SinkhornProblem._fields_]
    assert names[-2:] == ["flags", "ws"]


def test_default_flags_after_a_real_timeout(monkeypatch):
    """The on-chip solver stays the default in a multi-rank process group (rank-local solves);
    after one real timeout in this process -- re-solved on the sweep path -- later default solves
    start on the sweep; a timeout under GNNEA_SK_DEBUG_SPIN (the tests' forced one) changes
    nothing."""
    import torch.distributed as dist
    monkeypatch.setattr(sinkhorn, "_ONCHIP_TIMED_OUT", False)
    monkeypatch.setattr(dist, "is_initialized", lambda: True)
    monkeypatch.setattr(dist, "get_world_size", lambda group=None: 4)
    assert sinkhorn._default_flags() == sinkhorn.DEFAULT_FLAGS
    calls = []
    monkeypatch.setattr(sinkhorn, "_solve", _fake(calls, {_lib.GNNEA_SK_DEBUG_SPIN}))
    sinkhorn.solve(0, None, None, None, 0.01, 1e-9, 10, flags=_lib.GNNEA_SK_DEBUG_SPIN)
    assert sinkhorn._default_flags() == sinkhorn.DEFAULT_FLAGS
    calls.clear()
    monkeypatch.setattr(sinkhorn, "_solve", _fake(calls, {0}))
    sinkhorn.solve(0, None, None, None, 0.01, 1e-9, 10)
    assert calls == [0, _lib.GNNEA_SK_NO_ONCHIP]
    assert sinkhorn._default_flags() & _lib.GNNEA_SK_NO_ONCHIP
    calls.clear()
    sinkhorn.solve(0, None, None, None, 0.01, 1e-9, 10)
    assert calls == [_lib.GNNEA_SK_NO_ONCHIP]
