"""Host driver of the Sinkhorn kernels (gnnea_sinkhorn_*, scaling form with a resident fp64 K).

The loop has data-dependent exits (tolerance, numerical-error break), so the host enqueues
iterations in batches and reads the device status block between batches; kernels of iterations
past the stop condition are no-ops on the device.  All arithmetic is fp64 in the kernels.
"""
import ctypes

import torch

from . import _lib
from ._lib import SinkhornProblem, check, ptr, stream_of

ST_DONE, ST_ITERS, ST_REASON, ST_SLOT = 0, 1, 2, 3
# path of solve() calls that do not choose one: 0 = scaling form with the resident fp64 K
# (falls back to 1 above J = 16384), 1 = log-domain passes (no I x J workspace; KNOPP: the fused
# sweep), 3 = GNNEA_SK_AUTO: KNOPP on chip where it fits, else the fused log-domain sweep (one
# pass over C per iteration), the STAB family as 0
DEFAULT_VARIANT = _lib.GNNEA_SK_AUTO
# gnnea_sinkhorn.flags of solve() calls that pass none (the drop-in ot_loss / sinkhorn_loss
# functions): 0; tests select a path by setting it (GNNEA_SK_NO_ONCHIP: the resident-K sweep)
DEFAULT_FLAGS = 0
SD_ERR, SD_TPREV, SD_LOSS, SD_TNEW = 8, 9, 10, 12  # GNNEA_SK_SD_* (include/gnnea.h)
MAX_BATCH = 100  # iterations enqueued between two host polls of the status block, at most


class SinkhornResult:
    def __init__(self, plan, row_sum, col_sum, iters, reason, err, transport_new, transport_prev,
                 loss):
        self.plan = plan
        self.row_sum = row_sum
        self.col_sum = col_sum
        self.iters = iters
        self.reason = reason  # 0 max-iter, 1 tolerance, 2 numerical-error break
        self.err = err
        self.transport_new = transport_new
        self.transport_prev = transport_prev
        self.loss = loss


class SinkhornTimeout(RuntimeError):
    """A wait between the workgroups of the on-chip KNOPP kernel timed out (results invalid):
    its persistent grid was not all resident, e.g. because another stream's kernel (an RCCL
    collective) held CUs.  solve() / solve_batch() re-run the problem on the sweep path."""


def _status(ws):
    raw = ws[:_lib.GNNEA_SK_STATUS_BYTES].cpu()  # sync point between batches
    ints = raw.view(torch.int64)
    dbl = raw.view(torch.float64)
    if int(ints[_lib.GNNEA_SK_ST_TIMEOUT]):
        raise SinkhornTimeout("gnnea.sinkhorn: a wait between the workgroups of the on-chip "
                              "KNOPP kernel timed out (results invalid)")
    return ints, dbl


class _StatusPoll:
    """Look-ahead read of the device status block: after enqueueing batch k the host reads the
    status copied after batch k-1 (an async copy into pinned memory and an event), so the queue
    never drains while the host decides — the GPU runs batch k meanwhile — at the price of one
    batch of no-op launches after the stop.  ``done()`` is None until a copy is in flight."""

    def __init__(self, ws, rows=1, stride=None):
        self.src = ws if stride is None else ws.view(rows, stride)
        self.buf = torch.empty((rows, 8), dtype=torch.int64, pin_memory=True)
        self.ev = None

    def post(self):
        src = self.src[:64].view(torch.int64).view(1, 8) if self.src.dim() == 1 else \
            self.src[:, :64].contiguous().view(torch.int64)
        self.buf.copy_(src, non_blocking=True)
        self.ev = torch.cuda.Event()
        self.ev.record()

    def done(self):
        if self.ev is None:
            return None
        self.ev.synchronize()
        return self.buf[:, ST_DONE].clone()


# Set once an on-chip solve of this process timed out for real (not under GNNEA_SK_DEBUG_SPIN):
# the on-chip solver needs all its workgroups resident at once, which another stream's kernels
# holding CUs (an RCCL collective still in flight) can prevent; after one such timeout -- whose
# problem is re-solved on the sweep path -- later default solves start on the sweep.
_ONCHIP_TIMED_OUT = False


def _default_flags():
    """DEFAULT_FLAGS, plus GNNEA_SK_NO_ONCHIP once an on-chip solve has timed out in this
    process.  Rank-local solves of a multi-rank job (evaluation, per-rank OT losses) keep the
    on-chip path: a collective in flight costs at most one bounded wait and a re-solve."""
    if _ONCHIP_TIMED_OUT:
        return DEFAULT_FLAGS | _lib.GNNEA_SK_NO_ONCHIP
    return DEFAULT_FLAGS


def _note_timeout(flags):
    global _ONCHIP_TIMED_OUT
    if not flags & _lib.GNNEA_SK_DEBUG_SPIN:
        _ONCHIP_TIMED_OUT = True


def _retry_flags(flags):
    """The re-solve after an on-chip timeout: never on chip (the debug bit is moot there)."""
    return (flags | _lib.GNNEA_SK_NO_ONCHIP) & ~_lib.GNNEA_SK_DEBUG_SPIN


def solve(mode, C, a, b, eps, tol, max_iter, p=1.0, plan_dtype=torch.float64,
          want_plan=True, batch=10, variant=None, flags=None):
    """Run one Sinkhorn solve; C is [I, J] fp32 / fp64 on a HIP device, a / b the weights.
    ``flags``: gnnea_sinkhorn.flags bits (GNNEA_SK_NO_ONCHIP, GNNEA_SK_TWO_PASS,
    GNNEA_SK_DEBUG_SPIN).  An on-chip solve whose inter-workgroup wait timed out is solved again
    from the start on the sweep path (same iterates: both paths run the reference's operations);
    the result then carries ``onchip_timeout = True``."""
    flags = _default_flags() if flags is None else flags
    try:
        return _solve(mode, C, a, b, eps, tol, max_iter, p, plan_dtype, want_plan, batch,
                      variant, flags)
    except SinkhornTimeout:
        _note_timeout(flags)
        res = _solve(mode, C, a, b, eps, tol, max_iter, p, plan_dtype, want_plan, batch,
                     variant, _retry_flags(flags))
        res.onchip_timeout = True
        return res


def _solve(mode, C, a, b, eps, tol, max_iter, p, plan_dtype, want_plan, batch, variant, flags):
    _lib.require_device(C, a, b)
    if variant is None:
        variant = DEFAULT_VARIANT
    if C.dim() != 2:
        raise ValueError("gnnea.sinkhorn: C must be 2-D")
    if C.dtype not in (torch.float32, torch.float64):
        C = C.double()
    if C.stride(1) != 1:
        C = C.contiguous()
    I, J = C.shape
    dev = C.device
    wa = a.reshape(-1).to(torch.float64).contiguous()
    wb = b.reshape(-1).to(torch.float64).contiguous()
    if wa.numel() != I or wb.numel() != J:
        raise ValueError("gnnea.sinkhorn: weights must have I and J entries")
    L = _lib.lib()
    ws_bytes = int(L.gnnea_sinkhorn_ws_bytes(I, J))
    if ws_bytes < 0:
        check(ws_bytes)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    prob = SinkhornProblem(
        mode=mode, c_dtype=_lib.GNNEA_F32 if C.dtype == torch.float32 else _lib.GNNEA_F64,
        I=I, J=J, ldc=C.stride(0), C=C.data_ptr(), a=wa.data_ptr(), b=wb.data_ptr(),
        eps=float(eps), p=float(p), tol=float(tol), max_iter=int(max_iter), iters_run=0,
        variant=int(variant), flags=flags, ws=ws.data_ptr())
    pp = ctypes.byref(prob)
    st = stream_of(dev)
    with _lib.on_device(dev):
        path = L.gnnea_sinkhorn_path(pp)
        check(L.gnnea_sinkhorn_init(pp, st))
        run = 0
        # The device decides every stop itself (iterations past it are no-op launches), so the
        # host reads the status block only between batches that grow geometrically up to
        # MAX_BATCH, one batch behind (_StatusPoll: the GPU never waits for the host), at the
        # price of at most two batches of no-ops after the stop.
        poll = _StatusPoll(ws)
        if mode == _lib.GNNEA_SK_KNOPP:
            # utils/ot_loss.py:50  while err > stopThr and cpt < numItermax  (err starts at 1);
            # iteration k's err is evaluated by iteration k+1's combine: batches end at 10n + 2
            if 1.0 > tol and max_iter > 0:
                step, hi = 10, 2
                while run < max_iter:
                    hi = min(hi, max_iter)
                    check(L.gnnea_sinkhorn_iterate(pp, run, hi - run, st))
                    run = hi
                    done = poll.done()
                    if done is not None and done[0].item():
                        break
                    poll.post()
                    hi = run + step
                    step = min(2 * step, MAX_BATCH)
        else:
            step = max(1, batch)
            while run < max_iter:
                n = min(step, max_iter - run)
                check(L.gnnea_sinkhorn_iterate(pp, run, n, st))
                run += n
                done = poll.done()
                if done is not None and done[0].item():
                    break
                poll.post()
                step = min(2 * step, max(batch, MAX_BATCH))
        prob.iters_run = run
        plan = torch.empty((I, J), dtype=plan_dtype, device=dev) if want_plan else None
        row_sum = torch.empty(I, dtype=torch.float64, device=dev)
        col_sum = torch.empty(J, dtype=torch.float64, device=dev)
        check(L.gnnea_sinkhorn_finish(
            pp, ptr(plan), _lib.GNNEA_F32 if plan_dtype == torch.float32 else _lib.GNNEA_F64,
            J, ptr(row_sum), ptr(col_sum), st))
        ints, dbl = _status(ws)
    res = SinkhornResult(plan, row_sum, col_sum, int(ints[ST_ITERS]), int(ints[ST_REASON]),
                         float(dbl[SD_ERR]), float(dbl[SD_TNEW]), float(dbl[SD_TPREV]),
                         float(dbl[SD_LOSS]))
    res.path = ("sweep", "onchip", "logdomain")[path]  # gnnea_sinkhorn_path
    res.onchip_timeout = False
    return res


def solve_batch(mode, Cs, As, Bs, eps, tol, max_iter, p=1.0, plan_dtype=torch.float64, batch=10,
                variant=None, flags=None):
    """Solve a batch of problems of one shape [bt, I, J] as ONE launch sequence: every problem's
    iterations are enqueued batch by batch on the same stream and ONE device->host copy of all
    status blocks per round decides which problems continue (solve() polls once per problem
    per round).  Cs [bt, I, J], As [bt, I], Bs [bt, J] on the device; returns SinkhornResults.
    A timed-out on-chip wait re-runs the batch on the sweep path, as solve() does."""
    flags = _default_flags() if flags is None else flags
    try:
        return _solve_batch(mode, Cs, As, Bs, eps, tol, max_iter, p, plan_dtype, batch, variant,
                            flags)
    except SinkhornTimeout:
        _note_timeout(flags)
        out = _solve_batch(mode, Cs, As, Bs, eps, tol, max_iter, p, plan_dtype, batch, variant,
                           _retry_flags(flags))
        for r in out:
            r.onchip_timeout = True
        return out


def _solve_batch(mode, Cs, As, Bs, eps, tol, max_iter, p, plan_dtype, batch, variant, flags):
    _lib.require_device(Cs, As, Bs)
    if variant is None:
        variant = DEFAULT_VARIANT
    bt, I, J = Cs.shape
    if Cs.dtype not in (torch.float32, torch.float64):
        Cs = Cs.double()
    dev = Cs.device
    L = _lib.lib()
    ws_bytes = int(L.gnnea_sinkhorn_ws_bytes(I, J))
    if ws_bytes < 0:
        check(ws_bytes)
    stride = (ws_bytes + 255) // 256 * 256
    ws = torch.empty(bt * stride, dtype=torch.uint8, device=dev)
    wa = As.reshape(bt, I).to(torch.float64).contiguous()
    wb = Bs.reshape(bt, J).to(torch.float64).contiguous()
    probs = []
    for k in range(bt):
        C = Cs[k] if Cs[k].stride(1) == 1 else Cs[k].contiguous()
        probs.append((C, SinkhornProblem(
            mode=mode, c_dtype=_lib.GNNEA_F32 if C.dtype == torch.float32 else _lib.GNNEA_F64,
            I=I, J=J, ldc=C.stride(0), C=C.data_ptr(), a=wa[k].data_ptr(), b=wb[k].data_ptr(),
            eps=float(eps), p=float(p), tol=float(tol), max_iter=int(max_iter), iters_run=0,
            variant=int(variant), flags=flags, ws=ws[k * stride:].data_ptr())))
    st = stream_of(dev)
    status = ws.view(bt, stride)[:, :_lib.GNNEA_SK_STATUS_BYTES]
    results = []
    with _lib.on_device(dev):
        for _, pr in probs:
            check(L.gnnea_sinkhorn_init(ctypes.byref(pr), st))
        run = 0
        live = list(range(bt))
        knopp = mode == _lib.GNNEA_SK_KNOPP
        if knopp and not (1.0 > tol and max_iter > 0):
            live = []
        step, hi = (10, 2) if knopp else (max(1, batch), max(1, batch))
        poll = _StatusPoll(ws, bt, stride)  # one look-ahead read of all status blocks per round
        while live and run < max_iter:
            hi = min(hi, max_iter)
            for k in live:
                check(L.gnnea_sinkhorn_iterate(ctypes.byref(probs[k][1]), run, hi - run, st))
            for k in live:
                probs[k][1].iters_run = hi
            run = hi
            done = poll.done()
            if done is not None:
                live = [k for k in live if not int(done[k])]
            poll.post()
            hi = run + step
            step = min(2 * step, MAX_BATCH)
        for k, (C, pr) in enumerate(probs):
            pr.iters_run = max(pr.iters_run, 0)
            plan = torch.empty((I, J), dtype=plan_dtype, device=dev)
            row_sum = torch.empty(I, dtype=torch.float64, device=dev)
            col_sum = torch.empty(J, dtype=torch.float64, device=dev)
            check(L.gnnea_sinkhorn_finish(
                ctypes.byref(pr), ptr(plan),
                _lib.GNNEA_F32 if plan_dtype == torch.float32 else _lib.GNNEA_F64, J,
                ptr(row_sum), ptr(col_sum), st))
            results.append((plan, row_sum, col_sum))
        raw = status.contiguous().cpu()
    out = []
    for k, (plan, row_sum, col_sum) in enumerate(results):
        ints = raw[k].view(torch.int64)
        dbl = raw[k].view(torch.float64)
        if int(ints[_lib.GNNEA_SK_ST_TIMEOUT]):
            raise SinkhornTimeout("gnnea.sinkhorn: an inter-workgroup wait timed out (problem %d)"
                                  % k)
        out.append(SinkhornResult(plan, row_sum, col_sum, int(ints[ST_ITERS]),
                                  int(ints[ST_REASON]), float(dbl[SD_ERR]), float(dbl[SD_TNEW]),
                                  float(dbl[SD_TPREV]), float(dbl[SD_LOSS])))
        out[-1].onchip_timeout = False
    return out


# ------------------------------------------------------------------------------------------------
# §8e: KNOPP with the cost rows sharded over ranks (gnnea_sinkhorn_shard_*).  Rank r holds a
# contiguous block of rows; per iteration every rank reduces its rows to one row per column —
# the column sums of K^T u in the scaling form (variant 0, J <= 16384: the rank's fp64 K resident,
# sinkhorn.hip) or (max, sum-exp) pairs in the log domain (variant 1, sinkhorn_shard.hip) — the
# rows are all-gathered (one collective of W x pair_len doubles) and each rank merges them in
# rank order, so v and all stop decisions are bit-identical on every rank: the ranks poll their
# own status block and leave the loop on the same iteration.

class _Shard:
    """One rank's row block as a gnnea_sinkhorn problem (KNOPP)."""

    def __init__(self, C, a, b, reg, tol, max_iter, I_global, variant=0):
        _lib.require_device(C, a, b)
        if C.dim() != 2:
            raise ValueError("gnnea.sinkhorn: C must be 2-D")
        if C.dtype not in (torch.float32, torch.float64):
            C = C.double()
        if C.stride(1) != 1:
            C = C.contiguous()
        self.C = C
        self.I, self.J = C.shape
        self.a = a.reshape(-1).to(torch.float64).contiguous()
        self.b = b.reshape(-1).to(torch.float64).contiguous()
        if self.a.numel() != self.I or self.b.numel() != self.J:
            raise ValueError("gnnea.sinkhorn: weights must have I_local and J entries")
        L = _lib.lib()
        nb = int(L.gnnea_sinkhorn_shard_ws_bytes(self.I, self.J))
        if nb < 0:
            check(nb)
        dev = C.device
        self.ws = torch.empty(nb, dtype=torch.uint8, device=dev)
        self.flag = torch.empty(1, dtype=torch.float64, device=dev)
        self.prob = SinkhornProblem(
            mode=_lib.GNNEA_SK_KNOPP,
            c_dtype=_lib.GNNEA_F32 if C.dtype == torch.float32 else _lib.GNNEA_F64,
            I=self.I, J=self.J, ldc=C.stride(0), C=C.data_ptr(), a=self.a.data_ptr(),
            b=self.b.data_ptr(), eps=float(reg), p=1.0, tol=float(tol), max_iter=int(max_iter),
            iters_run=0, variant=int(variant), flags=0, ws=self.ws.data_ptr())
        self.pp = ctypes.byref(self.prob)
        # the gathered row: column sums (scaling form, K resident) or (max, sum-exp) pairs
        n = int(L.gnnea_sinkhorn_shard_pair_len(self.pp))
        if n < 0:
            check(n)
        self.pair = torch.empty(n, dtype=torch.float64, device=dev)
        self.st = stream_of(dev)
        check(L.gnnea_sinkhorn_shard_init(self.pp, int(I_global), self.st))


def _run_shards(shards, gather, reduce_sum, max_iter, tol, want_plan, plan_dtype):
    """The iteration loop over the shards this process drives; gather(list of local [n] tensors)
    -> [W, n] in rank order, reduce_sum(list of local tensors) -> their sum over all ranks."""
    L = _lib.lib()
    ref = shards[0]
    run = 0
    if 1.0 > tol and max_iter > 0:  # utils/ot_loss.py:50 (err starts at 1)
        step, hi = 10, 2
        while run < max_iter:
            hi = min(hi, max_iter)
            for it in range(run, hi):
                for s in shards:
                    check(L.gnnea_sinkhorn_shard_colpart(s.pp, it, ptr(s.pair), s.st))
                pairs = gather([s.pair for s in shards])
                W = pairs.shape[0]
                for s in shards:
                    check(L.gnnea_sinkhorn_shard_step(s.pp, it, ptr(pairs), W, s.st))
            run = hi
            if _status(ref.ws)[0][ST_DONE].item():
                break
            hi = run + step
            step = min(2 * step, MAX_BATCH)
    for s in shards:
        s.prob.iters_run = run
        check(L.gnnea_sinkhorn_shard_flag(s.pp, ptr(s.flag), s.st))
    flags = gather([s.flag for s in shards])
    W = flags.shape[0]
    out = []
    for s in shards:
        check(L.gnnea_sinkhorn_shard_close(s.pp, ptr(flags), W, s.st))
        plan = (torch.empty((s.I, s.J), dtype=plan_dtype, device=s.C.device)
                if want_plan else None)
        row_sum = torch.empty(s.I, dtype=torch.float64, device=s.C.device)
        loss = torch.empty(1, dtype=torch.float64, device=s.C.device)
        col = torch.empty(s.J, dtype=torch.float64, device=s.C.device)
        check(L.gnnea_sinkhorn_shard_finish(
            s.pp, ptr(plan), _lib.GNNEA_F32 if plan_dtype == torch.float32 else _lib.GNNEA_F64,
            s.J, ptr(row_sum), ptr(loss), ptr(col), s.st))
        out.append((plan, row_sum, loss, col))
    loss = reduce_sum([o[2] for o in out])
    col_sum = reduce_sum([o[3] for o in out])
    results = []
    for s, (plan, row_sum, _, _) in zip(shards, out):
        ints, dbl = _status(s.ws)
        results.append(SinkhornResult(plan, row_sum, col_sum, int(ints[ST_ITERS]),
                                      int(ints[ST_REASON]), float(dbl[SD_ERR]), 0.0, 0.0,
                                      float(loss.item())))
    return results


def solve_row_sharded(C_loc, a_loc, b, reg, tol, max_iter, group=None,
                      plan_dtype=torch.float64, want_plan=True, variant=None):
    """KNOPP over this rank's cost rows C_loc [I_loc, J] (ranks hold consecutive row blocks in
    rank order), a_loc its rows' source weights, b all J target weights.  One all-gather of the
    column pairs per iteration over `group` (RCCL on HIP devices).  Returns this rank's
    SinkhornResult: plan / row_sum of its rows, col_sum and loss of the whole plan."""
    import torch.distributed as dist
    W = dist.get_world_size(group)
    dev = C_loc.device
    n = torch.tensor([C_loc.shape[0]], dtype=torch.int64)
    if dist.get_backend(group) != "gloo":
        n = n.to(dev)
    dist.all_reduce(n, group=group)

    # gloo (CPU tests, a single-GPU rehearsal) exchanges host copies; RCCL the device buffers
    host = dist.get_backend(group) == "gloo"

    def gather(ts):
        (t,) = ts
        src = t.cpu() if host else t
        out = torch.empty(W * t.numel(), dtype=t.dtype, device=src.device)
        dist.all_gather_into_tensor(out, src, group=group)
        return out.view(W, t.numel()).to(dev)

    def reduce_sum(ts):
        (t,) = ts
        t = t.cpu() if host else t.clone()
        dist.all_reduce(t, group=group)
        return t.to(dev)

    with _lib.on_device(dev):
        shard = _Shard(C_loc, a_loc, b, reg, tol, max_iter, int(n.item()),
                       DEFAULT_VARIANT if variant is None else variant)
        return _run_shards([shard], gather, reduce_sum, max_iter, tol, want_plan, plan_dtype)[0]


def solve_row_blocks(C, a, b, reg, tol, max_iter, row_splits, plan_dtype=torch.float64,
                     want_plan=True, variant=None):
    """The row-sharded solve with every shard driven by this process on C's device (the
    exchange is a stack of the shards' pair rows in rank order): the same kernels and the same
    merge order as solve_row_sharded over len(row_splits) + 1 ranks, for tests and for a single
    device.  row_splits: the first row of shards 1..W-1.  Returns (plan, SinkhornResult)."""
    _lib.require_device(C, a, b)
    I = C.shape[0]
    bounds = [0] + list(row_splits) + [I]
    if any(bounds[k] >= bounds[k + 1] for k in range(len(bounds) - 1)):
        raise ValueError("gnnea.sinkhorn: row blocks must be non-empty and increasing")
    with _lib.on_device(C.device):
        var = DEFAULT_VARIANT if variant is None else variant
        shards = [_Shard(C[bounds[k]:bounds[k + 1]], a.reshape(-1)[bounds[k]:bounds[k + 1]], b,
                         reg, tol, max_iter, I, var) for k in range(len(bounds) - 1)]

        def gather(ts):
            return torch.stack(ts)

        def reduce_sum(ts):
            out = ts[0].clone()
            for t in ts[1:]:
                out += t
            return out

        res = _run_shards(shards, gather, reduce_sum, max_iter, tol, want_plan, plan_dtype)
    plan = torch.cat([r.plan for r in res]) if want_plan else None
    r0 = res[0]
    row_sum = torch.cat([r.row_sum for r in res])
    return plan, SinkhornResult(plan, row_sum, r0.col_sum, r0.iters, r0.reason, r0.err, 0.0, 0.0,
                                r0.loss)
