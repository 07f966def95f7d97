"""Halo exchange inside a KG group: direct peer transfers (SURVEY.md §8e "Transport").

MI355X nodes connect every GPU pair by its own xGMI link (7 links per GPU).  A ring collective
(RCCL all_gather / reduce_scatter) moves each block through g-1 hops and drives one link per
direction at a time; here every rank posts one send and one receive per group peer in a single
RCCL group call (``batch_isend_irecv``), so the g-1 blocks a rank needs arrive at once, each on
the link that joins the two GPUs, and nothing is forwarded.

  all_gather(h_loc, full)     full[p-block] = h_loc of peer p (the own block is not copied
                              unless asked: the remote-column CSR never reads it)
  reduce_scatter(partial)     owner's rows of sum_p partial_p: peer blocks sent raw, summed on
                              the owner in peer order (deterministic, no RCCL reduction kernel)

Both take the KG group, its global ranks and this rank's index; gloo (the CPU rehearsal and the
tests) runs the same point-to-point schedule on host tensors, staging device tensors through
host memory.  GNNEA_HALO=ring selects the RCCL ring collectives instead (comparison only).

Relay (two KG groups of g): the group's exchange alone loads the g-1 links inside the group
while the g links to the other group's GPUs sit idle.  ``all_gather`` given the other group's
ranks (``other``) cuts a rank's block into 2g units of rows: D1 (1 unit) and D2 (g-1 units) go
direct to every group peer in phases 1 and 2; R_k (1 unit each, k < g) goes in phase 1 to the
other group's k-th GPU, which forwards it in phase 2 to every one of this rank's group peers
(the payload is the same for all of them, so each relayed byte crosses one first hop) while
this rank forwards the other group's parts the same way.  Per direction every in-group link
carries 1 unit in phase 1 and g-1 in phase 2, every cross-group link 1 unit in phase 1 and g-1
in phase 2: g units in all instead of 2g, half the direct time at any g.  Both phases are
world-group RCCL group calls issued back to back on the same communicator (stream-ordered: a
phase-1 receive completes before the phase-2 send that forwards it); every rank of both groups
must call it at the same point.  The reduce-scatter relays too (``_relay_rs``: its payloads
differ per destination, so the split is g-1 / g-1 / 1.. units of 3g-2: 0.5 of the direct time at
g = 2, 0.6 at g = 4); GNNEA_HALO=p2p keeps the direct schedule.
"""
import os

import torch
import torch.distributed as dist

MODE = os.environ.get("GNNEA_HALO", "relay")
# The per-column-slice pipeline (all_gather_slices / reduce_scatter_start: several RCCL group
# calls in flight, each slice aggregated as soon as it has landed) against the unstaged path (the
# whole halo row-major, then one aggregation, and one blocking reduce-scatter back).  Both are
# exercised with gloo at world 2 / 4 / 8 and rehearsed on one MI355X (host-staged); RCCL refuses
# two ranks on one device ("Duplicate GPU detected"), so the staged path's asynchronous RCCL
# behaviour is proven on the job's own ranks: gnnea.dist_graph.validate_staged runs a HighWay,
# a GCN and a GAT layer both ways on the same inputs, and switches STAGED on only when every
# rank saw the two agree.  GNNEA_HALO_STAGED: "auto" (default: unstaged until validated; then
# staged for exactly the storage dtypes whose legs matched), "1" (staged for every dtype without
# validation: validate_staged reports but changes nothing), "0" (never staged, validate_staged
# reports but keeps it off).
STAGED_ENV = os.environ.get("GNNEA_HALO_STAGED", "auto")
STAGED = STAGED_ENV == "1"
# None: STAGED applies to every storage dtype (GNNEA_HALO_STAGED=1, tests); else the set of
# dtypes validate_staged saw match on this job's ranks
STAGED_DTYPES = None


def staged_for(dtype):
    """Whether the per-slice pipeline carries a halo of this storage dtype."""
    return STAGED and (STAGED_DTYPES is None or dtype in STAGED_DTYPES)


def _gloo(group):
    return dist.get_backend(group) == "gloo"


def _blocks(t, g):
    rows = t.shape[0] // g
    return [t[p * rows:(p + 1) * rows] for p in range(g)]


def relay_applies(ranks, other):
    return MODE == "relay" and other is not None and len(ranks) == len(other) >= 2


def _units(rows, g, d1=1, d2=None):
    """Row ranges of D1, D2, R_0..R_{g-1}: d1, d2 (default g-1) and 1 each of near-equal units
    (all-gather: 1, g-1, 1.. of 2g; reduce-scatter: g-1, g-1, 1.. of 3g-2)."""
    d2 = g - 1 if d2 is None else d2
    n = d1 + d2 + g
    cut = [rows * j // n for j in range(n + 1)]
    e = d1 + d2
    return [(cut[0], cut[d1]), (cut[d1], cut[e])] + [(cut[e + k], cut[e + k + 1]) for k in range(g)]


def _relay_rs(blocks, recv, ranks, li, other, sync=True):
    """Relayed exchange of a reduce-scatter over two groups of g: ``blocks[i]`` (this rank's
    partial of group rank i's rows) goes to rank i, its D1 / D2 (g-1 units each) direct in
    phases 1 / 2 and its R_k (1 unit of 3g-2) through the other group's k-th GPU; ``recv[p]``
    receives peer p's partial of this rank's rows.  Per direction every link carries g-1 units
    per phase: 2(g-1) of 3g-2 against the whole block direct (0.5 at g = 2, 0.6 at g = 4)."""
    me = ranks[li]
    mine, theirs = sorted(ranks), sorted(other)
    g = len(mine)
    u = _units(blocks[li].shape[0], g, g - 1, g - 1)
    peers = [p for p in mine if p != me]

    def rows(t, j):
        return t[u[j][0]:u[j][1]]

    def blk(p):
        return blocks[ranks.index(p)]

    ki = mine.index(me)
    # stage[(s, dst)]: other-group source s's partial for dst, unit R_ki (this rank relays it)
    stage = {(s, d): torch.empty_like(rows(blocks[li], 2 + ki))
             for s in theirs for d in theirs if d != s}
    ops1 = []
    for p in peers:
        ops1.append(dist.P2POp(dist.isend, rows(blk(p), 0), p))
        ops1.append(dist.P2POp(dist.irecv, rows(recv[p], 0), p))
    for k, o in enumerate(theirs):
        for d in peers:
            ops1.append(dist.P2POp(dist.isend, rows(blk(d), 2 + k), o))
    for s_ in theirs:
        for d in theirs:
            if d != s_:
                ops1.append(dist.P2POp(dist.irecv, stage[(s_, d)], s_))
    w1 = dist.batch_isend_irecv(ops1)
    if sync:
        for w in w1:
            w.wait()
    ops2 = []
    for p in peers:
        ops2.append(dist.P2POp(dist.isend, rows(blk(p), 1), p))
        ops2.append(dist.P2POp(dist.irecv, rows(recv[p], 1), p))
    for d in theirs:
        for s_ in theirs:
            if s_ != d:
                ops2.append(dist.P2POp(dist.isend, stage[(s_, d)], d))
    for k, o in enumerate(theirs):
        for p in peers:
            ops2.append(dist.P2POp(dist.irecv, rows(recv[p], 2 + k), o))
    w2 = dist.batch_isend_irecv(ops2)
    if sync:
        for w in w2:
            w.wait()
        return []
    return w1 + w2 + [_Keep(stage)]


def _relay(h_loc, full_parts, ranks, li, other, sync):
    """Two-phase relayed all-gather over two groups of g (module docstring).  ``full_parts``:
    the g blocks of ``full`` (this rank's is not written).  Global ranks throughout."""
    me = ranks[li]
    mine, theirs = sorted(ranks), sorted(other)
    g = len(mine)
    u = _units(h_loc.shape[0], g)
    peers = [p for p in mine if p != me]
    blk = {p: full_parts[ranks.index(p)] for p in peers}

    def rows(t, j):
        return t[u[j][0]:u[j][1]]

    # phase 1: D1 to every group peer; R_k to the other group's k-th GPU; receive the other
    # group's parts this rank forwards (source s sends R_{index of me among my group})
    ki = mine.index(me)
    stage = {s: torch.empty_like(rows(h_loc, 2 + ki)) for s in theirs}
    ops1 = []
    for p in peers:
        ops1.append(dist.P2POp(dist.isend, rows(h_loc, 0), p))
        ops1.append(dist.P2POp(dist.irecv, rows(blk[p], 0), p))
    for k, o in enumerate(theirs):
        ops1.append(dist.P2POp(dist.isend, rows(h_loc, 2 + k), o))
        ops1.append(dist.P2POp(dist.irecv, stage[o], o))
    w1 = dist.batch_isend_irecv(ops1)
    if sync:
        for w in w1:
            w.wait()
    # phase 2: D2 to every group peer; forward each staged part to every other-group GPU but
    # its source (destinations ascending, sources ascending); receive from the other group's
    # k-th GPU the R_k of every group peer (same order)
    ops2 = []
    for p in peers:
        ops2.append(dist.P2POp(dist.isend, rows(h_loc, 1), p))
        ops2.append(dist.P2POp(dist.irecv, rows(blk[p], 1), p))
    for dst in theirs:
        for s in theirs:
            if s != dst:
                ops2.append(dist.P2POp(dist.isend, stage[s], dst))
    for k, o in enumerate(theirs):
        for p in peers:
            ops2.append(dist.P2POp(dist.irecv, rows(blk[p], 2 + k), o))
    w2 = dist.batch_isend_irecv(ops2)
    if sync:
        for w in w2:
            w.wait()
        return []
    return w1 + w2 + [_Keep(stage)]


class _Keep:
    """Holds the relay's staging buffers until the caller has waited on the exchange."""

    def __init__(self, bufs):
        self.bufs = bufs

    def wait(self):
        self.bufs = None


def all_gather(h_loc, full, group, ranks, li, copy_own=False, async_op=False, other=None):
    """Assemble the group's rows in ``full`` ([g·rows, D], contiguous).  Returns the works to
    wait on (an empty list when done synchronously).  ``other``: the other KG group's ranks;
    with two KG groups the relayed schedule is taken (every rank must pass it then)."""
    g = len(ranks)
    h_loc = h_loc.contiguous()
    parts = _blocks(full, g)
    if copy_own:
        parts[li].copy_(h_loc)
    if g == 1:
        return []
    if relay_applies(ranks, other):
        if _gloo(group) and h_loc.is_cuda:  # host-staged rehearsal
            hb = [torch.empty(pp.shape, dtype=pp.dtype) for pp in parts]
            _relay(h_loc.detach().cpu(), hb, ranks, li, other, True)
            for p in range(g):
                if p != li:
                    parts[p].copy_(hb[p])
            return []
        return _relay(h_loc, parts, ranks, li, other, _gloo(group) or not async_op)
    if _gloo(group):
        src = h_loc.detach().cpu() if h_loc.is_cuda else h_loc
        bufs = [torch.empty_like(src) if full.is_cuda else parts[p] for p in range(g)]
        ops = []
        for p in range(g):
            if p != li:
                ops.append(dist.P2POp(dist.isend, src, ranks[p], group=group))
                ops.append(dist.P2POp(dist.irecv, bufs[p], ranks[p], group=group))
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        if full.is_cuda:
            for p in range(g):
                if p != li:
                    parts[p].copy_(bufs[p])
        return []
    if MODE == "ring":
        w = dist.all_gather_into_tensor(full, h_loc, group=group, async_op=async_op)
        return [w] if async_op else []
    ops = []
    for p in range(g):
        if p != li:
            ops.append(dist.P2POp(dist.isend, h_loc, ranks[p], group=group))
            ops.append(dist.P2POp(dist.irecv, parts[p], ranks[p], group=group))
    works = dist.batch_isend_irecv(ops)
    if not async_op:
        for w in works:
            w.wait()
        return []
    return works


class PendingSum:
    """An issued reduce-scatter: ``finish()`` waits for the receives (stream-ordered on the
    caller's stream for RCCL) and returns the owner's rows: its own partial plus the peers'
    partials in peer order (deterministic, no RCCL reduction kernel) for the relay and direct
    schedules.  Under GNNEA_HALO=ring ``own`` is already RCCL's reduce_scatter result, whose
    summation order is RCCL's (not order-deterministic across ring configurations)."""

    def __init__(self, own, recv, works, out=None):
        self.own, self.recv, self.works, self.out = own, recv, works, out

    def finish(self):
        for w in self.works:
            w.wait()
        out = _owner_sum(self.own, self.recv, self.out)
        self.own = self.recv = self.works = None
        return out


def _owner_sum(own, recv, out=None):
    """own + recv[0] + recv[1] + ... in that order.  Low-precision partials (bf16 storage) are
    summed in fp32 and rounded once into ``out`` (a bf16 running sum would round at every peer)."""
    if own.dtype in (torch.bfloat16, torch.float16) and recv:
        acc = own.float()
        for r in recv:
            acc += r.to(device=acc.device, dtype=torch.float32)
        if out is None:
            return acc.to(own.dtype)
        out.copy_(acc)
        return out
    if out is None:
        out = own.clone()
    else:
        out.copy_(own)
    for r in recv:
        out += r.to(out.device) if r.device != out.device else r
    return out


def reduce_scatter_start(partial, group, ranks, li, other=None, out=None):
    """Issue the reduce-scatter of ``partial`` ([g·rows, w], this rank's partial of every group
    row) without waiting: returns a PendingSum whose finish() gives this rank's rows (into
    ``out`` when given, e.g. a column block of a wider buffer).  Several can be in flight at once
    (the per-slice pipeline of gnnea.dist_graph); under gloo the exchange completes here."""
    g = len(ranks)
    partial = partial.contiguous()
    if g == 1:
        return PendingSum(partial, [], [], out)
    blocks = _blocks(partial, g)
    stage = _gloo(group) and partial.is_cuda
    send = [b.detach().cpu() if stage else b for b in blocks]
    if relay_applies(ranks, other):
        recv = {p: torch.empty_like(send[li]) for p in ranks if p != ranks[li]}
        works = _relay_rs(send, recv, ranks, li, other, sync=_gloo(group))
        return PendingSum(blocks[li], [recv[p] for p in ranks if p != ranks[li]], works, out)
    if not _gloo(group) and MODE == "ring":  # RCCL's reduce-scatter, as reduce_scatter does
        red = torch.empty_like(blocks[li])
        w = dist.reduce_scatter_tensor(red, partial, group=group, async_op=True)
        return PendingSum(red, [], [w], out)
    recv = [torch.empty_like(send[li]) for p in range(g) if p != li]
    ops = []
    k = 0
    for p in range(g):
        if p != li:
            ops.append(dist.P2POp(dist.isend, send[p], ranks[p], group=group))
            ops.append(dist.P2POp(dist.irecv, recv[k], ranks[p], group=group))
            k += 1
    works = dist.batch_isend_irecv(ops)
    if _gloo(group):
        for w in works:
            w.wait()
        works = []
    return PendingSum(blocks[li], recv, works, out)


def all_gather_slices(tables, row0, rows, group, ranks, li, other=None):
    """The halo exchange cut into column slices (SURVEY.md §8e overlap): ``tables`` are the
    KG group's feature tables, one contiguous [g·rows, w] table per column slice, this rank's
    rows [row0, row0 + rows) already in place.  Every slice's exchange is issued at once (in
    slice order on the communicator); returns one list of works per slice, so the caller can
    aggregate slice q as soon as its works are done while the later slices are in flight."""
    return [all_gather(t[row0:row0 + rows], t, group, ranks, li, copy_own=False, async_op=True,
                       other=other) for t in tables]


def reduce_scatter(partial, group, ranks, li, other=None):
    """This rank's rows of the group sum of the [g·rows, D] partials.  ``other`` as in
    all_gather: the relayed schedule (``_relay_rs``) when given."""
    g = len(ranks)
    partial = partial.contiguous()
    if g == 1:
        return partial
    blocks = _blocks(partial, g)
    if relay_applies(ranks, other):
        stage = _gloo(group) and partial.is_cuda
        send = [b.detach().cpu() if stage else b for b in blocks]
        recv = {p: torch.empty_like(send[li]) for p in ranks if p != ranks[li]}
        _relay_rs(send, recv, ranks, li, other, sync=True)
        # peer order, as the direct schedule sums
        return _owner_sum(blocks[li], [recv[p] for p in ranks if p != ranks[li]])
    if not _gloo(group) and MODE == "ring":
        out = torch.empty_like(blocks[li])
        dist.reduce_scatter_tensor(out, partial, group=group)
        return out
    stage = _gloo(group) and partial.is_cuda
    send = [b.detach().cpu() if stage else b for b in blocks]
    recv = [torch.empty_like(send[li]) if p != li else None for p in range(g)]
    ops = []
    for p in range(g):
        if p != li:
            ops.append(dist.P2POp(dist.isend, send[p], ranks[p], group=group))
            ops.append(dist.P2POp(dist.irecv, recv[p], ranks[p], group=group))
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    return _owner_sum(blocks[li], [recv[p] for p in range(g) if p != li])
