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

Relay (4 GPUs, two KG groups of 2): the group's exchange alone would load ONE link per direction
(the pair's), while the links to the other group's two GPUs sit idle.  ``all_gather`` given the
other group's ranks (``other``) splits the block into quarters: q0 goes direct in phase 1, q1
direct in phase 2, q2 / q3 go in phase 1 to the other group's GPUs, which forward them to the
partner in phase 2 while this rank forwards theirs.  Every link carries one quarter per
direction per phase, so the exchange takes two quarter-transfers instead of one whole-block
transfer (half the time).  Both phases are world-group RCCL group calls issued back to back on
the same communicator (stream-ordered: a phase-1 receive completes before the phase-2 send that
forwards it); every rank of both groups must call it at the same point.  GNNEA_HALO=p2p keeps
the direct schedule.
"""
import os

import torch
import torch.distributed as dist

MODE = os.environ.get("GNNEA_HALO", "relay")


def _gloo(group):
    return dist.get_backend(group) == "gloo"


def _blocks(t, g):
    rows = t.shape[0] // g
    return [t[p * rows:(p + 1) * rows] for p in range(g)]


def relay_applies(ranks, other):
    return MODE == "relay" and other is not None and len(ranks) == 2 and len(other) == 2


def _quarters(rows):
    """Row ranges [q0, q1, q2, q3) of a block of ``rows`` rows (near-equal quarters)."""
    cut = [rows * k // 4 for k in range(5)]
    return [(cut[k], cut[k + 1]) for k in range(4)]


def _relay(h_loc, part_full, ranks, li, other, sync):
    """Two-phase relayed exchange of a 2-rank group (module docstring).  ``part_full``: the
    partner's block of ``full``.  Global ranks throughout (world group)."""
    me, partner = ranks[li], ranks[1 - li]
    q = _quarters(h_loc.shape[0])

    def rows(t, k):
        return t[q[k][0]:q[k][1]]

    # phase 1: q0 direct; q2 / q3 to the other group's GPUs (sorted); receive the other
    # group's quarters this rank forwards (source s sends quarter 2 + index of me in the
    # sorted ranks of this group)
    mine = sorted(ranks)
    stage = {s: torch.empty_like(rows(h_loc, 2 + mine.index(me))) for s in other}
    ops1 = [dist.P2POp(dist.isend, rows(h_loc, 0), partner),
            dist.P2POp(dist.irecv, rows(part_full, 0), partner)]
    for k, o in enumerate(sorted(other)):
        ops1.append(dist.P2POp(dist.isend, rows(h_loc, 2 + k), o))
    for s in other:
        ops1.append(dist.P2POp(dist.irecv, stage[s], s))
    w1 = dist.batch_isend_irecv(ops1)
    if sync:
        for w in w1:
            w.wait()
    # phase 2: q1 direct; forward each staged quarter to its source's partner; receive the
    # partner's q2 / q3 from the relays
    ops2 = [dist.P2POp(dist.isend, rows(h_loc, 1), partner),
            dist.P2POp(dist.irecv, rows(part_full, 1), partner)]
    for s in other:
        dst = [r for r in other if r != s][0]
        ops2.append(dist.P2POp(dist.isend, stage[s], dst))
    for k, o in enumerate(sorted(other)):
        ops2.append(dist.P2POp(dist.irecv, rows(part_full, 2 + k), o))
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
    with two groups of two the relayed schedule is taken (every rank must pass it then)."""
    g = len(ranks)
    h_loc = h_loc.contiguous()
    parts = _blocks(full, g)
    if copy_own:
        parts[li].copy_(h_loc)
    if g == 1:
        return []
    if relay_applies(ranks, other):
        pf = parts[1 - li]
        if _gloo(group) and h_loc.is_cuda:  # host-staged rehearsal
            hb = torch.empty(pf.shape, dtype=pf.dtype)
            _relay(h_loc.detach().cpu(), hb, ranks, li, other, True)
            pf.copy_(hb)
            return []
        return _relay(h_loc, pf, ranks, li, other, _gloo(group) or not async_op)
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


def reduce_scatter(partial, group, ranks, li, other=None):
    """This rank's rows of the group sum of the [g·rows, D] partials.  ``other`` as in
    all_gather: with two groups of two the partner's block travels by the relayed schedule."""
    g = len(ranks)
    partial = partial.contiguous()
    if g == 1:
        return partial
    blocks = _blocks(partial, g)
    if relay_applies(ranks, other):
        # one block each way between the partners: the relay with the partner's block as the
        # payload; the owner adds it to its own (the order of the direct schedule's sum)
        stage = _gloo(group) and partial.is_cuda
        send = blocks[1 - li].detach().cpu() if stage else blocks[1 - li]
        recv = torch.empty_like(send)
        _relay(send, recv, ranks, li, other, True)
        return blocks[li] + (recv.to(partial.device) if stage else recv)
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
    out = blocks[li].clone()
    for p in range(g):
        if p != li:
            out += recv[p].to(out.device) if stage else recv[p]
    return out
