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
"""
import os

import torch
import torch.distributed as dist

MODE = os.environ.get("GNNEA_HALO", "p2p")


def _gloo(group):
    return dist.get_backend(group) == "gloo"


def _blocks(t, g):
    rows = t.shape[0] // g
    return [t[p * rows:(p + 1) * rows] for p in range(g)]


def all_gather(h_loc, full, group, ranks, li, copy_own=False, async_op=False):
    """Assemble the group's rows in ``full`` ([g·rows, D], contiguous).  Returns the works to
    wait on (an empty list when done synchronously)."""
    g = len(ranks)
    h_loc = h_loc.contiguous()
    parts = _blocks(full, g)
    if copy_own:
        parts[li].copy_(h_loc)
    if g == 1:
        return []
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


def reduce_scatter(partial, group, ranks, li):
    """This rank's rows of the group sum of the [g·rows, D] partials."""
    g = len(ranks)
    partial = partial.contiguous()
    if g == 1:
        return partial
    blocks = _blocks(partial, g)
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
