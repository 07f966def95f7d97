"""Sharding of the two-KG graph across the GPUs of one node.

Layout (one process per GPU, torch.distributed; backend "nccl" is RCCL over xGMI):
  * the adjacency is block-diagonal over the two KGs (no cross-KG entries), so ranks
    [0, W/2) serve KG1 and [W/2, W) serve KG2 — no traffic between the two groups
    (W = 1 keeps the whole graph on one GPU; W = 2 is one KG per GPU, nothing to exchange);
  * inside a KG group of g = W/2 ranks, three partitions are implemented:
    - "features": every rank holds the whole KG adjacency and a 16-B-aligned slice
      of the feature columns (300 = 76+76+76+72 at g = 4).  relu(A·H) is column-separable,
      so the aggregation needs NO exchange; in a full layer the group exchange moves to the
      projection input (all-gather of the previous layer's column slices, same volume);
    - "tiles": g = gr x gc ranks, gc = 2 column slices (>= 148 columns: slice-major tables)
      times gr = g/2 blocks of destination rows; every rank gathers from the whole KG's column
      slice, so again NO exchange (8 GPUs: 2 x 2 tiles of 500k rows x 150 columns instead of
      four 76-column slices of all rows);
    - "rows": each rank owns n/g destination rows (KG-local column ids) and gathers the
      group's projected rows (the halo: on uniform random graphs nearly every remote row is
      referenced) by peer transfers over xGMI (gnnea.exchange), slice by slice: the KG's
      table is held slice-major ([S][n][64] fp32, one Infinity-Cache-sized table per slice),
      every slice's exchange is issued at once and slice q is aggregated over the shard's CSR
      as soon as it has landed, while the later slices move (SURVEY.md §8e overlap).  This is
      what a graph layer executes (gnnea.dist_graph), so it is the bench default at N > 1;
      the two exchange-free partitions time the aggregation alone.
The partition / exchange logic is device-independent (numpy + torch.distributed) and is
exercised with gloo on CPU in tests/test_dist_gloo.py; the GPU path adds only the CSR upload.
"""
import numpy as np
import torch
import torch.distributed as dist

from . import synth


def feature_slices(D, g):
    """g contiguous slices of D columns, each a multiple of 4 wide (16-B rows) but the last."""
    base = (D // g + 3) // 4 * 4
    cuts = [min(D, k * base) for k in range(g)] + [D]
    return [(cuts[k], cuts[k + 1]) for k in range(g)]


class Partition:
    """Which rows / columns of the two-KG adjacency rank `rank` of `world` owns."""

    def __init__(self, n, rank, world, kind="rows", D=300):
        self.n, self.rank, self.world, self.kind = n, rank, world, kind
        self.col0, self.col1 = 0, D
        if world == 1:
            self.kg, self.g, self.li = None, 1, 0
            self.gr = self.gc = 1
            self.n_cols = 2 * n
            self.row0, self.row1 = 0, 2 * n
            self.global_row0 = 0
        else:
            if world % 2:
                raise ValueError("gnnea.dist: world size must be 1 or even (two KG groups)")
            self.g = world // 2
            if kind not in ("rows", "features", "tiles"):
                raise ValueError("gnnea.dist: partition must be 'rows', 'features' or 'tiles'")
            # tiles: gr row blocks x gc column slices, gc = 2 when the group is even (slices
            # of >= 148 columns keep the slice-major tables; 76-column slices do not)
            self.gc = (2 if self.g % 2 == 0 else 1) if kind == "tiles" else \
                (self.g if kind == "features" else 1)
            self.gr = self.g // self.gc
            if n % self.gr:
                raise ValueError("gnnea.dist: entities per KG must divide by the row blocks")
            self.kg = rank // self.g
            self.li = rank % self.g
            self.n_cols = n
            ri, ci = self.li // self.gc, self.li % self.gc
            rows = n // self.gr
            self.row0, self.row1 = ri * rows, (ri + 1) * rows
            if kind != "rows":
                self.col0, self.col1 = feature_slices(D, self.gc)[ci]
            self.global_row0 = self.kg * n + self.row0

    @property
    def n_rows(self):
        return self.row1 - self.row0

    def col0_col1(self):
        return self.col0, self.col1

    def group_ranks(self, kg):
        return list(range(kg * self.g, (kg + 1) * self.g))

    def other_ranks(self):
        """The other KG group's ranks (relay hops of gnnea.exchange), None on one GPU."""
        return None if self.kg is None else self.group_ranks(1 - self.kg)


def shard_coo(triples, n, t, part):
    """Local COO (rows relative to the shard, KG-local columns), sorted by (row, col)."""
    if part.kg is not None:
        tr = triples[part.kg * t:(part.kg + 1) * t].copy()
        tr[:, 0] -= part.kg * n
        tr[:, 2] -= part.kg * n
        r, c, v = synth.adjacency_coo(tr, n, reference_order=False)
    else:
        r, c, v = synth.adjacency_coo(triples, 2 * n, reference_order=False)
    keep = (r >= part.row0) & (r < part.row1)
    return r[keep] - part.row0, c[keep], v[keep]


def make_groups(part):
    """Both KG groups (every rank must create every group, in the same order)."""
    if part.world == 1:
        return None
    groups = [dist.new_group(part.group_ranks(k)) for k in range(2)]
    return groups[part.kg]


def halo_gather(h_local, h_full, group, group_size, async_op=False, part=None):
    """Assemble the group's projected rows in h_full [group_size * rows, D].

    Direct peer transfers (gnnea.exchange.all_gather: one send and one receive per group peer
    in one RCCL group call, each pair on its own xGMI link; async_op=True returns the works so
    the caller can overlap the locally owned part of the aggregation).  ``part`` gives the
    group's ranks and this rank's index; without it the group is taken as consecutive ranks.
    The own block is copied too (callers that read only remote blocks use exchange directly).
    gloo (CPU rehearsal of the multi-rank logic): synchronous, staged through host memory when
    the tensors live on a device."""
    from . import exchange
    if group_size == 1:
        return None
    if part is not None:
        ranks, li = part.group_ranks(part.kg), part.li
    else:
        me = dist.get_rank()
        base = me - me % group_size
        ranks, li = list(range(base, base + group_size)), me % group_size
    works = exchange.all_gather(h_local, h_full, group, ranks, li, copy_own=True,
                                async_op=async_op,
                                other=part.other_ranks() if part is not None else None)
    return _Works(works) if works else None


class _Works:
    def __init__(self, works):
        self.works = works

    def wait(self):
        for w in self.works:
            w.wait()


class KGShard:
    """A rank's device-resident CSR shard of the synthetic cfg graph."""

    def __init__(self, n, t, n_rel, rank, world, device, seed=0, kind="rows", D=300):
        from .graph import DeviceCSR
        self.part = Partition(n, rank, world, kind, D)
        self.n, self.device = n, device
        triples = synth.kg_pair_triples(n, t, n_rel, seed=seed)
        r, c, v = shard_coo(triples, n, t, self.part)
        self.nnz = int(r.size)

        def up(rr, cc, vv, ncols):
            return DeviceCSR.from_coo(torch.from_numpy(rr.astype(np.int32)).to(device),
                                      torch.from_numpy(cc.astype(np.int32)).to(device),
                                      torch.from_numpy(vv).to(device), self.part.n_rows, ncols)
        self.csr = up(r, c, v, self.part.n_cols)
        self.group = make_groups(self.part) if kind == "rows" else None
        self._tables = self._full = None

    @property
    def g(self):
        return self.part.g

    @property
    def n_rows(self):
        return self.part.n_rows

    @property
    def n_cols(self):
        return self.part.n_cols

    def halo_tables(self, D, dtype=torch.float32):
        """The KG's slice tables [S][n][W] (own rows packed in by aggregate), allocated once."""
        from . import ops
        W = ops.slice_w(dtype)
        S = (D + W - 1) // W
        t = self._tables
        if t is None or t.shape != (S, self.n_cols, W) or t.dtype != dtype:
            t = self._tables = torch.empty((S, self.n_cols, W), dtype=dtype, device=self.device)
        return t

    def slices(self, D, dtype=torch.float32):
        from . import ops
        W = ops.slice_w(dtype)
        return [(c0, min(D, c0 + W)) for c0 in range(0, D, W)]

    def aggregate(self, h_local, out, act, events=None, hs=None):
        """out = act(A_shard · H) for this rank's rows.  Row shards of a KG group: the own rows
        packed into the KG's slice tables, every slice's halo exchange issued at once, slice q
        aggregated as soon as it has landed (``events``: [start, end] + a pair per slice around
        its aggregation); with GNNEA_HALO_STAGED=0 the whole halo first, then one aggregation
        (one event pair around it).  ``hs``: H held slice-major (gnnea.ops.spmm_sliced) for the
        exchange-free partitions."""
        from . import exchange, ops
        rec = (lambda k: events[k].record()) if events is not None else (lambda k: None)
        if self.part.g == 1 or self.part.kind in ("features", "tiles"):  # no exchange
            rec(0)
            if hs is not None:
                ops.spmm_sliced(self.csr, hs, h_local.shape[1], act, out=out)
            else:
                ops.spmm(self.csr, h_local, act, out=out)
            rec(1)
            return out
        D = h_local.shape[1]
        if not exchange.staged_for(h_local.dtype):  # the whole halo row-major, then aggregate
            rec(0)
            full = self._full
            if full is None or full.shape != (self.n_cols, D) or full.dtype != h_local.dtype:
                full = self._full = torch.empty((self.n_cols, D), dtype=h_local.dtype,
                                                device=self.device)
            exchange.all_gather(h_local, full, self.group, self.part.group_ranks(self.part.kg),
                                self.part.li, copy_own=True, other=self.part.other_ranks())
            rec(2)
            if ops.use_sliced(self.n_cols, D, h_local.dtype):
                ops.spmm_sliced(self.csr, ops.slice_pack(full), D, act, out=out)
            else:
                ops.spmm(self.csr, full, act, out=out)
            rec(3)
            rec(1)
            return out
        tables = self.halo_tables(D, h_local.dtype)
        rec(0)
        with torch.cuda.device(self.device):
            ops.check(ops._sfn("gnnea_slice_pack", h_local.dtype)(
                ops.ptr(h_local), ops._ld(h_local), self.n_rows, D,
                ops._off(tables[0], self.part.row0), tables.stride(0),
                ops.stream_of(self.device)))
        works = exchange.all_gather_slices(list(tables), self.part.row0, self.n_rows, self.group,
                                           self.part.group_ranks(self.part.kg), self.part.li,
                                           other=self.part.other_ranks())
        for q, (c0, c1) in enumerate(self.slices(D, h_local.dtype)):
            for w in works[q]:
                w.wait()
            rec(2 + 2 * q)
            ops.spmm_sliced(self.csr, tables[q:q + 1], c1 - c0, act, out=out[:, c0:c1])
            rec(3 + 2 * q)
        rec(1)
        return out
