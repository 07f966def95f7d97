"""Node sharding of the two-KG graph across the GPUs of one node.

Layout (one process per GPU, torch.distributed; backend "nccl" is RCCL over xGMI):
  * the adjacency is block-diagonal over the two KGs (no cross-KG entries), so ranks
    [0, W/2) serve KG1 and [W/2, W) serve KG2 — no traffic between the two groups;
  * inside a KG group of g = W/2 ranks each rank owns a contiguous block of n/g destination
    rows; its CSR keeps KG-local column ids;
  * per aggregation the group all-gathers the projected rows (the halo: on uniform random graphs
    nearly every remote row is referenced) with RCCL, then every rank runs the CSR SpMM on its
    rows.  W = 1 keeps the whole graph on one GPU; W = 2 is one KG per GPU with no exchange.
The partition / exchange logic is device-independent (numpy + torch.distributed) and is
exercised with gloo on CPU in tests/test_dist_gloo.py; the GPU path adds only the CSR upload.
"""
import numpy as np
import torch
import torch.distributed as dist

from . import synth


class Partition:
    """Which rows / columns of the two-KG adjacency rank `rank` of `world` owns."""

    def __init__(self, n, rank, world):
        self.n, self.rank, self.world = n, rank, world
        if world == 1:
            self.kg, self.g, self.li = None, 1, 0
            self.n_cols = 2 * n
            self.row0, self.row1 = 0, 2 * n
            self.global_row0 = 0
        else:
            if world % 2:
                raise ValueError("gnnea.dist: world size must be 1 or even (two KG groups)")
            self.g = world // 2
            if n % self.g:
                raise ValueError("gnnea.dist: entities per KG must divide by the group size")
            self.kg = rank // self.g
            self.li = rank % self.g
            self.n_cols = n
            rows = n // self.g
            self.row0, self.row1 = self.li * rows, (self.li + 1) * rows
            self.global_row0 = self.kg * n + self.row0

    @property
    def n_rows(self):
        return self.row1 - self.row0

    def group_ranks(self, kg):
        return list(range(kg * self.g, (kg + 1) * self.g))


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


def halo_gather(h_local, h_full, group, group_size):
    """All-gather the group's projected rows into h_full [group_size * rows, D]."""
    if group_size == 1:
        return h_local
    if dist.get_backend(group) == "gloo":  # CPU rehearsal path
        parts = list(h_full.chunk(group_size, dim=0))
        dist.all_gather(parts, h_local.contiguous(), group=group)
        return h_full
    dist.all_gather_into_tensor(h_full, h_local, group=group)
    return h_full


class KGShard:
    """A rank's device-resident CSR shard of the synthetic cfg graph."""

    def __init__(self, n, t, n_rel, rank, world, device, seed=0):
        from .graph import DeviceCSR
        self.part = Partition(n, rank, world)
        self.n, self.device = n, device
        triples = synth.kg_pair_triples(n, t, n_rel, seed=seed)
        r, c, v = shard_coo(triples, n, t, self.part)
        self.csr = DeviceCSR.from_coo(torch.from_numpy(r.astype(np.int32)).to(device),
                                      torch.from_numpy(c.astype(np.int32)).to(device),
                                      torch.from_numpy(v).to(device), self.part.n_rows,
                                      self.part.n_cols)
        self.nnz = self.csr.nnz
        self.group = make_groups(self.part)

    @property
    def g(self):
        return self.part.g

    @property
    def n_rows(self):
        return self.part.n_rows

    @property
    def n_cols(self):
        return self.part.n_cols

    def gather_halo(self, h_local, h_full):
        return halo_gather(h_local, h_full, self.group, self.part.g)
