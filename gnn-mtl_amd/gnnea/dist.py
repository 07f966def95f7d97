"""Node sharding of the two-KG graph across the GPUs of one node.

Layout (one process per GPU, torch.distributed over RCCL):
  * the adjacency is block-diagonal over the two KGs (no cross-KG entries), so ranks
    [0, W/2) serve KG1 and [W/2, W) serve KG2 — no traffic between the two groups;
  * inside a KG group of g = W/2 ranks each rank owns a contiguous block of n/g destination
    rows (its CSR keeps KG-local column ids);
  * per aggregation the group all-gathers the projected rows (the halo: on uniform random graphs
    nearly every remote row is referenced) with RCCL over xGMI, then every rank runs the CSR
    SpMM on its rows.  W = 1 keeps the whole graph on one GPU; W = 2 is one KG per GPU with no
    exchange at all.
"""
import numpy as np
import torch
import torch.distributed as dist

from . import synth
from .graph import DeviceCSR


class KGShard:
    def __init__(self, n, t, n_rel, rank, world, device, seed=0):
        self.rank, self.world, self.device = rank, world, device
        self.n = n
        if world == 1:
            self.kg, self.g, self.li = None, 1, 0
            self.n_cols = 2 * n
            self.row0, self.row1 = 0, 2 * n
        else:
            if world % 2:
                raise ValueError("gnnea.dist: world size must be 1 or even (two KG groups)")
            self.g = world // 2
            if n % self.g:
                raise ValueError("gnnea.dist: n must be divisible by the group size")
            self.kg = rank // self.g
            self.li = rank % self.g
            self.n_cols = n
            rows = n // self.g
            self.row0, self.row1 = self.li * rows, (self.li + 1) * rows
        triples = synth.kg_pair_triples(n, t, n_rel, seed=seed)
        if self.kg is not None:
            tr = triples[self.kg * t:(self.kg + 1) * t].copy()
            tr[:, 0] -= self.kg * n
            tr[:, 2] -= self.kg * n
            r, c, v = synth.adjacency_coo(tr, n, reference_order=False)
        else:
            r, c, v = synth.adjacency_coo(triples, 2 * n, reference_order=False)
        keep = (r >= self.row0) & (r < self.row1)
        r, c, v = r[keep] - self.row0, c[keep], v[keep]
        self.csr = DeviceCSR.from_coo(torch.from_numpy(r.astype(np.int32)).to(device),
                                      torch.from_numpy(c.astype(np.int32)).to(device),
                                      torch.from_numpy(v).to(device), self.row1 - self.row0,
                                      self.n_cols)
        self.nnz = self.csr.nnz
        self.group = None
        if world > 1:
            groups = [dist.new_group(list(range(k * self.g, (k + 1) * self.g))) for k in range(2)]
            self.group = groups[self.kg]

    @property
    def n_rows(self):
        return self.row1 - self.row0

    def gather_halo(self, h_local, h_full):
        """All-gather the group's projected rows (RCCL) into h_full [n_cols, D]."""
        if self.g == 1:
            return h_local
        dist.all_gather_into_tensor(h_full, h_local, group=self.group)
        return h_full
