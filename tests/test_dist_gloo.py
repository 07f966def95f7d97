"""Multi-rank node sharding rehearsed on CPU with gloo (world sizes 2 and 4).

Every rank builds its shard with the product partition code (gnnea.dist), all-gathers the halo
inside its KG group, aggregates its rows with the CPU oracle, and rank 0 checks the union of the
shards against the single-process oracle over the whole graph.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, t, q, kind="rows"):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "gnn-mtl_amd"))
    sys.path.insert(0, root)
    from gnnea import synth
    from gnnea.dist import Partition, halo_gather, make_groups, shard_coo
    from oracle.gnn import coo_aggregate
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        part = Partition(n, rank, world, kind, 16)
        group = make_groups(part)
        triples = synth.kg_pair_triples(n, t, 50)
        r, c, v = shard_coo(triples, n, t, part)
        H = torch.from_numpy(synth.features(2 * n, 16, seed=4)).double()
        if part.kg is None:
            h_local = H
        else:
            h_local = H[part.global_row0:part.global_row0 + part.n_rows]
        h_full = torch.empty(part.n_cols, 16, dtype=torch.float64)
        if kind in ("features", "tiles") and part.g > 1:
            # the rank's rows x column slice, gathered from the whole KG's slice: no exchange
            hk = H[part.kg * n:(part.kg + 1) * n, part.col0:part.col1]
            ys = coo_aggregate(r, c, v, part.n_rows, hk)
            outs = [torch.empty_like(ys) for _ in range(world)]
            dist.all_gather(outs, ys)
            if rank == 0:
                full = torch.empty(2 * n, 16, dtype=torch.float64)
                for k in range(world):
                    pk = Partition(n, k, world, kind, 16)
                    full[pk.kg * n + pk.row0:pk.kg * n + pk.row1, pk.col0:pk.col1] = outs[k]
                R, Cc, V = synth.adjacency_coo(triples, 2 * n, reference_order=False)
                ref = coo_aggregate(R, Cc, V, 2 * n, H)
                q.put(float((full - ref).abs().max()))
            return
        if part.g == 1:
            y = coo_aggregate(r, c, v, part.n_rows, h_local)
        else:
            # the product's per-slice pipeline (gnnea.dist.KGShard.aggregate, DistAdj): the own
            # rows packed into the KG's slice tables, every slice's exchange issued at once
            # (relayed at world 4), slice q aggregated over the whole shard once it has landed
            from gnnea import exchange
            W = 6  # 16 columns: slices of 6, 6, 4
            S = (16 + W - 1) // W
            tables = torch.full((S, n, W), float("nan"), dtype=torch.float64)
            for k in range(S):
                blk = h_local[:, k * W:(k + 1) * W]
                tables[k, part.row0:part.row1, :blk.shape[1]] = blk
            works = exchange.all_gather_slices(list(tables), part.row0, part.n_rows, group,
                                               part.group_ranks(part.kg), part.li,
                                               other=part.other_ranks())
            y = torch.empty(part.n_rows, 16, dtype=torch.float64)
            for k in range(S):
                for w in works[k]:
                    w.wait()
                c1 = min(16, (k + 1) * W)
                y[:, k * W:c1] = coo_aggregate(r, c, v, part.n_rows,
                                               tables[k][:, :c1 - k * W].contiguous())
            # the whole-table gather as well (the unstaged fallback of DistAdj.halo)
            halo_gather(h_local, h_full, group, part.g, part=part)
            assert float((coo_aggregate(r, c, v, part.n_rows, h_full) - y).abs().max()) < 1e-12
        outs = [torch.empty_like(y) for _ in range(world)]
        dist.all_gather(outs, y)
        if rank == 0:
            full = torch.cat(outs)  # ranks are ordered KG1 rows then KG2 rows
            R, Cc, V = synth.adjacency_coo(triples, 2 * n, reference_order=False)
            ref = coo_aggregate(R, Cc, V, 2 * n, H)
            q.put(float((full - ref).abs().max()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,kind", [(2, "rows"), (4, "rows"), (4, "features"),
                                        (8, "features"), (4, "tiles"), (8, "tiles"),
                                        (2, "tiles")])
def test_sharded_aggregation_matches_single_process(world, kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 200, 700, q, kind))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) < 1e-12


def test_tiles_partition_covers_each_kg_once():
    from gnnea.dist import Partition
    n, D = 1000, 300
    for world in (2, 4, 8):
        cover = {}
        for k in range(world):
            p = Partition(n, k, world, "tiles", D)
            assert p.n_cols == n and p.gr * p.gc == p.g
            assert p.g < 2 or (p.col1 - p.col0) >= 148  # slice-major widths
            for r in range(p.row0, p.row1, 100):
                cover.setdefault((p.kg, r), []).append((p.col0, p.col1))
        for sl in cover.values():  # every (KG, row) covered by column slices tiling [0, D)
            sl.sort()
            assert sl[0][0] == 0 and sl[-1][1] == D
            assert all(sl[i][1] == sl[i + 1][0] for i in range(len(sl) - 1))


def test_feature_slices_aligned():
    from gnnea.dist import feature_slices
    for D, g in ((300, 2), (300, 4), (16, 4), (301, 3)):
        sl = feature_slices(D, g)
        assert sl[0][0] == 0 and sl[-1][1] == D
        assert all(a % 4 == 0 for a, _ in sl)
        assert all(sl[k][1] == sl[k + 1][0] for k in range(g - 1))


def test_partition_covers_every_row_once():
    from gnnea.dist import Partition
    for world in (1, 2, 4, 8):
        seen = np.zeros(2 * 1000, dtype=int)
        for rank in range(world):
            p = Partition(1000, rank, world)
            seen[p.global_row0:p.global_row0 + p.n_rows] += 1
        assert np.all(seen == 1)
    with pytest.raises(ValueError):
        Partition(1000, 0, 3)


def _relay_worker(rank, world, port, rows, q, mode="relay"):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "gnn-mtl_amd"))
    from gnnea import exchange
    from gnnea.dist import Partition, make_groups
    exchange.MODE = mode
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        part = Partition(world // 2 * rows, rank, world, "rows", 3)
        group = make_groups(part)
        ranks = part.group_ranks(part.kg)
        assert exchange.relay_applies(ranks, part.other_ranks()) == (mode == "relay")
        h = torch.arange(rows * 3, dtype=torch.float64).reshape(rows, 3) + 1000 * rank
        full = torch.full((world // 2 * rows, 3), -1.0, dtype=torch.float64)
        exchange.all_gather(h, full, group, ranks, part.li, copy_own=True,
                            other=part.other_ranks())
        want = torch.cat([torch.arange(rows * 3, dtype=torch.float64).reshape(rows, 3)
                          + 1000 * r for r in ranks])
        err = float((full - want).abs().max())
        # reduce-scatter: rank r's partial of every group row is (r + 1) * base; the owner's
        # rows must come back summed over the group
        g = len(ranks)
        base = torch.arange(g * rows * 3, dtype=torch.float64).reshape(g * rows, 3)
        got = exchange.reduce_scatter((rank + 1) * base, group, ranks, part.li,
                                      other=part.other_ranks())
        want_rs = sum(r + 1 for r in ranks) * base[part.li * rows:(part.li + 1) * rows]
        err = max(err, float((got - want_rs).abs().max()))
        q.put((rank, err))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["relay", "p2p"])
@pytest.mark.parametrize("world,rows", [(4, 1), (4, 7), (4, 100), (8, 5), (8, 77)])
def test_relay_exchange(world, rows, mode):
    """The two-phase relays (units direct and through the other group's GPUs) deliver exactly
    every group peer's block (all-gather) and the group sum of the owner's rows (reduce-scatter),
    for row counts that do not split into equal units; GNNEA_HALO=p2p (the direct schedule) the
    same.  (GNNEA_HALO=ring, RCCL's all_gather_into_tensor / reduce_scatter_tensor, has no gloo
    form: on gloo the p2p schedule runs.)"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_relay_worker, args=(r, world, port, rows, q, mode))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [q.get(timeout=5) for _ in range(world)]
    assert all(err == 0.0 for _, err in res), res
