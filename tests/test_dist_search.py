"""Hard-negative mining and Hits@k over a row-sharded output (gnnea.dist_search; models/models_ea.py:
19-30, utils/eval_utils.py:71-98, 161-167) across gloo ranks on CPU: the query rows by one
all-reduce, per-rank L1 top-k over the rank's own rows merged by (distance, index), per-rank
candidate blocks of the pair ranks summed.  Index-exact against the reference's own outputs in
tests/golden/l1_search.npz (get_neg x 2, get_hits on train / test, eval_at_1) and against the
single-process search on a tie-heavy embedding (duplicated rows: equal distances everywhere).

The local search is an exact fp64 double of the HIP kernels (scipy cityblock, the reference's own
distance; ties by index) — the engine is the only stand-in; the device kernels themselves are
pinned to the same fixture in tests/test_gpu_l1.py.
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


class CpuSearchEngine:
    """Exact fp64 double of gnnea.dist_search.HipSearchEngine (test stand-in, never shipped)."""

    @staticmethod
    def _d(Q, X):
        from scipy.spatial.distance import cdist
        return cdist(Q.double().numpy(), X.double().numpy(), metric="cityblock")

    def topk(self, Q, X, K):
        d = self._d(Q, X)
        idx = np.argsort(d, axis=1, kind="stable")[:, :K]  # (distance, index) order
        return torch.from_numpy(idx.astype(np.int64)), torch.from_numpy(
            np.take_along_axis(d, idx, 1))

    def pairs(self, A, B):
        return torch.from_numpy(np.abs(A.double().numpy() - B.double().numpy()).sum(1))

    def ranks(self, Q, X, diag, x_off):
        if X.shape[0] == 0:
            return torch.zeros(Q.shape[0], dtype=torch.int32)
        d = self._d(Q, X)
        dq = diag.numpy()[:, None]
        xs = x_off + np.arange(X.shape[0])[None, :]
        q = np.arange(Q.shape[0])[:, None]
        return torch.from_numpy(((d < dq) | ((d == dq) & (xs < q))).sum(1).astype(np.int32))


def _single(vec, ILL, k):
    """The single-process search on the whole embedding (same engine, one block)."""
    e = CpuSearchEngine()
    idx, _ = e.topk(vec[torch.as_tensor(ILL)], vec, k + 1)
    return idx[:, 1:].reshape(-1).numpy()


def _worker(rank, world, port, case, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "gnn-mtl_amd"))
    sys.path.insert(0, os.path.join(root, "tests"))
    from gnnea import dist_search
    from gnnea.dist import Partition
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        f = np.load(os.path.join(root, "tests", "golden", "l1_search.npz"))
        vec = torch.from_numpy(f["vec"])
        if case == "ties":  # every row repeated 4 times: equal distances everywhere
            vec = vec[torch.arange(vec.shape[0]) // 4 * 4].contiguous()
        n_all = vec.shape[0]
        part = Partition(n_all // 2, rank, world, "rows")
        out_loc = vec[part.global_row0:part.global_row0 + part.n_rows]
        eng = CpuSearchEngine()
        tr, te = f["train"], f["test"]
        res = {"neg_r": dist_search.get_neg(tr[:, 0], out_loc, part, 25, eng),
               "neg_l": dist_search.get_neg(tr[:, 1], out_loc, part, 25, eng),
               "hits_train": dist_search.get_hits(out_loc, part, tr, engine=eng),
               "hits_test": dist_search.get_hits(out_loc, part, te, engine=eng),
               "at1": float(dist_search.eval_at_1(out_loc, part, te, eng))}
        if case == "ties":
            res["single_r"] = _single(vec, tr[:, 0], 25)
            res["single_l"] = _single(vec, tr[:, 1], 25)
            lr, rl = dist_search.hits_ranks(out_loc, part, te, eng)
            res["lr"], res["rl"] = lr.numpy(), rl.numpy()
            L, R = vec[torch.as_tensor(te[:, 0])], vec[torch.as_tensor(te[:, 1])]
            diag = eng.pairs(L, R)
            res["lr1"] = eng.ranks(L, R, diag, 0).numpy()
            res["rl1"] = eng.ranks(R, L, diag, 0).numpy()
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _run(world, case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    import time
    out, t0 = [], time.time()
    while len(out) < world:  # fail fast when a rank dies (its peers would wait in a collective)
        try:
            out.append(q.get(timeout=1))
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            if dead or time.time() - t0 > 300:
                for p in procs:
                    p.kill()
                raise AssertionError("rank failed: %s" % [p.exitcode for p in procs])
    for p in procs:
        p.join(60)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return dict(out)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_search_vs_reference_fixture(golden, world):
    f = golden("l1_search")
    res = _run(world, "fixture")
    for rank, r in res.items():
        assert (r["neg_r"] == f["neg_right"]).all(), rank
        assert (r["neg_l"] == f["neg2_left"]).all(), rank
        for split in ("train", "test"):
            want = dict(zip(f["hits_%s_keys" % split], f["hits_%s_vals" % split]))
            got = r["hits_" + split]
            for key, v in want.items():
                assert got[key] == pytest.approx(v, abs=1e-12), (rank, split, key)
        assert r["at1"] == pytest.approx(float(f["eval_at_1"]), abs=1e-12)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_search_ties(world):
    """Duplicated rows: the merged per-rank lists keep the single-process (distance, index)
    order exactly, and the per-block pair ranks sum to the single-block ranks."""
    res = _run(world, "ties")
    for rank, r in res.items():
        assert (r["neg_r"] == r["single_r"]).all(), rank
        assert (r["neg_l"] == r["single_l"]).all(), rank
        assert (r["lr"] == r["lr1"]).all() and (r["rl"] == r["rl1"]).all(), rank


def test_sharded_search_bytes():
    """Per-rank traffic is O(t·D + W·t·k): the query all-reduce and the list all-gather only."""
    t, D, k, W = 4500, 300, 125, 8
    query = t * D * 4
    lists = W * t * (k + 1) * 16
    assert query + lists < 100e6  # vs 2.4 GB of gather_rows at cfg-4
