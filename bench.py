"""Headline benchmark: edges aggregated/s of the GCN CSR aggregation (+ Sinkhorn iters/s).

Workload (BASELINE.json configs[3] graph, the largest single-GPU configuration): the synthetic
2 x 1M-entity / 2 x 10M-triple KG pair of SURVEY.md §8d (41,999,552 nnz incl. self loops),
D = 300 fp32 features resident in HBM.  A step = one GCN aggregation pass Y = relu(A · H) over
the whole graph (layers/layers.py:35-38).  On N > 1 GPUs the two KGs go to two groups of N/2
ranks (N = 2: one KG per GPU, nothing to exchange); inside a group each rank owns a block of
destination rows and the step includes the halo exchange a graph layer needs — the group's
projected rows by direct peer transfers over xGMI (gnnea/exchange.py), overlapped with the
aggregation over the owned rows (default --partition rows).  The exchange-free partitions
(tiles / features: every rank aggregates a column slice from the whole KG, which a layer can
only do after an all-gather of its input) are reported as a labelled side number.

Side measurement `dbp15k_step_graph` (N = 1): the DBP15K-scale GCN-EA and GAT-EA iteration with
Adam (configs[1] / [2]), eager against one captured HIP graph replay (tools/graph_step.py).
Side measurements (`train_step`, `train_step_gat`, `train_step_gcn`, `train_step_gat_cfg5_bf16`):
the row-sharded EA training steps through the drop-in Encoder/Decoder modules with the RCCL halo
exchange (tools/dist_step.py) -- HGCN-EA on the cfg-4 graph (configs[3]), GAT-EA and GCN-EA fp32
on the same graph (configs[2]'s and configs[1]'s models), GAT-EA bf16 on the cfg-5 graph
(configs[4]) -- at N = 1 and row-sharded at N > 1, each with per-kernel-class GPU time.

  python bench.py [--gpus N] [--steps K] [--warmup W]   (N > 1: starts its own N ranks)
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (N > 1)

With --gpus N > 1 and no WORLD_SIZE in the environment, this process is only the launcher
(tools/launch.py): before anything imports torch it starts N children of this script with the
rank environment set (one per GPU, rendezvous on 127.0.0.1), relays their output and exits with
the first failing child's status.  Under torch.distributed.run each process is already a rank.

Prints ONE JSON line on rank 0.  `roofline` prices the SpMM kernel with the gather model
4(N+1) + 8E + 4ED + 4ND bytes per launch over its HIP-event duration on the
launching stream; at cfg-4 most of those gathered bytes are served by the Infinity Cache
(each 64-column slice of a KG is a 256 MB table), so `roofline.compulsory` adds the
compulsory-traffic model (CSR once per slice pass + the table once + Y once) and its fraction
of HBM.  `cpu_baseline` times the reference ops on the host cores (rank 0, N = 1 only):
torch.spmm on the uncoalesced COO (all threads and 1 thread), one GAT head
(layers/att_layers.py:29-61) and the ot_loss Sinkhorn loop (utils/ot_loss.py:50-66), each on a
bounded sample (oracle/cpu_baseline.py).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))


def self_launch(argv, script=None):
    """Launcher path: N > 1 ranks asked for and none set up (tools/launch.py).  Returns the exit
    status to leave with, or None when this process is a rank itself.  Runs before torch is
    imported, so the launcher process never initialises HIP."""
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    from tools import launch
    if not launch.needs_launch(argv):
        return None
    return launch.spawn(launch.requested_ranks(argv), script or os.path.abspath(__file__), argv)


if __name__ == "__main__":
    _rc = self_launch(sys.argv[1:])
    if _rc is not None:
        sys.exit(_rc)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))

from gnnea import _lib, ops, synth  # noqa: E402
from gnnea.dist import KGShard  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
D = 300


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pmc_traffic(world, kernel):
    """Per-launch memory-side bytes of the SpMM kernel from the newest committed rocprofv3 PMC
    summary of the same workload at N = 1 (tools/prof_sliced.sh + tools/pmc_summary.py):
    (traffic bytes, source, extra fields)."""
    if world != 1:
        return None, None, {}
    import glob
    files = [f for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_spmm*pmc*.json")))
             if json.load(open(f)).get("kernel") == kernel]
    if not files:
        return None, None, {}
    d = json.load(open(files[-1]))
    extra = {k: d[k] for k in ("l2_hit_rate", "dram_side_read_bytes") if k in d}
    return d.get("traffic_bytes"), os.path.relpath(files[-1], ROOT), extra


def gather_model_bytes(n_rows, nnz, d, elem=4):
    return 4 * (n_rows + 1) + 8 * nnz + elem * nnz * d + elem * n_rows * d


def compulsory_bytes(n_rows, n_cols, nnz, d, sliced, elem=4, slice_w=64):
    """Bytes that must cross HBM once per SpMM: the int32 CSR (re-read once per column slice by
    the slice-major kernel), the feature table once (padded to whole slices), Y once."""
    passes = (d + slice_w - 1) // slice_w if sliced else 1
    dt = passes * slice_w if sliced else d
    return passes * (4 * (n_rows + 1) + 8 * nnz) + elem * n_cols * dt + elem * n_rows * d


def sinkhorn_rate(device, B=3000, reg=0.01, n0=100, n1=1100, variant=None, flags=0):
    """Marginal iters/s of utils/ot_loss.sinkhorn and SinkhornOT sinkhorn_iteration at B x B."""
    from gnnea.sinkhorn import solve
    g = torch.Generator(device="cpu").manual_seed(0)
    X = 0.05 * torch.randn(B, 300, generator=g)
    Y = 0.05 * torch.randn(B, 300, generator=g)
    M = torch.cdist(X, Y)
    M = (M / M.max()).to(device)
    out, paths = {}, {}
    # ot_loss.sinkhorn as models_ea.py:217 calls it (a = b = ones); sinkhorn_iteration with the
    # uniform marginals mu = nu = 1/B
    for name, mode, w in (("ot_loss.sinkhorn", _lib.GNNEA_SK_KNOPP, 1.0),
                          ("sinkhorn_iteration", _lib.GNNEA_SK_STAB, 1.0 / B)):
        la_m = torch.full((B,), w, dtype=torch.float64, device=device)
        lb = la_m
        C = M if mode == _lib.GNNEA_SK_KNOPP else M.double()
        ts = []
        for n_it in (n0, n1):
            # tol = -1: never converges, so exactly n_it iterations run
            solve(mode, C, la_m, lb, reg, -1.0, n_it, want_plan=False, batch=100,
                  variant=variant, flags=flags)  # warm
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = solve(mode, C, la_m, lb, reg, -1.0, n_it, want_plan=False, batch=100,
                        variant=variant, flags=flags)
            assert res.iters == n_it, (name, res.iters, n_it)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        out[name] = round((n1 - n0) / (ts[1] - ts[0]), 1)
        paths[name] = res.path
    return {"iters_per_s": out, "B": B, "reg": reg, "dtype": "f64 (C fp32/fp64)", "path": paths,
            "method": "marginal (T(%d)-T(%d))/%d incl. the host's look-ahead status reads"
                      % (n1, n0, n1 - n0)}


def sinkhorn_large(device):
    """B = 15000 through the default path (GNNEA_SK_AUTO): KNOPP (utils/ot_loss.sinkhorn) on the
    fused log-domain sweep (fp32 C read once per iteration, I * J * 4 bytes, one exponential per
    element; csrc/sinkhorn_log.hip k_lsk_sweep), STAB on the scaling form with the fp64 K
    resident; beside it the scaling form for KNOPP too (variant 0: one sweep over the fp64 K per
    iteration, I * J * 8 bytes) and the two-pass log-domain form the fused sweep replaced
    (flag GNNEA_SK_TWO_PASS: C read twice, two exponentials per element): marginal iters/s."""
    B = 15000
    r = sinkhorn_rate(device, B=B, n0=20, n1=120)
    c_bytes = B * B * 4
    knopp = r["iters_per_s"]["ot_loss.sinkhorn"]
    r["kernels_knopp"] = ("fused log-domain sweep k_lsk_sweep + k_lsk_colfin + k_lsk_fix (one pass "
                          "over fp32 C, one table exponential per element)")
    r["bytes_per_iter_knopp"] = c_bytes
    r["GBps_knopp"] = round(knopp * c_bytes / 1e9, 1)
    r["bound_knopp"] = ("the fp32 C stream (%.2f GB per iteration; %.0f iters/s at 8 TB/s) against "
                        "2.25e8 fp64 table exponentials per iteration" % (c_bytes / 1e9,
                                                                          8e12 / c_bytes))
    sc = sinkhorn_rate(device, B=B, n0=20, n1=120, variant=0)
    k_bytes = B * B * 8
    r["scaling_form"] = {
        "iters_per_s": sc["iters_per_s"], "path": sc["path"], "bytes_per_iter": k_bytes,
        "GBps_knopp": round(sc["iters_per_s"]["ot_loss.sinkhorn"] * k_bytes / 1e9, 1),
        "kernels": "fp64 K resident in HBM (k_sk_sweep, wide: column scaling in LDS)",
        "bound": "HBM: the K stream (%.2f GB per iteration; %.0f iters/s at 8 TB/s)"
                 % (k_bytes / 1e9, 8e12 / k_bytes)}
    two = sinkhorn_rate(device, B=B, n0=20, n1=120, variant=1, flags=_lib.GNNEA_SK_TWO_PASS)
    r["logdomain_two_pass_iters_per_s"] = two["iters_per_s"]
    return r


def sinkhorn_sharded(device, rank, world, B=15000, reg=0.01, n0=20, n1=120):
    """§8e: utils/ot_loss.sinkhorn at B = 15000 with the cost rows sharded over the ranks
    (gnnea.sinkhorn.solve_row_sharded: per iteration one all-gather of W x (2B + 2) doubles of
    column (max, sum-exp) pairs).  Marginal iters/s, max over ranks; every rank calls this."""
    from gnnea.sinkhorn import solve_row_sharded
    g = torch.Generator(device="cpu").manual_seed(0)
    X = (0.05 * torch.randn(B, 300, generator=g)).to(device)
    Y = (0.05 * torch.randn(B, 300, generator=g)).to(device)
    r0, r1 = B * rank // world, B * (rank + 1) // world
    M = torch.cdist(X[r0:r1], Y)
    host = dist.get_backend() == "gloo"  # --rehearse: the logic on one device, host-staged

    def allreduce_max(t):
        t = t.cpu() if host else t
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t.to(device)
    mx = allreduce_max(M.max().reshape(1))
    M = (M / mx).contiguous()
    del X, Y
    a = torch.ones(r1 - r0, dtype=torch.float64, device=device)
    b = torch.ones(B, dtype=torch.float64, device=device)
    ts = []
    for n_it in (n0, n0, n1):  # the first solve warms the kernels and the communicator
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = solve_row_sharded(M, a, b, reg, -1.0, n_it, want_plan=False)
        torch.cuda.synchronize()
        t = allreduce_max(torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                                       device=device))
        assert res.iters == n_it, (res.iters, n_it)
        ts.append(t.item())
    return {"iters_per_s": round((n1 - n0) / (ts[2] - ts[1]), 1), "B": B, "reg": reg,
            "ranks": world, "rows_per_rank": r1 - r0,
            "exchange_bytes_per_iter_per_rank": world * (2 * B + 2) * 8,
            "method": "marginal (T(%d)-T(%d))/%d, max over ranks, incl. the per-iteration "
                      "all-gather and host batch syncs" % (n1, n0, n1 - n0),
            "kernels": "gnnea_sinkhorn_shard_* (csrc/sinkhorn_shard.hip)"}


def gw_rate(device, B=3000):
    """One GW outer-iteration cost rebuild (SinkhornOT/cderivation.py:160-162, get_LT:
    constC - C1 . T . C2^T) in fp64 on the f64 MFMA GEMM, 2 * I * J * (I + J) flops."""
    from SinkhornOT.cderivation import get_LT
    g = torch.Generator(device="cpu").manual_seed(0)
    C1 = torch.rand(B, B, generator=g, dtype=torch.float64).to(device)
    C2 = torch.rand(B, B, generator=g, dtype=torch.float64).to(device)
    T = torch.full((B, B), 1.0 / (B * B), dtype=torch.float64, device=device)
    constC = torch.rand(B, B, generator=g, dtype=torch.float64).to(device)
    ms = _timed(lambda: get_LT(constC, C1, C2, T), 5)
    flop = 2.0 * B * B * (B + B)
    return {"ms": round(ms, 3), "TFLOPs": round(flop / ms / 1e9, 1), "I": B, "J": B,
            "dtype": "f64", "kernel": "gnnea::k_gemm_f64 (v_mfma_f64_16x16x4_f64), 2 launches",
            "peak_TFLOPs": 78.6, "peak_source": "AMD MI355X spec FP64 matrix (not in MI355X_MICROARCH.md)"}


def fgw_rate(device, B=3000, outer=4, eps=0.1, alpha=0.5):
    """The FGW outer loop of configs[4] (SinkhornOT/iterative_projection.py:125 fgw_iterative_1,
    cderivation.py:147-189) at the EA batch B = 3000 in fp32 and bf16 inputs: per outer
    iteration the cost rebuild C1·T·C2ᵀ (two GEMMs, x3 fp32 / bf16 MFMA) and the stabilised
    Sinkhorn solve on it (sinkhorn_iteration, <= 100 iterations, fp64 on the device).  ms per
    outer iteration = (T(outer) - T(1)) / (outer - 1) with tol = -1 (every iteration runs)."""
    from SinkhornOT.cderivation import get_LT
    from SinkhornOT.iterative_projection import fgw_iterative_1
    g = torch.Generator(device="cpu").manual_seed(0)
    X = 0.05 * torch.randn(B, 300, generator=g)
    Y = 0.05 * torch.randn(B, 300, generator=g)
    out = {"B": B, "epsilon": eps, "alpha": alpha, "p": 1, "inner": "sinkhorn_iteration "
           "(numIterMax 100, tol 1e-9)", "method": "(T(%d) - T(1)) / %d outer iterations, "
           "tol = -1" % (outer, outer - 1)}
    for name, dt in (("f32", torch.float32), ("bf16", torch.bfloat16)):
        C1 = torch.cdist(X, X)
        C2 = torch.cdist(Y, Y)
        D_ = torch.cdist(X, Y)
        C1, C2, D_ = [(m / m.max()).to(device=device, dtype=dt) for m in (C1, C2, D_)]
        mu = torch.full((B,), 1.0 / B, dtype=dt, device=device)
        nu = torch.full((B,), 1.0 / B, dtype=dt, device=device)
        ts = []
        for n_out in (1, outer):
            fgw_iterative_1(D_, C1, C2, mu, nu, alpha, 1, n_out, eps, tol=-1.0)  # warm
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fgw_iterative_1(D_, C1, C2, mu, nu, alpha, 1, n_out, eps, tol=-1.0)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        T = torch.full((B, B), 1.0 / (B * B), dtype=dt, device=device)
        constC = torch.rand(B, B, generator=g).to(device=device, dtype=dt)
        ms_lt = _timed(lambda: get_LT(constC, C1, C2, T), 5)
        out[name] = {"ms_per_outer_iteration": round((ts[1] - ts[0]) / (outer - 1) * 1e3, 3),
                     "cost_rebuild_ms": round(ms_lt, 3),
                     "cost_rebuild_TFLOPs": round(4.0 * B ** 3 / ms_lt / 1e9, 1)}
    return out


def bf16_rate(device, steps):
    """The aggregation with bf16 feature storage (cfg-5's dtype, fp32 arithmetic) on cfg-5's
    own graph (synth.CONFIGS["cfg5"]: 2 x 2M entities, 2 x 20M triples, ~84M nnz): the table
    slice-major in 128-column (256-B pieces, ops.spmm_sliced) and 64-column (128-B pieces,
    ops.spmm_sliced64) slices -- the value is the faster one's -- and the row-major kernel."""
    cf = synth.CONFIGS["cfg5"]
    t0 = time.time()
    shard = KGShard(cf["n"], cf["t"], cf["n_rel"], 0, 1, device, kind="rows", D=D)
    build_s = time.time() - t0
    gen = torch.Generator(device=device).manual_seed(5)
    Hb = torch.randn(shard.n_cols, D, device=device, generator=gen)
    Hb /= Hb.norm(dim=1, keepdim=True)
    Hb = Hb.to(torch.bfloat16)
    Yb = torch.empty((shard.n_rows, D), dtype=torch.bfloat16, device=device)
    relu = _lib.GNNEA_ACT_RELU
    sliced = ops.use_sliced(shard.n_cols, D, torch.bfloat16)
    ms_row = _timed(lambda: ops.spmm(shard.csr, Hb, relu, out=Yb), steps)
    W = ops.slice_w(torch.bfloat16)
    ms128 = ms64 = None
    kernel = "gnnea::k_spmm_v4<relu,act,2,bf16,bf16>"
    if sliced:
        Hs = ops.slice_pack(Hb)
        ms128 = _timed(lambda: ops.spmm_sliced(shard.csr, Hs, D, relu, out=Yb), steps)
        del Hs
        # 64-column slices (128 B per row piece): one KG slice = n * 128 B = 256 MB at 2M rows
        Hs = ops.slice_pack64(Hb)
        ms64 = _timed(lambda: ops.spmm_sliced64(shard.csr, Hs, D, relu, out=Yb), steps)
        del Hs
        # the value is the faster layout's (both reported)
        if ms64 <= ms128:
            ms, W, kernel = ms64, 64, "gnnea::k_spmm_sliced64_bf16<1, 2, unsigned short>"
        else:
            ms, W, kernel = ms128, 128, "gnnea::k_spmm_sliced<1, 2, false, unsigned short, unsigned short>"
    else:
        ms = ms_row
    traffic = gather_model_bytes(shard.n_rows, shard.nnz, D, elem=2)
    launches = len(shard.csr.row_blocks())
    achieved = traffic / (ms * 1e-3) / 1e9
    out = {"graph": "cfg-5: 2x%d entities, 2x%d triples, %d nnz (built in %.1f s)"
                    % (cf["n"], cf["t"], shard.nnz, build_s),
           "value": round(shard.nnz / ms * 1e3, 1), "unit": "edges/s", "ms_per_step": round(ms, 4),
           "dtype": "bf16 storage, f32 accumulate", "timing": TIMING,
           "layout": ("slice-major (%d-column slices: %d MB per KG slice)"
                      % (W, cf["n"] * W * 2 >> 20)) if sliced else "row-major",
           "rowmajor_edges_per_s": round(shard.nnz / ms_row * 1e3, 1),
           "slices128_edges_per_s": round(shard.nnz / ms128 * 1e3, 1) if ms128 else None,
           "slices64_edges_per_s": round(shard.nnz / ms64 * 1e3, 1) if ms64 else None,
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                        "kernel": kernel,
                        "launches_per_step": launches,
                        "model": "gather: 4(N+1)+8E+2ED+2ND"}}
    del shard, Hb, Yb
    torch.cuda.empty_cache()
    return out


TIMING = "median of >= 21 per-call HIP events after 3 warm-ups"


def _timed(fn, steps):
    """Median of max(21, steps) per-call HIP-event durations (ms) after 3 warm-up calls
    (SURVEY.md §8d)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(max(21, steps))]
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in evs]))


def anchors(device, copy_bytes=4 << 30, n_gather=16 << 20):
    """The bandwidth anchors the roofline fractions are read against (csrc/ubench.hip): a
    hand-written streaming copy (16 B per lane) and uniform-random whole-row gathers from tables
    far larger than the 256-MB Infinity Cache, at the row sizes of the gather passes: 600 B (a
    bf16 cfg-5 row, the row-major GAT passes), 1200 B (an fp32 cfg-4 row), 256 B (a 64-column
    fp32 slice row of the sliced passes); median of 21 HIP-event timings each."""
    L = _lib.lib()
    st = lambda: _lib.stream_of(device)  # noqa: E731
    out = {}
    src = torch.empty(copy_bytes // 4, dtype=torch.float32, device=device).fill_(1.0)
    dst = torch.empty_like(src)
    ncu = torch.cuda.get_device_properties(device).multi_processor_count
    # the copy (and its loads alone) over grids of 4 / 8 / 16 workgroups per CU, 4 or 8 accesses
    # in flight, plain or nontemporal: the best of each is the anchor, the whole sweep is kept
    sweep = {}
    for ro in (0, _lib.GNNEA_UB_READ_ONLY):
        for fl in (0, _lib.GNNEA_UB_NT, _lib.GNNEA_UB_DEEP, _lib.GNNEA_UB_NT | _lib.GNNEA_UB_DEEP):
            for per_cu in (4, 8, 16):
                f = ro | fl
                ms = _timed(lambda: _lib.check(L.gnnea_ub_copy(_lib.ptr(src), _lib.ptr(dst),
                                                               copy_bytes, per_cu * ncu, f,
                                                               st())), 11)
                moved = copy_bytes if ro else 2 * copy_bytes
                sweep["%s%s%s/%dpercu" % ("read" if ro else "copy", "_nt" if fl & 1 else "",
                                          "_deep" if fl & 2 else "", per_cu)] = round(
                    moved / (ms * 1e-3) / 1e9, 1)
    best_copy = max((k for k in sweep if k.startswith("copy")), key=sweep.get)
    best_read = max((k for k in sweep if k.startswith("read")), key=sweep.get)
    out["copy"] = {"GBps": sweep[best_copy], "config": best_copy, "bytes": 2 * copy_bytes,
                   "kernel": "gnnea::k_ub_copy (16 B per lane)"}
    out["read"] = {"GBps": sweep[best_read], "config": best_read, "bytes": copy_bytes,
                   "kernel": "gnnea::k_ub_copy read only (16 B per lane)"}
    out["copy_sweep_GBps"] = sweep
    ms_t = _timed(lambda: dst.copy_(src), 21)
    out["torch_copy"] = {"GBps": round(2 * copy_bytes / (ms_t * 1e-3) / 1e9, 1),
                         "ms": round(ms_t, 4)}
    del src, dst
    torch.cuda.empty_cache()
    g = torch.Generator(device=device).manual_seed(11)
    res = torch.empty((n_gather + 63) // 64, dtype=torch.float32, device=device)
    for row_bytes, rows in ((600, 4_000_000), (1200, 2_000_000), (256, 4_000_000)):
        table = torch.empty(rows * row_bytes, dtype=torch.uint8, device=device).fill_(3)
        idx = torch.randint(0, rows, (n_gather,), dtype=torch.int32, device=device, generator=g)
        ms = _timed(lambda: _lib.check(L.gnnea_ub_gather(_lib.ptr(table), row_bytes,
                                                         _lib.ptr(idx), n_gather, _lib.ptr(res),
                                                         0, st())), 21)
        out["gather_%dB" % row_bytes] = {
            "GBps": round(n_gather * row_bytes / (ms * 1e-3) / 1e9, 1), "ms": round(ms, 4),
            "table_MB": rows * row_bytes >> 20, "rows_gathered": n_gather,
            "kernel": "gnnea::k_ub_gather (8-B chunks, 4 rows in flight per wave)"}
        del table, idx
        torch.cuda.empty_cache()
    # the row-major bf16 GAT passes' access shapes: 600-B rows read as 12-B windows per lane
    # (their layout) against rows padded to 608 B read 16 B per lane (38 lanes)
    for name, mode, row_bytes in (("gat_win12_600B", _lib.GNNEA_UB_GAT_WIN12, 600),
                                  ("gat_v16_608B", _lib.GNNEA_UB_GAT_V16, 608)):
        rows = 4_000_000
        table = torch.empty(rows * row_bytes, dtype=torch.uint8, device=device).fill_(3)
        idx = torch.randint(0, rows, (n_gather,), dtype=torch.int32, device=device, generator=g)
        ms = _timed(lambda: _lib.check(L.gnnea_ub_gather(_lib.ptr(table), row_bytes,
                                                         _lib.ptr(idx), n_gather, _lib.ptr(res),
                                                         mode, st())), 21)
        out[name] = {"GBps_row_bytes": round(n_gather * row_bytes / (ms * 1e-3) / 1e9, 1),
                     "GBps_600B_payload": round(n_gather * 600 / (ms * 1e-3) / 1e9, 1),
                     "ms": round(ms, 4), "table_MB": rows * row_bytes >> 20}
        del table, idx
        torch.cuda.empty_cache()
    out["peak_spec_GBps"] = HBM_PEAK_GBS
    return out


def layout_rates(shard, H, Y, steps):
    """Side measurements of the same aggregation: the row-major table (k_spmm_v4 over 1,200-B
    rows) and the drop-in path for a row-major hidden no gnnea GEMM produced (pack into slices +
    sliced aggregation, what ops.AggregateFn does above the Infinity Cache)."""
    relu = _lib.GNNEA_ACT_RELU
    D_ = H.shape[1]
    out = {}
    for name, fn in (("rowmajor", lambda: ops.spmm(shard.csr, H, relu, out=Y)),
                     ("pack_then_sliced",
                      lambda: ops.spmm_sliced(shard.csr, ops.slice_pack(H), D_, relu, out=Y))):
        ms = _timed(fn, steps)
        out[name] = {"edges_per_s": round(shard.nnz / ms * 1e3, 1), "ms_per_step": round(ms, 4)}
    return out


def cpu_baseline(shard, H, budget_s=12.0):
    """Reference ops on the host: torch.spmm on the uncoalesced COO rows of a bounded sample
    (all threads, then 1 thread), one GAT head and the ot_loss Sinkhorn loop."""
    from oracle.cpu_baseline import (cpu_model, time_reference_gat, time_reference_sinkhorn,
                                     time_reference_spmm)
    threads = torch.get_num_threads()
    n = shard.n
    tr = synth.kg_pair_triples(n, shard_t(n), synth.CONFIGS["cfg4"]["n_rel"])
    r, c, v = synth.adjacency_coo(tr, 2 * n, reference_order=True)
    Hc = H.detach().cpu()
    N = 2 * n
    rate, nnz, dt = time_reference_spmm(r, c, v, N, N, Hc, sample_rows=N // 50)
    want_rows = int(min(N, max(N // 50, rate * budget_s / max(nnz / (N // 50), 1))))
    rate, nnz, dt = time_reference_spmm(r, c, v, N, N, Hc, sample_rows=want_rows)
    out = {"value": round(rate, 1), "unit": "edges/s", "cores": threads, "kind": "port",
           "cpu_model": cpu_model(),
           "sample": "torch.spmm(uncoalesced int64 COO, H fp32) over the first %d of %d rows "
                     "(%d edges, %.1f s) of the same cfg-4 graph, reference entry order" %
                     (want_rows, N, nnz, dt)}
    try:
        torch.set_num_threads(1)
        rows1 = max(1000, N // 5)
        r1, nnz1, dt1 = time_reference_spmm(r, c, v, N, N, Hc, sample_rows=rows1)
        out["value_1thread"] = round(r1, 1)
        out["sample_1thread"] = "first %d rows (%d edges, %.1f s)" % (rows1, nnz1, dt1)
    finally:
        torch.set_num_threads(threads)
    # one GAT head (4 x 75 heads per layer at cfg-4): head-edges/s on a row sample
    g = torch.Generator().manual_seed(3)
    W = torch.randn(H.shape[1], 75, generator=g) * 0.05
    a = torch.randn(1, 150, generator=g) * 0.05
    rows_g = max(1000, N // 100)
    rg, eg, dtg = time_reference_gat(r, c, v, N, Hc, W, a, rows_g)
    out["gat_head"] = {"value": round(rg, 1), "unit": "head-edges/s", "cores": threads,
                       "sample": "one SpGraphAttentionLayer head (layers/att_layers.py:29-61, "
                                 "300 -> 75) over destination rows < %d (%d edges, %.1f s; "
                                 "h = x.W over all %d rows included)" % (rows_g, eg, dtg, N)}
    gs = torch.Generator().manual_seed(0)
    X = 0.05 * torch.randn(3000, 300, generator=gs)
    Y = 0.05 * torch.randn(3000, 300, generator=gs)
    M = torch.cdist(X, Y)
    rs, dts = time_reference_sinkhorn(M / M.max(), 0.01, 300)
    out["sinkhorn"] = {"value": round(rs, 1), "unit": "iters/s", "cores": threads, "B": 3000,
                       "sample": "utils/ot_loss.py:50-66 loop body, fp64, 300 iterations "
                                 "(%.1f s)" % dts}
    return out


# EA training-step legs (tools/dist_step.measure): line key -> (encoder, graph, storage dtype).
# HGCN-EA on cfg-4 is BASELINE configs[3]; GAT-EA on cfg-4 in fp32 is configs[2]'s model at
# configs[3]'s size, GCN-EA configs[1]'s; GAT-EA on the cfg-5 graph (2 x 2M entities, ~84M nnz)
# in bf16 is configs[4]
TRAIN_LEGS = {"train_step": ("HGCN", "cfg4", "f32"),
              "train_step_gat": ("GAT", "cfg4", "f32"),
              "train_step_gcn": ("GCN", "cfg4", "f32"),
              "train_step_gat_cfg5_bf16": ("GAT", "cfg5", "bf16")}


def shard_t(n):
    return synth.CONFIGS["cfg4"]["t"] if n == synth.CONFIGS["cfg4"]["n"] else 10 * n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--entities", type=int, default=synth.CONFIGS["cfg4"]["n"],
                    help="entities per KG (default: cfg-4, 1M)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sinkhorn", action="store_true")
    ap.add_argument("--partition", choices=("rows", "tiles", "features"), default="rows",
                    help="inside a KG group: row blocks with the halo exchange a layer needs "
                         "(rows, default), or the exchange-free aggregation-only partitions: row "
                         "blocks x 2 feature-column slices (tiles), feature-column slices of all "
                         "rows (features)")
    ap.add_argument("--no-side", action="store_true",
                    help="N > 1: skip the labelled exchange-free side number (tiles)")
    ap.add_argument("--no-train", action="store_true",
                    help="skip the side measurements of the row-sharded EA training steps")
    ap.add_argument("--train-steps", type=int, default=21)
    ap.add_argument("--train-models", default=",".join(TRAIN_LEGS),
                    help="comma-separated EA training-step legs (default all: %s)"
                         % ", ".join(TRAIN_LEGS))
    ap.add_argument("--layout", choices=("sliced", "rowmajor"), default="sliced",
                    help="feature table layout of the aggregation input (sliced: 64-column "
                         "slices, each one Infinity-Cache-sized table at 1M rows)")
    ap.add_argument("--headline-only", action="store_true",
                    help="only the headline aggregation (profiling passes): no side numbers")
    ap.add_argument("--rehearse", action="store_true",
                    help="multi-rank logic on ONE device with gloo (halo staged through host)")
    args = ap.parse_args()
    if args.headline_only:
        args.no_cpu_baseline = args.no_sinkhorn = args.no_train = args.no_side = True

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("warning: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world))
    if args.rehearse:
        local = 0
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        # an explicit collective timeout: a rank stuck in a collective (e.g. the staged halo
        # misbehaving on RCCL) ends the run with a logged error instead of at the driver's kill
        import datetime
        tmo = datetime.timedelta(seconds=float(os.environ.get("GNNEA_PG_TIMEOUT_S", "300")))
        if args.rehearse:
            dist.init_process_group("gloo", timeout=tmo)
        else:
            dist.init_process_group("nccl", device_id=device, timeout=tmo)

    t0 = time.time()
    n = args.entities
    shard = KGShard(n, shard_t(n), synth.CONFIGS["cfg4"]["n_rel"], rank, world, device,
                    kind=args.partition, D=D)
    part = shard.part
    Dl = part.col1 - part.col0  # feature columns this rank aggregates
    log("rank %d: shard rows %d nnz %d built in %.1fs" % (rank, shard.n_rows, shard.nnz,
                                                         time.time() - t0))
    gen = torch.Generator(device=device).manual_seed(1 + rank)
    free = part.kind in ("features", "tiles")  # exchange-free: the whole KG's column slice
    h_local = torch.randn(shard.n_cols if (world == 1 or free) else shard.n_rows, Dl,
                          device=device, generator=gen)
    h_local /= h_local.norm(dim=1, keepdim=True)
    y = torch.empty(shard.n_rows, Dl, device=device)
    # H as the projection GEMM of a GCN layer leaves it: slice-major [ceil(D/64)][rows][64]
    # (gnnea_gemm_sliced_f32 writes this layout; ops.GCNLayerFn) where the table exceeds the
    # Infinity Cache, row-major otherwise (or with --layout rowmajor)
    sliced = (args.layout == "sliced" and (shard.g == 1 or free)
              and ops.use_sliced(shard.n_cols, Dl, torch.float32))
    hs = ops.slice_pack(h_local) if sliced else None

    from gnnea import exchange as _ex
    # N > 1, row shards: prove the per-slice staged halo on THESE ranks (RCCL) before using it --
    # one HighWay, one GCN and one GAT layer fwd + bwd staged and unstaged on the same inputs
    # (gnnea.dist_graph.validate_staged); the step and the train legs take the staged path only
    # for the dtypes whose legs every rank saw agree (GNNEA_HALO_STAGED=0: always off; =1: on
    # without validation, the report still says what matched)
    # the legs run in fp32 and in bf16 (configs[4]'s storage, whose GAT stages move bf16
    # 64-column tables); each dtype takes the staged path only if its own legs matched
    halo_ab = None
    if shard.g > 1 and part.kind == "rows":
        from gnnea.dist_graph import DistAdj, validate_staged
        t_ab = time.time()
        halo_ab = validate_staged(DistAdj.from_shard(shard), D=D,
                                  dtypes=(torch.float32, torch.bfloat16))
        for dn, rep in halo_ab["dtypes"].items():
            log("rank %d: halo_ab %s match=%s err=%.3g (tol %.0e)" % (
                rank, dn, rep["match"], rep["max_norm_rel_err"], rep["tol"]))
        log("rank %d: halo_ab staged %.2f ms / unstaged %.2f ms, in use %s (%.1fs)"
            % (rank, halo_ab["staged_ms"], halo_ab["unstaged_ms"], halo_ab["staged_in_use"],
               time.time() - t_ab))
        torch.cuda.empty_cache()
    staged32 = _ex.staged_for(torch.float32)
    n_slices = (len(shard.slices(Dl)) if staged32 else 1) \
        if shard.g > 1 and part.kind == "rows" else 0

    def step(ev=None):
        shard.aggregate(h_local, y, _lib.GNNEA_ACT_RELU, ev, hs=hs)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2 + 2 * n_slices)]
           for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if shard.g == 1 or free:
        kernel_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    else:  # the per-slice aggregations (each after its slice's exchange has landed)
        kernel_ms = float(np.mean([sum(e[2 + 2 * q].elapsed_time(e[3 + 2 * q])
                                       for q in range(n_slices)) for e in evs]))
    # units = edge aggregations over the full feature width: a rank that aggregates its KG's
    # edges over Dl of the D columns contributes nnz * Dl / D of them (the slices of a KG group
    # add up to each edge exactly once); row shards contribute their own rows' edges
    units = float(shard.nnz) * Dl / D
    stats = torch.tensor([elapsed, units, kernel_ms], dtype=torch.float64,
                         device="cpu" if args.rehearse else device)
    if world > 1:
        allst = [torch.zeros_like(stats) for _ in range(world)]
        dist.all_gather(allst, stats)
        allst = torch.stack(allst).cpu()
        elapsed = float(allst[:, 0].max())
        total_nnz = float(allst[:, 1].sum())  # = nnz of the whole graph
    else:
        total_nnz = units
    ms_per_step = elapsed / args.steps * 1e3
    value = total_nnz / (elapsed / args.steps)
    # per-step HIP events on the launching stream (median; rank 0): the SURVEY §8d statistic,
    # reported beside the contract's wall-clock mean over the K steps
    step_ms = [e[0].elapsed_time(e[1]) for e in evs]

    # the same headline step in the other halo mode (staged <-> unstaged), for halo_ab
    if halo_ab is not None:
        other = {}
        keep = _ex.STAGED
        for mode in (True, False):
            if mode == staged32:
                other[mode] = ms_per_step
                continue
            if mode and not halo_ab["dtypes"]["float32"]["match"]:
                continue  # never time a pipeline that did not validate
            _ex.STAGED = mode
            try:
                for _ in range(2):
                    step()
                torch.cuda.synchronize()
                dist.barrier()
                t1 = time.perf_counter()
                for _ in range(args.steps):
                    step()
                torch.cuda.synchronize()
                dist.barrier()
                other[mode] = (time.perf_counter() - t1) / args.steps * 1e3
            finally:
                _ex.STAGED = keep
        halo_ab["headline_step_ms"] = {("staged" if m else "unstaged"): round(v, 4)
                                       for m, v in other.items()}

    # the exchange alone (rows partition inside a group): bytes each rank receives per step and
    # the time of K back-to-back exchanges, max over ranks
    exchange = None
    if shard.g > 1 and part.kind == "rows" and not args.rehearse:
        from gnnea import exchange as ex
        ranks = part.group_ranks(part.kg)

        if staged32:
            tables = shard.halo_tables(Dl)

            def xchg():  # the same per-slice exchanges as the step, without the aggregation
                for ws in ex.all_gather_slices(list(tables), part.row0, part.n_rows,
                                               shard.group, ranks, part.li,
                                               other=part.other_ranks()):
                    for w in ws:
                        w.wait()
        else:
            full = torch.empty((shard.n_cols, Dl), dtype=h_local.dtype, device=device)

            def xchg():  # the step's whole-halo exchange, without the aggregation
                ex.all_gather(h_local, full, shard.group, ranks, part.li, copy_own=True,
                              other=part.other_ranks())
        for _ in range(2):
            xchg()
        torch.cuda.synchronize()
        dist.barrier()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            xchg()
        torch.cuda.synchronize()
        xt = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=device)
        dist.all_reduce(xt, op=dist.ReduceOp.MAX)
        x_ms = float(xt) / args.steps * 1e3
        x_bytes = (shard.g - 1) * part.n_rows * Dl * 4
        relay = ex.relay_applies(ranks, part.other_ranks())
        exchange = {"transport": "RCCL ring all_gather" if ex.MODE == "ring" else
                    ("two-phase relay: quarters direct and through the other group's GPUs "
                     "(batch_isend_irecv, every link one quarter per phase)" if relay else
                     "direct peer transfers (batch_isend_irecv, one per group peer)"),
                    "peers": shard.g - 1, "bytes_recv_per_rank_per_step": x_bytes,
                    "ms_alone": round(x_ms, 4),
                    "GBps_recv_per_rank": round(x_bytes / (x_ms * 1e-3) / 1e9, 1),
                    "spmm_kernel_ms": round(kernel_ms, 4),
                    # SURVEY §8e overlap: the exchange and the aggregation cut into column
                    # slices, slice q aggregated while slices > q move; the hidden fraction of
                    # the exchange = (exchange alone + aggregation - step) / exchange alone
                    "pipeline": ("%d column slices (64 fp32 columns; slice-major KG tables)"
                                 % n_slices) if staged32 else
                                "none (GNNEA_HALO_STAGED=0: the whole halo, then the "
                                "aggregation)",
                    "step_ms": round(ms_per_step, 4),
                    "exchange_hidden_frac": round(min(1.0, max(0.0, (x_ms + kernel_ms
                                                                     - ms_per_step) / x_ms)), 3)}

    # labelled side number: the exchange-free tiles partition (aggregation only; a layer would
    # first all-gather its input, which this number does not contain)
    side = None
    if world > 2 and part.kind == "rows" and not args.no_side and not args.rehearse:
        sh2 = KGShard(n, shard_t(n), synth.CONFIGS["cfg4"]["n_rel"], rank, world, device,
                      kind="tiles", D=D)
        p2 = sh2.part
        D2 = p2.col1 - p2.col0
        h2 = torch.randn(sh2.n_cols, D2, device=device, generator=gen)
        y2 = torch.empty(sh2.n_rows, D2, device=device)
        hs2 = ops.slice_pack(h2) if ops.use_sliced(sh2.n_cols, D2, torch.float32) else None
        for _ in range(2):
            sh2.aggregate(h2, y2, _lib.GNNEA_ACT_RELU, hs=hs2)
        torch.cuda.synchronize()
        dist.barrier()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            sh2.aggregate(h2, y2, _lib.GNNEA_ACT_RELU, hs=hs2)
        torch.cuda.synchronize()
        st = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=device)
        dist.all_reduce(st, op=dist.ReduceOp.MAX)
        s_ms = float(st) / args.steps * 1e3
        side = {"partition": "tiles: %d row blocks x %d feature-column slices per KG group, "
                             "aggregation only, NO exchange (a layer needs its input "
                             "all-gathered first)" % (p2.gr, p2.gc),
                "edges_per_s": round(total_nnz / (s_ms * 1e-3), 1), "ms_per_step": round(s_ms, 4)}
        del sh2, h2, y2, hs2

    # side measurements (every rank, same collective sequence): the row-sharded EA training
    # steps through the drop-in modules with the RCCL halo exchange -- HGCN-EA (configs[3]),
    # GAT-EA fp32 on the same graph, GAT-EA bf16 on the cfg-5 graph (configs[4]); each with
    # per-kernel-class attribution.  These legs run collectives at N > 1: an exception there
    # propagates (the run exits non-zero) instead of being recorded on one rank while the others
    # wait in the next collective.  --rehearse (one device, gloo): 1 warm-up + --train-steps
    # steps, no attribution -- the code path, not a rate.
    train = {}
    if not args.no_train:
        from tools.dist_step import measure
        want = [k.strip() for k in args.train_models.split(",") if k.strip()]
        for key in want:
            model, gname, dn = TRAIN_LEGS[key]
            n_leg = n if gname == "cfg4" else (synth.CONFIGS["cfg5"]["n"]
                                               if n == synth.CONFIGS["cfg4"]["n"] else 2 * n)
            dt = torch.bfloat16 if dn == "bf16" else torch.float32
            kw = dict(min_steps=1, min_warmup=1, attribute=0) if args.rehearse else {}

            def leg():
                r = measure(model, n_leg, rank, world, device, args.train_steps,
                            1 if args.rehearse else 3, dt, **kw)
                r["config"] = {"graph_config": gname, "entities_per_kg": n_leg,
                               "storage": dn}
                return r
            if world == 1:
                try:
                    train[key] = leg()
                except Exception as e:  # report, never hide
                    train[key] = {"error": repr(e)}
            else:
                train[key] = leg()
            torch.cuda.empty_cache()
    sk_shard = None
    if world > 1 and not args.no_sinkhorn:
        # (--rehearse: the code path only; the rate means nothing there)
        sk_shard = sinkhorn_sharded(device, rank, world)

    if rank == 0:
        # the SpMM is launched once per diagonal (KG) block of rows when the gathered matrix is
        # larger than the Infinity Cache (gnnea.ops._blocks): bytes and time per launch
        launches = 1
        if shard.g == 1 or free:
            blocks = ops._blocks(shard.csr, h_local)
            launches = len(blocks)
        else:  # one sliced launch per column slice over the KG halo tables
            launches = n_slices
            sliced = True
        traffic = gather_model_bytes(shard.n_rows, shard.nnz, Dl)
        achieved = traffic / (kernel_ms * 1e-3) / 1e9
        comp = compulsory_bytes(shard.n_rows, shard.n_cols, shard.nnz, Dl, sliced)
        comp_gbs = comp / (kernel_ms * 1e-3) / 1e9
        pmc_bytes, pmc_src, pmc_extra = pmc_traffic(world, "k_spmm_sliced" if sliced else
                                                     "k_spmm_v4")
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "edges/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic",
            "ms_per_step_events_median": round(float(np.median(step_ms)), 4),
            "edges_per_s_events_median": round(total_nnz / (float(np.median(step_ms)) * 1e-3), 1),
            "config": {"workload": "GCN aggregation relu(A.H) (layers/layers.py:35-38) on the "
                                   "cfg-4 synthetic 2x%d-entity / 2x%d-triple KG pair, D=%d"
                                   % (n, shard_t(n), D),
                       "nnz": int(round(total_nnz)), "nodes": 2 * n, "D": D,
                       "parallelism": "single GPU" if world == 1 else
                       ("2 KG groups of %d GPUs, %d row blocks x %d feature-column slices "
                        "(aggregation only, no exchange)" % (shard.g, part.gr, part.gc) if free
                        else ("2 KG groups (one KG per GPU, nothing to exchange)" if shard.g == 1
                              else ("2 KG groups of %d GPUs, row blocks + per-column-slice halo "
                                    "exchange (relayed peer transfers) pipelined with the "
                                    "per-slice aggregation, inside the timed step" % shard.g)
                              if staged32 else
                              ("2 KG groups of %d GPUs, row blocks + the whole halo exchange "
                               "(relayed peer transfers), then the aggregation, inside the "
                               "timed step" % shard.g)))},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": pmc_bytes, "traffic_source": pmc_src,
                         "kernel": ("gnnea::k_spmm_sliced<1, 2, false, float, float>" if sliced else
                                    "gnnea::k_spmm_v4<relu,act,2>"),
                         "launches_per_step": launches,
                         "kernel_ms": round(kernel_ms / launches, 4),
                         "bytes_per_launch": int(traffic / launches),
                         "model": "gather: 4(N+1)+8E+4ED+4ND (rank 0 shard, D = its slice), "
                                  "split evenly over the per-KG launches",
                         "bound_detail": "gather rate: each 64-column slice of a KG is a 256 MB "
                                         "table, so most gathered bytes are Infinity-Cache "
                                         "(MALL) hits; the gather model counts them, HBM sees "
                                         "the compulsory bytes" if sliced else
                                         ("gather rate from HBM (row-major table >> the 256 MB "
                                          "Infinity Cache)" if shard.n_cols * Dl * 4 > 2 ** 28
                                          else "gather rate of an Infinity-Cache-resident table"),
                         "compulsory": {"bytes_per_step": int(comp),
                                        "achieved": round(comp_gbs, 1),
                                        "frac": round(comp_gbs / HBM_PEAK_GBS, 4),
                                        "model": "CSR 4(N+1)+8E once per slice pass (%d) + "
                                                 "table 4*N*%d once + Y 4*N*D once" %
                                                 ((Dl + 63) // 64 if sliced else 1,
                                                  ((Dl + 63) // 64) * 64 if sliced else Dl)}},
        }
        if pmc_extra:
            line["roofline"]["pmc"] = dict(pmc_extra, note="memory-side counters include "
                                           "Infinity-Cache hits (upper bound on HBM bytes)")
        if exchange is not None:
            line["exchange"] = exchange
        if halo_ab is not None:
            if exchange is not None:
                halo_ab["exchange_hidden_frac"] = exchange["exchange_hidden_frac"]
            line["halo_ab"] = halo_ab
        if side is not None:
            line["exchange_free_side"] = side
        line["config"]["layout"] = ("slice-major [%d][%d][64] fp32 (as gnnea_gemm_sliced_f32 "
                                    "writes the projection)" % ((Dl + 63) // 64, shard.n_cols)
                                    if sliced else "row-major [%d][%d] fp32" % (shard.n_cols, Dl))
        if world == 1 and not args.headline_only:
            try:
                line["layouts"] = layout_rates(shard, h_local, y, args.steps)
            except Exception as e:  # report, never hide
                line["layouts"] = {"error": repr(e)}
        for key, val in train.items():
            line[key] = val
        if sk_shard is not None:
            line["sinkhorn_B15000_row_sharded"] = sk_shard
        if world == 1 and not args.no_sinkhorn:
            try:
                line["sinkhorn"] = sinkhorn_rate(device)
            except Exception as e:  # report, never hide
                line["sinkhorn"] = {"error": repr(e)}
            try:
                line["sinkhorn_B15000"] = sinkhorn_large(device)
            except Exception as e:  # report, never hide
                line["sinkhorn_B15000"] = {"error": repr(e)}
            try:
                line["gw_cost"] = gw_rate(device)
            except Exception as e:  # report, never hide
                line["gw_cost"] = {"error": repr(e)}
            try:
                line["fgw_outer"] = fgw_rate(device)
            except Exception as e:  # report, never hide
                line["fgw_outer"] = {"error": repr(e)}
        if world == 1 and not args.no_train:
            # configs[1] / [2]'s DBP15K-scale EA iteration (with Adam) eager and as one captured
            # HIP graph (tools/graph_step.py; replay checked bit-identical to the eager step)
            try:
                from tools.graph_step import run as graph_run
                line["dbp15k_step_graph"] = {m: graph_run(m, synth.CONFIGS["dbp15k"]["n"],
                                                          synth.CONFIGS["dbp15k"]["t"], 30,
                                                          device) for m in ("GCN", "GAT")}
            except Exception as e:  # report, never hide
                line["dbp15k_step_graph"] = {"error": repr(e)}
        if world == 1 and not args.headline_only:
            try:
                line["hbm_anchors"] = anchors(device)
            except Exception as e:  # report, never hide
                line["hbm_anchors"] = {"error": repr(e)}
            try:
                del hs
                torch.cuda.empty_cache()
                line["bf16"] = bf16_rate(device, args.steps)
            except Exception as e:  # report, never hide
                line["bf16"] = {"error": repr(e)}
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(shard, h_local)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    # deterministic teardown: the package's cached buffers and torch's cached device / pinned
    # blocks go back to the runtime now, not from the C-level exit handlers
    del shard, h_local, y
    import gnnea
    gnnea.release()


def _dump_maps_at_exit(path):
    """Diagnostics (GNNEA_EXIT_MAPS=file): copy /proc/self/maps when the interpreter finalises, so
    the PCs of a crash in a C-level exit handler can be symbolised (tools/symbolize_crash.py)."""
    import atexit

    def dump():
        with open("/proc/self/maps") as src, open(path, "w") as dst:
            dst.write(src.read())
    atexit.register(dump)


if __name__ == "__main__":
    if os.environ.get("GNNEA_EXIT_MAPS"):
        _dump_maps_at_exit(os.environ["GNNEA_EXIT_MAPS"])
    main()
