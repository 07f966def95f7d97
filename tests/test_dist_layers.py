"""Row-sharded GCN / HighWay / GAT layers (gnnea.dist_graph.DistAdj) across ranks: forward rows,
input gradients and all-reduced weight gradients equal the single-process computation.

* CPU (gloo, world 2 / 4 / 8): the collective logic (halo all-gather, reduce-scatter of the
  transposed aggregation, row gather for the loss, one-bucket gradient all-reduce) with a CPU
  double of the kernel engine (fp64 torch sparse products) — the engine is the only stand-in.
* GPU (gloo rehearsal, world 2 / 4 on one MI355X, exchanges staged through host memory): the
  drop-in GraphConvolution + HighWayGraphConvolution (fused and composed) on the HIP kernels,
  handed a DistAdj,
  against the same layers on the whole adjacency in one process (fp32 tolerance 1e-4).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N_KG, T_KG, D = 48, 160, 12


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _mm(A, x):
    """A·x in x's dtype (the fp64 adjacency cast for bf16 storage: torch's CPU bf16 sparse mm)."""
    return torch.sparse.mm(A if A.dtype == x.dtype else A.to(x.dtype), x)


class CpuEngine:
    """fp64 torch double of gnnea.dist_graph.HipEngine (test stand-in, never shipped)."""

    def csr(self, r, c, v, n_rows, n_cols, device):
        idx = torch.from_numpy(np.stack([np.asarray(r, np.int64), np.asarray(c, np.int64)]))
        return torch.sparse_coo_tensor(idx, torch.from_numpy(np.asarray(v, np.float64)),
                                       (n_rows, n_cols)).coalesce()

    @staticmethod
    def _act(y, act):
        return torch.relu(y) if act == 1 else y

    def spmm(self, A, x, act, out=None, beta=0.0):
        y = _mm(A, x)
        if out is not None:
            y = y + beta * out
            out.copy_(self._act(y, act))
            return out
        return self._act(y, act)

    def spmm_t(self, A, x, out=None):
        y = _mm(A.t().coalesce(), x)
        if out is not None:
            out.copy_(y)
            return out
        return y

    def act_bwd(self, dy, y, act):
        return dy * (y > 0) if act == 1 else dy

    def act_spmm_t(self, A, dy, y, act):
        return self.spmm_t(A, self.act_bwd(dy, y, act))

    def highway_fwd(self, A, h, gate_pre, resid, bias, act):
        S = self._act(_mm(A, h), act)
        g = torch.sigmoid(gate_pre + bias if bias is not None else gate_pre)
        return g * S + (1 - g) * resid, S, g

    def highway_bwd(self, dy, S, g, resid, act, want):
        dS = dy * g * ((S > 0).to(dy.dtype) if act == 1 else 1.0)
        return dS, dy * (S - resid) * g * (1 - g), (dy * (1 - g) if want else None)

    # ---- column-slice stages (DistAdj's pipelined halo); W = 4 gives D = 12 three stages ----
    W = 4

    def slice_w(self, dtype):
        return self.W

    def pack_slices(self, x, tables, row0):
        S, _, W = tables.shape
        for q in range(S):
            c0, c1 = q * W, min(x.shape[1], (q + 1) * W)
            tables[q, row0:row0 + x.shape[0], :c1 - c0] = x[:, c0:c1]
        return tables

    def spmm_slice(self, A, table, w, act, out):
        out.copy_(self._act(_mm(A, table[:, :w].contiguous()), act))
        return out

    def spmm_t_slice(self, A, table, w):
        return _mm(A.t().coalesce(), table[:, :w].contiguous())

    def _slices(self, x):
        S = (x.shape[1] + self.W - 1) // self.W
        return self.pack_slices(x, torch.zeros((S, x.shape[0], self.W), dtype=x.dtype), 0)

    def act_bwd_slices(self, dy, y, act):
        return self._slices(self.act_bwd(dy, y, act))

    def highway_slice(self, A, table, w, gates, c0, bias, resid, out, S, G, act):
        sv = self._act(_mm(A, table[:, :w].contiguous()), act)
        gp = gates[c0 // self.W][:, :w]
        g = torch.sigmoid(gp + bias[c0:c0 + w] if bias is not None else gp)
        out[:, c0:c0 + w] = g * sv + (1 - g) * resid[:, c0:c0 + w]
        S[:, c0:c0 + w] = sv
        G[:, c0:c0 + w] = g
        return out

    def highway_bwd_slices(self, dy, S, g, resid, act, want, dgate):
        dS, dg, dres = self.highway_bwd(dy, S, g, resid, act, want)
        dgate.copy_(dg)
        return self._slices(dS), dres

    @staticmethod
    def gat_dense(A, H, a, heads, dh, alpha, act, row0):
        """layers/att_layers.py:29-61 per head over A's edges (destination i = row0 + row)."""
        i, j = A.indices()
        n = A.shape[0]
        outs = []
        for h in range(heads):
            Hh = H[:, h * dh:(h + 1) * dh]
            z = Hh[row0 + i] @ a[h, :dh] + Hh[j] @ a[h, dh:]
            e = torch.exp(-torch.nn.functional.leaky_relu(z, alpha))
            den = torch.zeros(n, dtype=H.dtype).index_add(0, i, e)
            num = torch.zeros(n, dh, dtype=H.dtype).index_add(0, i, e[:, None] * Hh[j])
            outs.append(num / den[:, None])
        y = torch.cat(outs, 1)
        return torch.relu(y) if act == 1 else y

    # ---- staged GAT halo (DistAdj.gat_staged_*): the same stages in fp64 torch ----------
    GW = 8  # GAT slice width: D = 12 = slices of 8 + 4, slice 0 holds heads 0 and 1

    def gat_slice_w(self, dtype):
        return self.GW

    def gat_staged_ok(self, heads, d_head):
        return True

    def gat_pack(self, x, tables, row0):
        S, _, W = tables.shape
        for q in range(S):
            c0, c1 = q * W, min(x.shape[1], (q + 1) * W)
            tables[q, row0:row0 + x.shape[0], :c1 - c0] = x[:, c0:c1]
        return tables

    @staticmethod
    def _heads(H, heads, dh):
        return H.reshape(H.shape[0], heads, dh)

    def gat_scores(self, H, a, heads, dh):
        Hh = self._heads(H, heads, dh)
        return (Hh * a[:, :dh]).sum(-1), (Hh * a[:, dh:]).sum(-1)

    def gat_rowstats(self, A, s1, s2, heads, dh, alpha):
        i, j = A.indices()
        sc = -torch.nn.functional.leaky_relu(s1[i] + s2[j], alpha)
        m = torch.full((A.shape[0], heads), -float("inf"), dtype=s1.dtype)
        m = m.scatter_reduce(0, i[:, None].expand(-1, heads), sc, "amax")
        w = torch.exp(sc - m[i])
        den = torch.zeros((A.shape[0], heads), dtype=s1.dtype).index_add(0, i, w)
        return m, den, w

    def gat_fwd_slice(self, A, tables, q, s1, s2, stats, heads, dh, alpha, act, Y):
        _, den, w = stats
        i, j = A.indices()
        W = tables.shape[2]
        c0, c1 = q * W, min(heads * dh, (q + 1) * W)
        hc = torch.arange(c0, c1) // dh
        num = torch.zeros((A.shape[0], c1 - c0), dtype=Y.dtype).index_add(
            0, i, w[:, hc] * tables[q][j, :c1 - c0])
        y = num / den[:, hc]
        Y[:, c0:c1] = torch.relu(y) if act == 1 else y
        return Y

    def gat_bwd_prep(self, dY, Y, s1, stats, heads, dh, act):
        m, den, _ = stats
        G = dY * (Y > 0) if act == 1 else dY.clone()
        c = self._heads(G * Y, heads, dh).sum(-1)
        return self._slices_w(G, self.GW), (s1, m, den, c)

    def _slices_w(self, x, W):
        S = (x.shape[1] + W - 1) // W
        t = torch.zeros((S, x.shape[0], W), dtype=x.dtype)
        for q in range(S):
            c0, c1 = q * W, min(x.shape[1], (q + 1) * W)
            t[q, :, :c1 - c0] = x[:, c0:c1]
        return t

    def gat_bwd_buffers(self, AT, S, heads, n_src, dtype, device):
        return {"pd": torch.zeros((S, AT._nnz(), heads), dtype=dtype),
                "P": torch.zeros((S, n_src, self.GW), dtype=dtype)}

    def _alpha(self, AT, s2, rec, alpha):
        s1, m, den, _ = rec
        j, i = AT.indices()
        z = s1[i] + s2[j]
        return z, torch.exp(-torch.nn.functional.leaky_relu(z, alpha) - m[i]) / den[i]

    def gat_bwd_src_slice(self, AT, tables, q, s2, rec, Gs, bufs, heads, dh, alpha, weights):
        j, i = AT.indices()
        _, al = self._alpha(AT, s2, rec, alpha)
        W = tables.shape[2]
        c0, c1 = q * W, min(heads * dh, (q + 1) * W)
        hc = torch.arange(c0, c1) // dh
        G = Gs[q][i, :c1 - c0]
        Hj = tables[q][j, :c1 - c0]
        P = bufs["P"]
        P[q].zero_()
        P[q][:, :c1 - c0] = torch.zeros((AT.shape[0], c1 - c0), dtype=G.dtype).index_add(
            0, j, al[:, hc] * G)
        bufs["pd"][q] = torch.zeros((AT._nnz(), heads), dtype=G.dtype).index_add(
            1, hc, G * Hj)
        return P[q]

    def gat_bwd_edge(self, AT, s2, rec, bufs, a, heads, dh, alpha):
        j, i = AT.indices()
        z, al = self._alpha(AT, s2, rec, alpha)
        da = bufs["pd"].sum(0)
        dz = -(al * (da - rec[3][i])) * torch.where(z > 0, z.new_tensor(1.0), z.new_tensor(alpha))
        ds2 = torch.zeros((AT.shape[0], heads), dtype=dz.dtype).index_add(0, j, dz)
        return dz, ds2

    def gat_bwd_dst(self, A, dzT, a, ds2, dH, heads, dh):
        AT = A.t().coalesce()
        ds1 = torch.zeros((A.shape[0], heads), dtype=dzT.dtype).index_add(0, AT.indices()[1],
                                                                           dzT)
        upd = ds1[:, :, None] * a[None, :, :dh] + ds2[:, :, None] * a[None, :, dh:]
        dH += upd.reshape(dH.shape)
        return ds1

    def gat_da(self, H, ds, heads, dh):
        return (ds[:, :, None] * self._heads(H, heads, dh)).sum(0).reshape(-1)

    def transpose(self, A):
        return A.t().coalesce()

    def unpack64(self, Ts, D):
        S, n, W = Ts.shape
        return Ts.permute(1, 0, 2).reshape(n, S * W)[:, :D]

    def gat_fwd(self, A, H, a_all, heads, dh, alpha, act, row0):
        Hd = H.detach().clone().requires_grad_(True)
        ad = a_all.detach().clone().requires_grad_(True)
        with torch.enable_grad():
            y = self.gat_dense(A, Hd, ad, heads, dh, alpha, act, row0)
        return y.detach(), (Hd, ad, y)

    def gat_bwd(self, A, saved, dY, heads, dh, alpha, act, row0, need_da):
        Hd, ad, y = saved
        gH, ga = torch.autograd.grad(y, (Hd, ad), dY)
        return gH, (ga if need_da else None)


class CpuLossEngine:
    """fp64 torch double of gnnea.dist_loss.HipLossEngine (test stand-in, never shipped)."""

    def l1_terms(self, X, a, b):
        return (X[a] - X[b]).abs().sum(1).double()

    def margin_grad(self, X, idx, m, t, k, g):
        left, right, nl1, nr1, nl2, nr2 = idx
        a, b = torch.cat([nl1, nl2, left]), torch.cat([nr1, nr2, right])
        s = torch.sign(X[a] - X[b])
        coef = (m.to(X.dtype) * g.to(X.dtype) / (2.0 * t * k))[:, None]
        grad = torch.zeros_like(X)
        grad.index_add_(0, a, coef * s)
        grad.index_add_(0, b, -coef * s)
        return grad


def _ref_margin(out, left, right, nl1, nr1, nl2, nr2, t, k):
    """models/models_ea.py:103-123 on the whole embedding (torch ops)."""
    A = (out[left] - out[right]).abs().sum(1)
    B1 = (out[nl1] - out[nr1]).abs().sum(1).view(t, k)
    B2 = (out[nl2] - out[nr2]).abs().sum(1).view(t, k)
    D_ = (A + 1.0).view(t, 1)
    return (torch.relu(D_ - B1).sum() + torch.relu(D_ - B2).sum()) / (2.0 * t * k)


def _loss_indices(n_kg, t=10, k=5):
    rng = np.random.default_rng(3)
    left = rng.choice(n_kg, t, replace=False)
    right = n_kg + rng.choice(n_kg, t, replace=False)
    nl1 = np.repeat(left, k)
    nr1 = rng.integers(0, 2 * n_kg, t * k)
    nl2 = rng.integers(0, 2 * n_kg, t * k)
    nr2 = np.repeat(right, k)
    return [left, right, nl1, nr1, nl2, nr2], t, k


def _worker(rank, world, port, mode, q, staged=True):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "gnn-mtl_amd"))
    sys.path.insert(0, root)
    import torch.nn.functional as F
    from gnnea import exchange, synth
    exchange.STAGED = staged  # GNNEA_HALO_STAGED: per-slice pipeline or the whole halo at once
    from gnnea.dist_graph import DistAdj, allreduce_grads
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr = synth.kg_pair_triples(N_KG, T_KG, 20)
        R, C, V = synth.adjacency_coo(tr, 2 * N_KG, reference_order=False)
        # the HIP rehearsal uses 132 columns: three 64-column slices of the pipelined halo
        D = 132 if mode == "gpu" else globals()["D"]
        X = torch.from_numpy(synth.features(2 * N_KG, D, seed=5)).double()
        Rw = torch.from_numpy(np.random.default_rng(9).standard_normal((2 * N_KG, D)))
        HEADS, DH = 3, D // 3
        if mode in ("gat_cpu", "gat_cpu_bf16"):
            # gat_cpu_bf16: every tensor the DistAdj moves (H halo, slice tables, dH partials,
            # parameter gradients) in bf16 through gloo; the engine double computes in torch's
            # CPU bf16 arithmetic, so the bar is the bf16 one
            dt = torch.bfloat16 if mode == "gat_cpu_bf16" else torch.float64
            dev = torch.device("cpu")
            dadj = DistAdj.from_triples(tr, N_KG, T_KG, rank, world, dev, engine=CpuEngine())
            torch.manual_seed(0)
            X, Rw = X.to(dt), Rw.to(dt)
            Wg = (torch.randn(D, D, dtype=torch.float64) * 0.3).to(dt)
            a_all = (torch.randn(HEADS, 2 * DH, dtype=torch.float64) * 0.3).to(dt)
            W2 = (torch.randn(D, D, dtype=torch.float64) / D ** 0.5).to(dt)
            params = [p.requires_grad_() for p in (Wg, a_all, W2)]

            def model(x, adj):
                if adj is None:
                    A = CpuEngine().csr(R, C, V, 2 * N_KG, 2 * N_KG, None)
                    y = CpuEngine.gat_dense(A, x @ Wg, a_all, HEADS, DH, 0.2, 1, 0)
                    return CpuEngine.gat_dense(A, y @ W2, a_all, HEADS, DH, 0.2, 0, 0)
                y = adj.gat(x @ Wg, a_all, HEADS, DH, 0.2, F.relu)
                return adj.gather_rows(adj.gat(y @ W2, a_all, HEADS, DH, 0.2, None))
            tol = 5e-2 if dt == torch.bfloat16 else 1e-12
        elif mode in ("gat_gpu", "gat_gpu_bf16"):
            # gat_gpu_bf16: configs[4]'s storage dtype -- the bf16 projection, the bf16 halo and
            # (staged) the bf16 64-column GAT slice tables / dH partials, against the same bf16
            # layers on the whole adjacency in one process (the row-major bf16 passes)
            from layers.att_layers import GraphAttentionLayer
            dt = torch.bfloat16 if mode == "gat_gpu_bf16" else torch.float32
            dev = torch.device("cuda:0")
            torch.cuda.set_device(dev)
            X, Rw = X.to(device=dev, dtype=dt), Rw.float().to(dev)
            dadj = DistAdj.from_triples(tr, N_KG, T_KG, rank, world, dev)
            torch.manual_seed(0)
            g1 = GraphAttentionLayer(D, DH, 0.0, F.relu, 0.2, HEADS, True).to(dev, dt)
            g2 = GraphAttentionLayer(D, DH, 0.0, F.elu, 0.2, HEADS, True).to(dev, dt)  # torch act
            params = list(g1.parameters()) + list(g2.parameters())
            adj_full = torch.sparse_coo_tensor(torch.from_numpy(np.stack([R, C])).long(),
                                               torch.from_numpy(V), (2 * N_KG, 2 * N_KG)).to(dev)

            def model(x, adj):
                if adj is None:
                    return g2(g1((x, adj_full)))[0]
                return adj.gather_rows(g2(g1((x, adj)))[0])
            # bf16: the storage tolerance of tests/test_gpu_scale_cfg5.py on gradients (2e-2)
            tol = 2e-2 if dt == torch.bfloat16 else 1e-4
        elif mode == "loss_cpu":
            # the column-sharded EA margin loss (gnnea.dist_loss) on a GCN + HighWay shard
            # against the reference loss on the whole graph's output
            from gnnea.dist_loss import sharded_margin_loss
            dev = torch.device("cpu")
            dadj = DistAdj.from_triples(tr, N_KG, T_KG, rank, world, dev, engine=CpuEngine())
            torch.manual_seed(0)
            W1, b1 = torch.randn(D, D, dtype=torch.float64), torch.randn(D, dtype=torch.float64)
            Kg = torch.randn(D, D, dtype=torch.float64)
            params = [p.requires_grad_() for p in (W1, b1, Kg)]
            idx, t_, k_ = _loss_indices(N_KG)

            def model(x, adj):
                h1 = x @ W1.t() + b1
                if adj is None:
                    A = torch.sparse_coo_tensor(torch.from_numpy(np.stack([R, C])).long(),
                                                torch.from_numpy(V).double(),
                                                (2 * N_KG, 2 * N_KG))
                    y1 = torch.relu(torch.sparse.mm(A, h1))
                    g = torch.sigmoid(y1 @ Kg)
                    y2 = g * torch.relu(torch.sparse.mm(A, y1 @ W1.t())) + (1 - g) * y1
                    ti = [torch.from_numpy(np.asarray(a)) for a in idx]
                    return _ref_margin(y2, *ti, t_, k_)
                y1 = adj.aggregate(h1, F.relu)
                y2 = adj.highway(y1 @ W1.t(), y1 @ Kg, y1, None, F.relu)
                return sharded_margin_loss(y2, adj, *idx, t_, k_, engine=CpuLossEngine())
            tol = 1e-12
        elif mode == "loss_gpu":
            # the column-sharded loss on the HIP kernels (gnnea_l1_terms_f32, the multiplier
            # backward) against the gathered loss of the single-GPU kernels (gnnea.margin)
            from layers.layers import GraphConvolution
            from gnnea.dist_loss import sharded_margin_loss
            from gnnea.margin import margin_loss
            dev = torch.device("cuda:0")
            torch.cuda.set_device(dev)
            X = X.float().to(dev)
            dadj = DistAdj.from_triples(tr, N_KG, T_KG, rank, world, dev)
            torch.manual_seed(0)
            l1 = GraphConvolution(D, D, 0.0, F.relu, True).to(dev)
            params = list(l1.parameters())
            adj_full = torch.sparse_coo_tensor(torch.from_numpy(np.stack([R, C])).long(),
                                               torch.from_numpy(V), (2 * N_KG, 2 * N_KG)).to(dev)
            idx, t_, k_ = _loss_indices(N_KG)

            def model(x, adj):
                if adj is None:
                    return margin_loss(l1((x, adj_full))[0], *idx, t_, k_)
                return sharded_margin_loss(l1((x, adj))[0], adj, *idx, t_, k_)
            tol = 1e-5
        elif mode == "gpu_bf16":
            # bf16 storage through the DistAdj hooks: the aggregation and the fused HighWay
            # tail (HaloHighwayFn; staged: the 128-column bf16 slice tables, a partial last
            # slice at D = 132) against an fp32 torch restatement on the whole graph
            dev = torch.device("cuda:0")
            torch.cuda.set_device(dev)
            X, Rw = X.bfloat16().to(dev), Rw.float().to(dev)
            dadj = DistAdj.from_triples(tr, N_KG, T_KG, rank, world, dev)
            torch.manual_seed(0)
            W1 = (torch.randn(D, D) / D ** 0.5).bfloat16().to(dev)
            Kg = (torch.randn(D, D) / D ** 0.5).bfloat16().to(dev)
            bg = (0.1 * torch.randn(D)).to(dev)
            params = [p.requires_grad_() for p in (W1, Kg)]
            A = torch.sparse_coo_tensor(torch.from_numpy(np.stack([R, C])).long(),
                                        torch.from_numpy(V).float(), (2 * N_KG, 2 * N_KG)).to(dev)

            def model(x, adj):
                if adj is None:
                    xf, Wf, Kf = x.float(), W1.float(), Kg.float()
                    y1 = torch.relu(torch.sparse.mm(A, xf @ Wf.t()))
                    g = torch.sigmoid(y1 @ Kf + bg)
                    return g * torch.relu(torch.sparse.mm(A, y1 @ Wf.t())) + (1 - g) * y1
                y1 = adj.aggregate(x @ W1.t(), F.relu)
                y2 = adj.highway(y1 @ W1.t(), y1 @ Kg, y1, bg, F.relu)
                return adj.gather_rows(y2)
            tol = 5e-2
        elif mode == "cpu":
            dev = torch.device("cpu")
            dadj = DistAdj.from_triples(tr, N_KG, T_KG, rank, world, dev, engine=CpuEngine())
            torch.manual_seed(0)
            W1, b1 = torch.randn(D, D, dtype=torch.float64), torch.randn(D, dtype=torch.float64)
            W2, b2 = torch.randn(D, D, dtype=torch.float64), torch.randn(D, dtype=torch.float64)
            Kg = torch.randn(D, D, dtype=torch.float64)
            params = [p.requires_grad_() for p in (W1, b1, W2, b2)]

            bg = torch.randn(D, dtype=torch.float64) * 0.1

            def model(x, adj):
                h1 = x @ W1.t() + b1
                if adj is None:
                    A = torch.sparse_coo_tensor(torch.from_numpy(np.stack([R, C])).long(),
                                                torch.from_numpy(V).double(),
                                                (2 * N_KG, 2 * N_KG))
                    y1 = torch.relu(torch.sparse.mm(A, h1))
                    h2 = y1 @ W2.t() + b2
                    g = torch.sigmoid(y1 @ Kg)
                    y2 = g * torch.sparse.mm(A, h2) + (1 - g) * y1
                    g3 = torch.sigmoid(y2 @ Kg + bg)
                    return g3 * torch.relu(torch.sparse.mm(A, y2 @ W1.t())) + (1 - g3) * y2
                y1 = adj.aggregate(h1, F.relu)
                h2 = y1 @ W2.t() + b2
                y2 = adj.highway(h2, y1 @ Kg, y1, torch.zeros(D, dtype=torch.float64),
                                 lambda t: t)  # composed: aggregate + torch blend
                # fusable act: HaloHighwayFn (the staged HighWay tail slice by slice)
                return adj.gather_rows(adj.highway(y2 @ W1.t(), y2 @ Kg, y2, bg, F.relu))
            tol = 1e-12
        else:
            from layers.layers import GraphConvolution, HighWayGraphConvolution
            dev = torch.device("cuda:0")
            torch.cuda.set_device(dev)
            X, Rw = X.float().to(dev), Rw.float().to(dev)
            dadj = DistAdj.from_triples(tr, N_KG, T_KG, rank, world, dev)
            torch.manual_seed(0)
            l1 = GraphConvolution(D, D, 0.0, F.relu, True).to(dev)
            # l2: fused HighWay layer (HighwayLayerFn through the DistAdj hooks); l3: an act the
            # kernels cannot fuse, so the composed path (DistAdj.aggregate + torch blend)
            l2 = HighWayGraphConvolution(D, D, 0.0, torch.tanh, True, 0, dev).to(dev)
            l3 = HighWayGraphConvolution(D, D, 0.0, lambda t: t * 0.5, True, 0, dev).to(dev)
            params = list(l1.parameters()) + list(l2.parameters()) + list(l3.parameters())
            adj_full = torch.sparse_coo_tensor(torch.from_numpy(np.stack([R, C])).long(),
                                               torch.from_numpy(V), (2 * N_KG, 2 * N_KG)).to(dev)

            def model(x, adj):
                if adj is None:
                    return l3(l2(l1((x, adj_full))))[0]
                return adj.gather_rows(l3(l2(l1((x, adj))))[0])
            tol = 1e-4

        # single process, whole graph
        xr = X.clone().requires_grad_()
        out_ref = model(xr, None)
        (out_ref if out_ref.dim() == 0 else (out_ref * Rw).sum()).backward()
        g_ref = [p.grad.clone() for p in params]
        for p in params:
            p.grad = None
        # sharded
        p0 = dadj.part.global_row0
        xl = X[p0:p0 + dadj.part.n_rows].clone().requires_grad_()
        out = model(xl, dadj)
        (out if out.dim() == 0 else (out * Rw).sum()).backward()
        allreduce_grads(params)

        def rel(a, b):
            a, b = a.detach().double().cpu(), b.detach().double().cpu()
            return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))
        errs = [rel(out, out_ref), rel(xl.grad, xr.grad[p0:p0 + dadj.part.n_rows])]
        errs += [rel(p.grad, g) for p, g in zip(params, g_ref)]
        q.put((rank, max(errs), tol))
    finally:
        dist.destroy_process_group()


def _run(world, mode, staged=True):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q, staged))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [q.get(timeout=5) for _ in range(world)]
    for rank, err, tol in res:
        assert err < tol, (rank, err)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dist_layers_gloo_cpu(world):
    _run(world, "cpu")


@pytest.mark.parametrize("world", [4, 8])
def test_dist_layers_gloo_cpu_unstaged(world):
    """GNNEA_HALO_STAGED=0: the whole halo, one aggregation, one blocking reduce-scatter."""
    _run(world, "cpu", staged=False)


@pytest.mark.gpu
@pytest.mark.parametrize("world,staged", [(2, True), (4, True), (4, False)])
def test_dist_layers_rehearsal_on_device(device, world, staged):
    _run(world, "gpu", staged)


@pytest.mark.gpu
@pytest.mark.parametrize("staged", [True, False])
def test_dist_layers_bf16_rehearsal_on_device(device, staged):
    """bf16 storage on the HIP engine, world 4 (two ranks per KG): the staged halo carries the
    HighWay tail on the 128-column bf16 slice tables (gnnea_spmm_highway_bf16 per slice,
    gnnea_highway_bwd_ld_bf16 per slice into the dS tables), and without staging the whole
    halo; both against an fp32 restatement at bf16 tolerance (5e-2 of the max)."""
    _run(4, "gpu_bf16", staged)


class BrokenStagedEngine(CpuEngine):
    """A staged pipeline that is wrong in one slice (test stand-in): validate_staged must see
    the mismatch and leave the halo unstaged."""

    def spmm_slice(self, A, table, w, act, out):
        super().spmm_slice(A, table, w, act, out)
        out.mul_(1.25)  # (wrong by more than the bf16 bar too)
        return out


def _ab_worker(rank, world, port, broken, q, env="auto"):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "gnn-mtl_amd"))
    from gnnea import exchange, synth
    from gnnea.dist_graph import DistAdj, validate_staged
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        exchange.STAGED_ENV = env
        exchange.STAGED = env == "1"
        exchange.STAGED_DTYPES = None
        tr = synth.kg_pair_triples(N_KG, T_KG, 20)
        eng = BrokenStagedEngine() if broken else CpuEngine()
        dadj = DistAdj.from_triples(tr, N_KG, T_KG, rank, world, torch.device("cpu"), engine=eng)
        # fp64 (the engine double's exact arithmetic) and bf16 (configs[4]'s storage; the
        # double computes in CPU bf16 arithmetic, hence the looser bar)
        rep = validate_staged(dadj, D=D, heads=3, reps=2, tol=1e-12, tol_bf16=5e-2,
                              dtypes=(torch.float64, torch.bfloat16))
        q.put((rank, {k: (v["match"], v["max_norm_rel_err"], sorted(v["legs"]))
                      for k, v in rep["dtypes"].items()}, rep["match"],
               [exchange.staged_for(t) for t in (torch.float64, torch.bfloat16, torch.float32)],
               rep["staged_in_use"]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,broken,env", [(4, False, "auto"), (4, True, "auto"),
                                              (8, False, "auto"), (4, True, "1"),
                                              (4, False, "0")])
def test_validate_staged_gloo_cpu(world, broken, env):
    """gnnea.dist_graph.validate_staged (the N > 1 bench's halo_ab): staged and unstaged HighWay,
    GCN and GAT layers on the same inputs, in fp64 and in bf16; a correct pipeline matches in
    both and is switched on for exactly those dtypes (fp32, never validated here, stays
    unstaged), a pipeline wrong in one slice is caught on every rank and the halo stays
    unstaged.  GNNEA_HALO_STAGED=1 keeps the staged path on whatever validation says (the report
    still records the mismatch); =0 keeps it off."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ab_worker, args=(r, world, port, broken, q, env))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [q.get(timeout=5) for _ in range(world)]
    for rank, per, match, staged_for, in_use in res:
        assert sorted(per) == ["bfloat16", "float64"]
        for name, (m, err, legs) in per.items():
            assert legs == ["gat", "gcn", "highway"]
            assert m is (not broken), (rank, name, err)
            if broken:
                assert err > 1e-4
            else:
                assert err <= (1e-12 if name == "float64" else 5e-2), (name, err)
        assert match is (not broken)
        if env == "1":
            want = [True, True, True]
        elif env == "0" or broken:
            want = [False, False, False]
        else:
            want = [True, True, False]
        assert staged_for == want, (rank, staged_for)
        assert in_use == {"float64": want[0], "bfloat16": want[1]}


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dist_margin_loss_gloo_cpu(world):
    """Column-sharded EA margin loss (gnnea.dist_loss: all-to-all to column blocks, one
    all-reduce of the per-term partial distances, reverse all-to-all of the gradient): loss,
    input and parameter gradients equal the reference loss on the whole graph's output."""
    _run(world, "loss_cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_dist_margin_loss_rehearsal_on_device(device, world):
    _run(world, "loss_gpu")


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dist_gat_gloo_cpu(world):
    """Row-sharded GAT (DistAdj.gat / HaloGATFn): at world >= 4 the staged halo (s2 of every
    KG row first, 64-column slices of H exchanged and aggregated one after another, the
    backward's per-slice dH partials reduce-scattered as each is computed, ds2 reduce-scattered,
    da from the own rows), at world 2 nothing to exchange; da partials summed by
    allreduce_grads."""
    _run(world, "gat_cpu")


@pytest.mark.parametrize("world", [4, 8])
def test_dist_gat_gloo_cpu_unstaged(world):
    """GNNEA_HALO_STAGED=0: the whole H halo, one aggregation, one blocking reduce-scatter."""
    _run(world, "gat_cpu", staged=False)


@pytest.mark.parametrize("world,staged", [(2, True), (4, True), (4, False), (8, True)])
def test_dist_gat_bf16_gloo_cpu(world, staged):
    """configs[4]'s storage dtype through the row-sharded GAT: the bf16 H halo, slice tables,
    dH partials and ds2 sums move through the same exchange schedule (gloo), the bf16 parameter
    gradients through allreduce_grads; against the single-process bf16 computation."""
    _run(world, "gat_cpu_bf16", staged)


@pytest.mark.gpu
@pytest.mark.parametrize("world,staged", [(2, True), (4, True), (4, False)])
def test_dist_gat_bf16_rehearsal_on_device(device, world, staged):
    """The drop-in GraphAttentionLayer in bf16 (configs[4]) handed a DistAdj on the HIP kernels:
    world 4 staged runs gnnea_gat_fwd_sliced_range_bf16 / gnnea_gat_bwd_src_sliced_range_bf16
    over the exchanged bf16 64-column tables, unstaged the row-major bf16 passes over the whole
    halo; against the same bf16 layers on the whole adjacency (2e-2 norm-relative)."""
    _run(world, "gat_gpu_bf16", staged)


@pytest.mark.gpu
@pytest.mark.parametrize("world,staged", [(2, True), (4, True), (4, False)])
def test_dist_gat_rehearsal_on_device(device, world, staged):
    """The drop-in GraphAttentionLayer handed a DistAdj, on the HIP GAT kernels (row offset of
    the shard's logits and dH), against the same layers on the whole adjacency; world 4 with the
    staged halo (gnnea_gat_fwd_sliced_range / gnnea_gat_bwd_src_sliced_range) and without."""
    _run(world, "gat_gpu", staged)
