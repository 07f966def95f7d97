"""Row-sharded adjacency that the drop-in GCN / HighWay layers accept in place of ``adj``
(node-sharded HGCN-EA across the GPUs of one node with the halo all-gather).

One process per GPU.  The two-KG adjacency is block-diagonal, so ranks [0, W/2) serve KG1 and
[W/2, W) serve KG2 (gnnea.dist.Partition, kind "rows"); inside a KG group of g ranks, rank l
owns the n/g destination rows [l·n/g, (l+1)·n/g) of its KG, and the layers run on those rows
only.  Per graph layer (layers/layers.py:30-39, 58-77):

  forward   hidden_loc = x_loc·Wᵀ + b                local MFMA GEMM (unchanged drop-in code)
            hidden_KG  = all_gather(hidden_loc)       peer transfers inside the KG group, overlapped
            out_loc    = act(A_own·hidden_loc           with the SpMM over the owned columns
                             + A_remote·hidden_KG)
  backward  G_loc      = dY_loc ⊙ act'(out_loc)
            P          = A_shardᵀ · G_loc             [n, D]: this rank's share of every row
            dhidden_loc= reduce_scatter(P)            peer transfers, summed by the owner
            dW, db     = local GEMMs; summed over ALL ranks by allreduce_grads() (one bucket)

Overlap (§8e): the halo exchange and the aggregation are cut into column slices of the
feature table (the slice-major layout's 64-column fp32 / 128-column bf16 slices; one KG slice of
cfg-4 is 256 MB).  The own rows are packed into the KG's [S][n][W] table, every slice's exchange
is issued at once (gnnea.exchange.all_gather_slices), and slice q is aggregated over the whole
shard CSR (KG-local columns, Infinity-Cache-sized table) as soon as it has landed, while the
later slices are in flight.  Backward mirrors it: Aᵀ·G of slice q is computed and its
reduce-scatter issued at once (exchange.reduce_scatter_start), the next slice computing while
it moves; the owners sum once every slice has arrived.

The HighWay gate (x_loc·K_g, the blend with x_loc) is row-local.  ``gather_rows`` assembles the
final embeddings of both KGs on every rank (all_gather over the world) for the EA loss, which
every rank then evaluates identically; its backward keeps the rank's own rows of the gradient.

The engine (the SpMM / elementwise kernels) is the HIP library; tests substitute a CPU double
only to check the collective logic with gloo (tests/test_dist_gloo.py).  gloo cannot move
device tensors: under gloo the exchanges are staged through host memory (the 1-GPU rehearsal).
"""
import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from .dist import Partition, make_groups, shard_coo


class HipEngine:
    """The product engine: libgnnea kernels through gnnea.ops (device tensors only)."""

    def csr(self, r, c, v, n_rows, n_cols, device):
        from .graph import DeviceCSR
        return DeviceCSR.from_coo(torch.from_numpy(np.ascontiguousarray(r, np.int32)).to(device),
                                  torch.from_numpy(np.ascontiguousarray(c, np.int32)).to(device),
                                  torch.from_numpy(np.ascontiguousarray(v, np.float32)).to(device),
                                  n_rows, n_cols)

    def spmm(self, csr, x, act, out=None, beta=0.0):
        from . import ops
        if beta == 0.0 and ops.use_sliced(csr.n_cols, x.shape[1], x.dtype) and \
                (out is None or x.dtype == torch.bfloat16 or out.dtype == torch.float32):
            # above the Infinity Cache: pack into 64-column slices, aggregate slice by slice
            return ops.spmm_sliced(csr, ops.slice_pack(x), x.shape[1], act, out=out)
        return ops.spmm(csr, x, act, out=out, beta=beta)

    def spmm_t(self, csr, x, out=None):
        return self.spmm(csr.transpose(), x, _lib.GNNEA_ACT_IDENTITY, out=out)

    def act_spmm_t(self, csr, dy, y, act):
        """Aᵀ·(dy ⊙ act'(y)) (the aggregation's backward; slice-major above the cache)."""
        from . import ops
        return ops.aggregate_t_into(csr, dy.contiguous(), y, act)

    def act_bwd(self, dy, y, act):
        from . import ops
        return ops.act_bwd(dy, y, act)

    def highway_fwd(self, csr, hidden, gate_pre, resid, bias_gate, act):
        from . import ops
        return ops.highway_fwd(csr, hidden, gate_pre, resid, bias_gate, act)

    def highway_bwd(self, dy, S, G, resid, act, want_dresid):
        from . import ops
        return ops.highway_bwd(dy, S, G, resid, act, want_dresid)

    def gat_fwd(self, csr, H, a_all, heads, d_head, alpha, act, row0):
        """All-head GAT aggregation of the shard's rows over the KG's H rows; returns
        (Y_loc [n_rows, heads*d_head], saved state for gat_bwd)."""
        from . import ops
        D = heads * d_head
        Hp = ops._pad4(H, D)
        a32 = ops._featc(a_all, torch.float32)
        Y, m, den, s1, s2 = ops.gat_forward(csr, Hp, a32, heads, d_head, alpha, act, row0=row0)
        return (Y if Y.shape[1] == D else Y[:, :D]), (Hp, a32, s1, s2, m, den, Y)

    # ---- column-slice stages (the pipelined halo of DistAdj) ---------------------------
    def slice_w(self, dtype):
        """Columns per exchange / aggregation stage: one slice of the slice-major table (256 B
        of row: 64 fp32 / 128 bf16 columns; one KG slice of cfg-4 is 256 MB)."""
        from . import ops
        return ops.slice_w(dtype)

    def pack_slices(self, x, tables, row0):
        """tables[q, row0:row0+rows, :w_q] = x[:, q-th column block] (one pass)."""
        from . import ops
        x = ops._rows(x)
        S, n, W = tables.shape
        with _lib.on_device(x.device):
            _lib.check(ops._sfn("gnnea_slice_pack", x.dtype)(
                _lib.ptr(x), ops._ld(x), x.shape[0], x.shape[1],
                ops._off(tables[0], row0), n * W, _lib.stream_of(x.device)))
        return tables

    def spmm_slice(self, csr, table, w, act, out):
        """out (a [rows, w] column block) = act(A · table[:, :w]) over one slice table."""
        from . import ops
        return ops.spmm_sliced(csr, table.unsqueeze(0), w, act, out=out)

    def spmm_t_slice(self, csr, table, w):
        """Aᵀ · table[:, :w] ([csr.n_cols, w]) over one slice table of the shard's rows."""
        from . import ops
        return ops.spmm_sliced(csr.transpose(), table.unsqueeze(0), w)

    def act_bwd_slices(self, dy, y, act):
        """dy ⊙ act'(y) written slice-major ([S][rows][W])."""
        from . import ops
        return ops.act_bwd_sliced(dy, y, act)

    def highway_slice(self, csr, table, w, gates, c0, bias_gate, resid, out, S, G, act):
        """Columns [c0, c0+w) of the HighWay tail (layers/layers.py:64-76) from one slice
        table of the hidden rows: gate_pre from the shard's own slice-major gate table."""
        from . import ops
        L = _lib.lib()
        if table.dtype == torch.bfloat16:
            # a bf16 slice table [n, 128] is a row-major matrix of w columns (ld 128), and so
            # is the shard's own gate slice: the row-major HighWay kernel over the column block
            W = table.shape[1]
            gq = gates[c0 // W]
            with _lib.on_device(table.device):
                for r0, r1 in csr.row_blocks():
                    _lib.check(L.gnnea_spmm_highway_bf16(
                        ops._off32(csr.rowptr, r0), _lib.ptr(csr.col), _lib.ptr(csr.val),
                        r1 - r0, w, _lib.ptr(table), W, ops._off(gq, r0), W,
                        None if bias_gate is None else
                        ops._off(ops._featc(bias_gate, torch.float32).view(1, -1), 0, c0),
                        ops._off(resid, r0, c0), resid.stride(0), ops._off(out, r0, c0),
                        out.stride(0), ops._off(S, r0, c0), ops._off(G, r0, c0), S.stride(0),
                        int(act), _lib.stream_of(table.device)))
            return out
        with _lib.on_device(table.device):
            for r0, r1 in csr.row_blocks():
                _lib.check(L.gnnea_spmm_highway_sliced_f32(
                    ops._off32(csr.rowptr, r0), _lib.ptr(csr.col), _lib.ptr(csr.val), r1 - r0, w,
                    _lib.ptr(table), table.numel(), ops._off(gates[0], r0), gates.stride(0), c0,
                    None if bias_gate is None else ops._off(bias_gate.view(1, -1), 0, c0),
                    ops._off(resid, r0, c0), resid.stride(0), ops._off(out, r0, c0),
                    out.stride(0), ops._off(S, r0, c0), ops._off(G, r0, c0), S.stride(0),
                    int(act), _lib.stream_of(table.device)))
        return out

    def highway_bwd_slices(self, dy, S, G, resid, act, want_dresid, dgate):
        """(dS slice-major, dresid): dS = dy·g·act'(S), dgate written into ``dgate``."""
        from . import ops
        if S.dtype != torch.bfloat16:
            return ops.highway_bwd_sliced(dy, S, G, resid, act, want_dresid, dgate)
        # bf16: each 128-column slice table of dS is a row-major [rows, 128] matrix, written
        # by the row-major elementwise backward over the slice's column block
        S = ops._featc(S)
        dy, G, resid = (ops._featc(t, S.dtype) for t in (dy, G, resid))
        N, D = S.shape
        dSs = ops.sliced_empty(N, D, S.device, S.dtype)
        W = dSs.shape[2]
        dres = torch.empty_like(S) if want_dresid else None
        L = _lib.lib()
        with _lib.on_device(S.device):
            for q in range(dSs.shape[0]):
                c0 = q * W
                _lib.check(L.gnnea_highway_bwd_ld_bf16(
                    ops._off(dy, 0, c0), ops._off(S, 0, c0), ops._off(G, 0, c0),
                    ops._off(resid, 0, c0), S.stride(0), N, min(W, D - c0), _lib.ptr(dSs[q]), W,
                    ops._off(dgate, 0, c0), ops._ld(dgate),
                    ops._off(dres, 0, c0), D, int(act), _lib.stream_of(S.device)))
        return dSs, dres

    # ---- the staged GAT halo (64-column slices of the head-concatenated projection) -------
    def gat_slice_w(self, dtype):
        """Columns per GAT stage: the sliced GAT kernels' 64-column tables (256 B fp32, 128 B
        bf16 per row piece)."""
        return 64

    def gat_staged_ok(self, heads, d_head):
        from . import ops
        D = heads * d_head
        return ops.gat_two_heads_per_slice(heads, d_head) and D % 4 == 0 and heads <= 8 and \
            D <= 1024

    def gat_pack(self, x, tables, row0):
        """tables[q, row0:row0+rows, :] = x's q-th 64-column block (the GAT tables)."""
        from . import ops
        x = ops._rows(x)
        S, n, W = tables.shape
        with _lib.on_device(x.device):
            _lib.check(ops._sfn("gnnea_slice_pack64", x.dtype)(
                _lib.ptr(x), ops._ld(x), x.shape[0], x.shape[1], ops._off(tables[0], row0),
                n * W, _lib.stream_of(x.device)))
        return tables

    def gat_scores(self, H, a_all, heads, d_head):
        """Per-row logits (s1, s2) [rows, heads] of the rank's own projected rows."""
        from . import ops
        return ops.gat_scores(H, ops._featc(a_all, torch.float32), heads, d_head)

    def gat_rowstats(self, csr, s1, s2, heads, d_head, alpha):
        """Row max / denominator of the shard's rows and every edge's weight (the sliced
        forward's statistics pass: s1 of the own rows, s2 of every KG row)."""
        from . import ops
        N = csr.n_rows
        dev = s1.device
        m = torch.empty((N, heads), dtype=torch.float32, device=dev)
        den = torch.empty_like(m)
        wgt = torch.empty((max(csr.nnz, 1), heads), dtype=torch.float32, device=dev)
        D = heads * d_head
        fn = ops._gat_fn("gnnea_gat_fwd_sliced_range", torch.float32)
        with _lib.on_device(dev):
            _lib.check(fn(_lib.ptr(csr.rowptr), _lib.ptr(csr.col), N, None, 64, heads, d_head,
                          _lib.ptr(s1), _lib.ptr(s2), float(alpha), None, _lib.GNNEA_ACT_IDENTITY,
                          None, (D + 3) // 4 * 4, _lib.ptr(m), _lib.ptr(den), _lib.ptr(wgt), 0, 0,
                          1, _lib.stream_of(dev)))
        return m, den, wgt

    def gat_fwd_slice(self, csr, tables, q, s1, s2, stats, heads, d_head, alpha, act, Y):
        """Y's columns of slice q from the slice-q table (weights from gat_rowstats)."""
        from . import ops
        m, den, wgt = stats
        S, n, W = tables.shape
        fn = ops._gat_fn("gnnea_gat_fwd_sliced_range", tables.dtype)
        with _lib.on_device(Y.device):
            _lib.check(fn(_lib.ptr(csr.rowptr), _lib.ptr(csr.col), csr.n_rows, _lib.ptr(tables),
                          n * W, heads, d_head, _lib.ptr(s1), _lib.ptr(s2), float(alpha), None,
                          int(act), _lib.ptr(Y), Y.stride(0), _lib.ptr(m), _lib.ptr(den),
                          _lib.ptr(wgt), q, q + 1, 0, _lib.stream_of(Y.device)))
        return Y

    def gat_bwd_prep(self, dY, Y, s1, stats, heads, d_head, act):
        """(G slice-major [S][rows][64], records) of the shard's destination rows."""
        from . import ops
        m, den, _ = stats
        N = Y.shape[0]
        D = heads * d_head
        dY = ops._pad4(dY, D, Y.dtype)
        Gs = ops.sliced_empty(N, D, Y.device, Y.dtype, W=64)
        rec = torch.empty((N, heads, 4), dtype=torch.float32, device=Y.device)
        with _lib.on_device(Y.device):
            _lib.check(ops._gat_fn("gnnea_gat_bwd_prep_sliced", Y.dtype)(
                N, heads, d_head, _lib.ptr(dY), _lib.ptr(Y), Y.stride(0), _lib.ptr(s1),
                _lib.ptr(m), _lib.ptr(den), int(act), _lib.ptr(Gs), Gs.stride(0), _lib.ptr(rec),
                _lib.stream_of(Y.device)))
        return Gs, rec

    def gat_bwd_buffers(self, csrT, S, heads, n_src, dtype, device):
        """(wT, pd, P): per-edge weights, per-slice head-product partials, and the slice-major
        dH partial [S][n_src][64] of every KG row."""
        nnzT = max(csrT.nnz, 1)
        return (torch.empty((nnzT, heads), dtype=torch.float32, device=device),
                torch.empty((S, nnzT, 2), dtype=torch.float32, device=device),
                torch.empty((S, n_src, 64), dtype=dtype, device=device))

    def gat_bwd_src_slice(self, csrT, tables, q, s2, rec, Gs, bufs, heads, d_head, alpha,
                          weights):
        """P[q] = sum_i w_ij G_i over slice q for every KG source row j, and slice q's share of
        the per-edge head products G_i . H_j (H_j read from the halo's slice-q table)."""
        from . import ops
        wT, pd, P = bufs
        S, n, W = tables.shape
        with _lib.on_device(P.device):
            _lib.check(ops._gat_fn("gnnea_gat_bwd_src_sliced_range", tables.dtype)(
                _lib.ptr(csrT.rowptr), _lib.ptr(csrT.col), _lib.ptr(csrT.perm), csrT.n_rows,
                heads, d_head, _lib.ptr(tables), 64, n * W, _lib.ptr(s2), float(alpha), None,
                _lib.ptr(rec), _lib.ptr(Gs), Gs.stride(0), _lib.ptr(wT), _lib.ptr(pd),
                csrT.nnz, _lib.ptr(P), 64, P.stride(0), q, q + 1, 1 if weights else 0,
                _lib.stream_of(P.device)))
        return P[q]

    def gat_bwd_edge(self, csrT, s2, rec, bufs, a, heads, d_head, alpha):
        """(dz in A^T order, ds2 partial of every KG row); dH is left alone."""
        from . import ops
        a32 = ops._featc(a, torch.float32)
        _, pd, _ = bufs
        dev = s2.device
        dzT = torch.empty((max(csrT.nnz, 1), heads), dtype=torch.float32, device=dev)
        ds2 = torch.empty((csrT.n_rows, heads), dtype=torch.float32, device=dev)
        with _lib.on_device(dev):
            _lib.check(ops._gat_fn("gnnea_gat_bwd_edge_sliced", torch.float32)(
                _lib.ptr(csrT.rowptr), _lib.ptr(csrT.col), _lib.ptr(csrT.perm), csrT.n_rows,
                heads, d_head, _lib.ptr(s2), float(alpha), None, _lib.ptr(rec), _lib.ptr(pd),
                csrT.nnz, _lib.ptr(a32), None, heads * d_head, _lib.ptr(dzT), _lib.ptr(ds2),
                _lib.stream_of(dev)))
        return dzT, ds2

    def gat_bwd_dst(self, csr, dzT, a, ds2, dH, heads, d_head):
        """ds1 of the shard's rows and dH_i += ds1_i (x) a1 + ds2_i (x) a2 (own rows)."""
        from . import ops
        a32 = ops._featc(a, torch.float32)
        dev = dH.device
        ds1 = torch.empty((csr.n_rows, heads), dtype=torch.float32, device=dev)
        with _lib.on_device(dev):
            _lib.check(ops._gat_fn("gnnea_gat_bwd_dst_sliced", dH.dtype)(
                _lib.ptr(csr.rowptr), _lib.ptr(csr.tpos()), csr.n_rows, heads, d_head,
                _lib.ptr(dzT), _lib.ptr(a32), _lib.ptr(ds2), _lib.ptr(dH), dH.stride(0),
                _lib.ptr(ds1), _lib.stream_of(dev)))
        return ds1

    def gat_da(self, H, ds, heads, d_head):
        from . import ops
        return ops.gat_da(H, ds, heads, d_head)

    def transpose(self, csr):
        return csr.transpose()

    def unpack64(self, Ts, D):
        """[S][rows][64] slice-major -> row-major [rows, D] (a view of a [rows, 64 S] copy)."""
        S, n, W = Ts.shape
        return Ts.permute(1, 0, 2).reshape(n, S * W)[:, :D]

    def gat_bwd(self, csr, saved, dY, heads, d_head, alpha, act, row0, need_da):
        """(dH partial over every KG row, da partial) of sum(Y_loc ⊙ dY)."""
        from . import ops
        Hp, a32, s1, s2, m, den, Y = saved
        D = heads * d_head
        dH, da = ops.gat_backward(csr, Hp, a32, s1, s2, m, den, Y, dY, heads, d_head, alpha,
                                  act, row0=row0, need_da=need_da)
        return (dH if dH.shape[1] == D else dH[:, :D]), da


def _is_gloo(group):
    return dist.get_backend(group) == "gloo"


class DistAdj:
    """This rank's shard of the two-KG adjacency plus its KG group.

    Build it on every rank (group creation is collective) with ``from_triples`` (the synthetic
    cfg graphs) or from the rank's COO shard (local rows, KG-local columns), then pass it as the
    ``adj`` of GraphConvolution / HighWayGraphConvolution / Encoder.encode / Decoder.decode with
    the rank's own feature rows ``x[part.global_row0 : part.global_row0 + part.n_rows]``."""

    def __init__(self, part, r, c, v, device, engine=None):
        if part.world > 1 and part.kind != "rows":
            raise ValueError("gnnea.DistAdj: the layers need the row partition")
        self.part = part
        self.device = device
        self.engine = engine or HipEngine()
        e = self.engine
        self.nnz = int(np.asarray(r).size)
        self.csr = e.csr(r, c, v, part.n_rows, part.n_cols, device)
        self.group = make_groups(part) if part.world > 1 else None

    @classmethod
    def from_triples(cls, triples, n, t, rank, world, device, engine=None):
        """Shard of the synthetic cfg pair (gnnea.synth.kg_pair_triples layout: KG k's t triples
        at rows [k·t, (k+1)·t), entities [k·n, (k+1)·n))."""
        part = Partition(n, rank, world, "rows")
        r, c, v = shard_coo(triples, n, t, part)
        return cls(part, r, c, v, device, engine)

    @classmethod
    def from_shard(cls, shard):
        """The layers' view of a bench KGShard (gnnea.dist, rows partition): its CSR and KG
        group are shared, nothing is rebuilt."""
        if shard.part.kind != "rows":
            raise ValueError("gnnea.DistAdj: the layers need the row partition")
        self = cls.__new__(cls)
        self.part, self.device, self.engine = shard.part, shard.device, HipEngine()
        self.nnz, self.csr, self.group = shard.nnz, shard.csr, shard.group
        return self

    # ---- the drop-in layer hooks ------------------------------------------------------------
    def aggregate(self, hidden, act_fn):
        from .ops import act_code
        code = act_code(act_fn) if act_fn is not None else _lib.GNNEA_ACT_IDENTITY
        if code is None:
            return act_fn(HaloAggregateFn.apply(hidden, self, _lib.GNNEA_ACT_IDENTITY))
        return HaloAggregateFn.apply(hidden, self, code)

    def highway(self, hidden, gate_pre, resid, bias_gate, act_fn):
        from .ops import act_code
        code = act_code(act_fn)
        if code is None:
            s = act_fn(HaloAggregateFn.apply(hidden, self, _lib.GNNEA_ACT_IDENTITY))
            g = torch.sigmoid(gate_pre + bias_gate) if bias_gate is not None else \
                torch.sigmoid(gate_pre)
            return g * s + (1.0 - g) * resid
        return HaloHighwayFn.apply(hidden, gate_pre, resid, bias_gate, self, code)

    def gat(self, H, a_all, heads, d_head, alpha, act_fn):
        """All heads of a GraphAttentionLayer over the shard (layers/att_layers.py:29-61, 86):
        H = x_loc·[W_0|...|W_{h-1}] is row-local; the KG group's H rows arrive by the halo
        all-gather, the logits / softmax / aggregation of the owned rows run on them, and the
        backward reduce-scatters the gradient of every KG row back to its owner."""
        from .ops import act_code
        code = act_code(act_fn) if act_fn is not None else _lib.GNNEA_ACT_IDENTITY
        if code not in (_lib.GNNEA_ACT_IDENTITY, _lib.GNNEA_ACT_RELU):
            return act_fn(HaloGATFn.apply(H, a_all, self, heads, d_head, alpha,
                                          _lib.GNNEA_ACT_IDENTITY))
        return HaloGATFn.apply(H, a_all, self, heads, d_head, alpha, code)

    def highway_fwd(self, hidden, gate_pre, resid, bias_gate, act):
        """HighWay tail over the shard (gnnea.ops.HighwayLayerFn's aggregation hook): the
        group's hidden rows by the halo all-gather, gate_pre / resid row-local."""
        if self.staged(hidden, highway=True):
            return self.staged_highway(hidden, gate_pre, resid, bias_gate, act)
        full, _ = self.halo(hidden)
        return self.engine.highway_fwd(self.csr, full, gate_pre, resid, bias_gate, act)

    # ---- the per-slice pipeline (§8e overlap) ------------------------------------------------
    def staged(self, t, highway=False):
        """The halo of ``t`` moves slice by slice, overlapped with the per-slice aggregation:
        every row shard (g > 1) whose engine has the slice operations; fp32 / bf16 with whole
        4-column chunks (the HighWay tail too: the fp32 sliced kernel, or for bf16 the
        row-major kernel over each 128-column slice table)."""
        from . import exchange
        if (self.part.g == 1 or not exchange.staged_for(t.dtype)
                or not hasattr(self.engine, "slice_w") or t.shape[1] % 4):
            return False
        if isinstance(self.engine, HipEngine):
            return t.dtype in (torch.float32, torch.bfloat16)
        return True

    def stages(self, D, dtype):
        """Column blocks [(c0, c1)] of width W = the engine's slice width."""
        W = self.engine.slice_w(dtype)
        return W, [(c0, min(D, c0 + W)) for c0 in range(0, D, W)]

    def _peers(self):
        return self.part.group_ranks(self.part.kg), self.part.li, self.part.other_ranks()

    def staged_gat(self, heads, d_head, dtype):
        """The GAT halo moves slice by slice (64-column tables), overlapped with the per-slice
        aggregation: row shards (g > 1) whose engine has the staged GAT operations."""
        from . import exchange
        return (self.part.g > 1 and exchange.staged_for(dtype)
                and hasattr(self.engine, "gat_fwd_slice")
                and self.engine.gat_staged_ok(heads, d_head))

    def halo_slices(self, h_loc, gat=False):
        """Pack the own rows into the KG's slice tables [S][n][W] and issue every slice's
        exchange: returns (tables, stages, works per slice).  gat: the GAT kernels' 64-column
        tables for either storage type."""
        from . import exchange
        D = h_loc.shape[1]
        if gat:
            W = self.engine.gat_slice_w(h_loc.dtype)
            st = [(c0, min(D, c0 + W)) for c0 in range(0, D, W)]
        else:
            W, st = self.stages(D, h_loc.dtype)
        tables = torch.empty((len(st), self.part.n_cols, W), dtype=h_loc.dtype,
                             device=h_loc.device)
        if gat:
            self.engine.gat_pack(h_loc, tables, self.part.row0)
        else:
            self.engine.pack_slices(h_loc, tables, self.part.row0)
        ranks, li, other = self._peers()
        works = exchange.all_gather_slices(list(tables), self.part.row0, self.part.n_rows,
                                           self.group, ranks, li, other)
        return tables, st, works

    def staged_aggregate(self, hidden, act, events=None):
        """out = act(A_shard · hidden_KG), slice q aggregated as soon as it has landed."""
        tables, st, works = self.halo_slices(hidden)
        out = torch.empty((self.part.n_rows, hidden.shape[1]), dtype=hidden.dtype,
                          device=hidden.device)
        for q, (c0, c1) in enumerate(st):
            for w in works[q]:
                w.wait()
            if events is not None:
                events[q][0].record()
            self.engine.spmm_slice(self.csr, tables[q], c1 - c0, act, out[:, c0:c1])
            if events is not None:
                events[q][1].record()
        return out

    def staged_aggregate_t(self, Gs, D, out=None):
        """This rank's rows of sum_group A_shardᵀ·G from G held as local slice tables
        ([S][rows][W]): per slice, Aᵀ·G_q then its reduce-scatter issued at once (the owner sums
        in peer order once every slice has arrived).  ``out``: [rows, D] (a column block of a
        wider buffer is fine)."""
        from . import exchange
        _, st = self.stages(D, Gs.dtype)
        if out is None:
            out = torch.empty((self.part.n_rows, D), dtype=Gs.dtype, device=Gs.device)
        ranks, li, other = self._peers()
        pend = []
        for q, (c0, c1) in enumerate(st):
            P = self.engine.spmm_t_slice(self.csr, Gs[q], c1 - c0)
            pend.append(exchange.reduce_scatter_start(P, self.group, ranks, li, other,
                                                      out=out[:, c0:c1]))
        for p in pend:
            p.finish()
        return out

    def staged_highway(self, hidden, gate_pre, resid, bias_gate, act):
        """HighWay tail (layers/layers.py:64-76) slice by slice over the halo tables; the gate
        is row-local (packed into the shard's own slice tables)."""
        tables, st, works = self.halo_slices(hidden)
        n_rows, D = self.part.n_rows, hidden.shape[1]
        gates = torch.empty((len(st), n_rows, tables.shape[2]), dtype=hidden.dtype,
                            device=hidden.device)
        self.engine.pack_slices(gate_pre, gates, 0)
        out = torch.empty((n_rows, D), dtype=hidden.dtype, device=hidden.device)
        S = torch.empty_like(out)
        G = torch.empty_like(out)
        resid = resid.contiguous()
        for q, (c0, c1) in enumerate(st):
            for w in works[q]:
                w.wait()
            self.engine.highway_slice(self.csr, tables[q], c1 - c0, gates, c0, bias_gate, resid,
                                      out, S, G, act)
        return out, S, G

    def local_csr(self):
        """The shard's CSR when this rank aggregates without any exchange (one KG per rank, or
        the whole graph at world 1) on the HIP engine, else None."""
        return self.csr if self.part.g == 1 and isinstance(self.engine, HipEngine) else None

    def sliced_ok(self, D, dtype):
        """Slice-major fused HighWay layer: only without exchange (the halo moves row-major
        rows)."""
        from .ops import use_sliced
        return (dtype == torch.float32 and self.local_csr() is not None
                and use_sliced(self.csr.n_cols, D, dtype))

    def highway_fwd_sliced(self, Zs, D, resid, bias_gate, act, goff=None, save_s=True):
        from . import ops
        return ops.highway_fwd_sliced(self.csr, Zs, D, resid, bias_gate, act, save_g=False,
                                      goff=goff, save_s=save_s)

    def highway_fwd_sliced_m(self, Zs, D, resid, bias_gate, goff):
        from . import ops
        return ops.highway_fwd_sliced_m(self.csr, Zs, D, resid, bias_gate, goff)

    def aggregate_t_sliced(self, gs, D, out):
        from . import ops
        return ops.spmm_sliced(self.csr.transpose(), gs, D, out=out)

    def aggregate_t(self, g, out):
        """out = (A_shardᵀ·g) summed over the KG group, this rank's rows (HighwayLayerFn's
        backward hook; out may be a column block of a wider buffer)."""
        if self.part.g == 1:
            return self.engine.spmm_t(self.csr, g, out=out)
        if self.staged(g):
            W, st = self.stages(g.shape[1], g.dtype)
            Gs = torch.empty((len(st), self.part.n_rows, W), dtype=g.dtype, device=g.device)
            self.engine.pack_slices(g, Gs, 0)
            return self.staged_aggregate_t(Gs, g.shape[1], out)
        out.copy_(self.reduce_scatter(self.engine.spmm_t(self.csr, g)))
        return out

    def gat_staged_forward(self, H, a_all, heads, d_head, alpha, act):
        """GAT of the shard's rows with the halo cut into 64-column slices: the logits s2 of
        every KG row first (one small all-gather: the row statistics need them), the row
        statistics and edge weights while the slices move, then slice q aggregated as soon as
        it has landed.  Returns (Y [rows, D], saved state for gat_staged_backward)."""
        from . import exchange
        e = self.engine
        D = heads * d_head
        s1, s2_loc = e.gat_scores(H, a_all, heads, d_head)
        s2 = torch.empty((self.part.n_cols, heads), dtype=s2_loc.dtype, device=s2_loc.device)
        ranks, li, other = self._peers()
        exchange.all_gather(s2_loc, s2, self.group, ranks, li, copy_own=True, other=other)
        tables, st, works = self.halo_slices(H, gat=True)
        stats = e.gat_rowstats(self.csr, s1, s2, heads, d_head, alpha)
        Y = torch.empty((self.part.n_rows, D), dtype=H.dtype, device=H.device)
        for q in range(len(st)):
            for w in works[q]:
                w.wait()
            e.gat_fwd_slice(self.csr, tables, q, s1, s2, stats, heads, d_head, alpha, act, Y)
        return Y, (tables, s1, s2, stats, Y, H)

    def gat_staged_backward(self, saved, dY, a_all, heads, d_head, alpha, act, need_da):
        """Backward of gat_staged_forward: the source pass slice by slice over every KG row,
        each slice's dH partial reduce-scattered as soon as it is computed (the next slice
        computing while it moves); the edge pass's ds2 partials reduce-scattered too (tiny), so
        the owners add ds1 (x) a1 + ds2 (x) a2 to their rows; da from the own rows only."""
        from . import exchange
        tables, s1, s2, stats, Y, H = saved
        e = self.engine
        D = heads * d_head
        a = a_all.detach()
        Gs, rec = e.gat_bwd_prep(dY, Y, s1, stats, heads, d_head, act)
        csrT = e.transpose(self.csr)
        S = tables.shape[0]
        bufs = e.gat_bwd_buffers(csrT, S, heads, self.part.n_cols, Y.dtype, Y.device)
        out = torch.empty((S, self.part.n_rows, tables.shape[2]), dtype=Y.dtype,
                          device=Y.device)
        ranks, li, other = self._peers()
        pend = []
        for q in range(S):
            P = e.gat_bwd_src_slice(csrT, tables, q, s2, rec, Gs, bufs, heads, d_head, alpha,
                                    q == 0)
            pend.append(exchange.reduce_scatter_start(P, self.group, ranks, li, other,
                                                      out=out[q]))
        dzT, ds2 = e.gat_bwd_edge(csrT, s2, rec, bufs, a, heads, d_head, alpha)
        ds2_own = self.reduce_scatter(ds2)
        for p in pend:
            p.finish()
        dH = e.unpack64(out, D)
        ds1 = e.gat_bwd_dst(self.csr, dzT, a, ds2_own, dH, heads, d_head)
        da = None
        if need_da:
            p1 = e.gat_da(H, ds1, heads, d_head)
            p2 = e.gat_da(H, ds2_own, heads, d_head)
            da = torch.cat([p1.view(heads, d_head), p2.view(heads, d_head)], dim=1)
        return dH, da

    def gather_rows(self, out_loc):
        """[2n, D] embeddings of both KGs in global entity order, on every rank."""
        return GatherRowsFn.apply(out_loc, self)

    # ---- exchanges ------------------------------------------------------------------------
    def halo(self, h_loc, async_op=False, copy_own=True):
        """The KG group's rows [n, D] by direct peer transfers (gnnea.exchange): returns
        (h_KG, work or None); copy_own=False leaves the own block unwritten (for the
        remote-column CSR, which never reads it)."""
        from . import exchange
        from .dist import _Works
        g = self.part.g
        if g == 1:
            return h_loc, None
        h_loc = h_loc.contiguous()
        full = torch.empty((g * h_loc.shape[0], h_loc.shape[1]), dtype=h_loc.dtype,
                           device=h_loc.device)
        works = exchange.all_gather(h_loc, full, self.group, self.part.group_ranks(self.part.kg),
                                    self.part.li, copy_own=copy_own, async_op=async_op,
                                    other=self.part.other_ranks())
        return full, (_Works(works) if works else None)

    def reduce_scatter(self, partial):
        """Sum the group's [n, D] partials and keep this rank's n/g rows (peer transfers, the
        owner sums in peer order)."""
        from . import exchange
        if self.part.g == 1:
            return partial
        return exchange.reduce_scatter(partial, self.group, self.part.group_ranks(self.part.kg),
                                       self.part.li, other=self.part.other_ranks())

    def all_rows(self, out_loc):
        W = self.part.world
        if W == 1:
            return out_loc
        out_loc = out_loc.contiguous()
        if dist.get_backend() == "gloo":
            hl = out_loc.detach().cpu()
            parts = [torch.empty_like(hl) for _ in range(W)]
            dist.all_gather(parts, hl)
            return torch.cat(parts).to(out_loc.device)
        full = torch.empty((W * out_loc.shape[0], out_loc.shape[1]), dtype=out_loc.dtype,
                           device=out_loc.device)
        dist.all_gather_into_tensor(full, out_loc)
        return full


class HaloAggregateFn(torch.autograd.Function):
    """out_loc = act(A_shard · all_gather(hidden_loc)); backward reduce_scatter(A_shardᵀ · G)."""

    @staticmethod
    def forward(ctx, hidden, dadj, act):
        e = dadj.engine
        if dadj.part.g == 1:
            out = e.spmm(dadj.csr, hidden, act)
        elif dadj.staged(hidden):
            out = dadj.staged_aggregate(hidden, act)  # per-slice exchange / aggregation
        else:
            full, _ = dadj.halo(hidden)
            out = e.spmm(dadj.csr, full, act)
        ctx.dadj, ctx.act = dadj, act
        ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, dy):
        (out,) = ctx.saved_tensors
        dadj = ctx.dadj
        if dadj.part.g > 1 and dadj.staged(out):
            Gs = dadj.engine.act_bwd_slices(dy.contiguous(), out, ctx.act)
            return dadj.staged_aggregate_t(Gs, out.shape[1]), None, None
        return dadj.reduce_scatter(dadj.engine.act_spmm_t(dadj.csr, dy, out, ctx.act)), None, None


class HaloHighwayFn(torch.autograd.Function):
    """HighWay tail on the shard: S = act(A_shard·hidden_KG); g = sigmoid(gate_pre + b_g);
    out = g*S + (1-g)*resid (gate_pre, resid row-local)."""

    @staticmethod
    def forward(ctx, hidden, gate_pre, resid, bias_gate, dadj, act):
        out, S, G = dadj.highway_fwd(hidden, gate_pre, resid, bias_gate, act)
        ctx.dadj, ctx.act = dadj, act
        ctx.save_for_backward(S, G, resid)
        return out

    @staticmethod
    def backward(ctx, dy):
        S, G, resid = ctx.saved_tensors
        dadj = ctx.dadj
        e = dadj.engine
        if dadj.part.g > 1 and dadj.staged(S, highway=True):
            dgate = torch.empty_like(S)
            dSs, dres = e.highway_bwd_slices(dy.contiguous(), S, G, resid, ctx.act,
                                             ctx.needs_input_grad[2], dgate)
            return (dadj.staged_aggregate_t(dSs, S.shape[1]), dgate, dres, None, None, None)
        dS, dgate, dres = e.highway_bwd(dy.contiguous(), S, G, resid, ctx.act,
                                        ctx.needs_input_grad[2])
        dh = dadj.reduce_scatter(e.spmm_t(dadj.csr, dS))
        return dh, dgate, dres, None, None, None


class HaloGATFn(torch.autograd.Function):
    """Y_loc = GAT(A_shard, all_gather(H_loc)) for the owned rows; backward: the shard's dH
    partial over every KG row is reduce-scattered to the owners, da stays a per-rank partial
    (summed with the other parameter gradients by allreduce_grads)."""

    @staticmethod
    def forward(ctx, H, a_all, dadj, heads, d_head, alpha, act):
        ctx.dadj = dadj
        ctx.meta = (heads, d_head, float(alpha), int(act))
        ctx.staged = dadj.staged_gat(heads, d_head, H.dtype) and H.shape[1] == heads * d_head
        if ctx.staged:  # per-slice exchange / aggregation (§8e overlap)
            Y, ctx.saved = dadj.gat_staged_forward(H.contiguous(), a_all, heads, d_head, alpha,
                                                   act)
            ctx.a_all = a_all.detach()
            return Y
        full, _ = dadj.halo(H)
        row0 = dadj.part.row0 if dadj.part.g > 1 else 0
        Y, saved = dadj.engine.gat_fwd(dadj.csr, full, a_all, heads, d_head, alpha, act, row0)
        ctx.row0 = row0
        ctx.saved = saved
        return Y

    @staticmethod
    def backward(ctx, dY):
        heads, d_head, alpha, act = ctx.meta
        dadj = ctx.dadj
        if ctx.staged:
            dH, da = dadj.gat_staged_backward(ctx.saved, dY.contiguous(), ctx.a_all, heads,
                                              d_head, alpha, act, ctx.needs_input_grad[1])
            ctx.saved = None
            return dH, da, None, None, None, None, None
        dH, da = dadj.engine.gat_bwd(dadj.csr, ctx.saved, dY.contiguous(), heads, d_head, alpha,
                                     act, ctx.row0, ctx.needs_input_grad[1])
        ctx.saved = None
        return dadj.reduce_scatter(dH), da, None, None, None, None, None


class GatherRowsFn(torch.autograd.Function):
    """All ranks' rows in global order.  The loss on top is evaluated identically on every
    rank, so d loss / d out_loc is this rank's slice of the (replicated) gradient."""

    @staticmethod
    def forward(ctx, out_loc, dadj):
        ctx.rows = out_loc.shape[0]
        ctx.rank = dadj.part.rank
        return dadj.all_rows(out_loc)

    @staticmethod
    def backward(ctx, dfull):
        r0 = ctx.rank * ctx.rows
        return dfull[r0:r0 + ctx.rows].contiguous(), None


def _world_reduce(vals, op):
    """All-reduce a few float64 scalars over the world (host tensors under gloo)."""
    if dist.get_backend() == "gloo":
        t = torch.tensor(vals, dtype=torch.float64)
    else:
        t = torch.tensor(vals, dtype=torch.float64,
                         device=torch.device("cuda", torch.cuda.current_device()))
    dist.all_reduce(t, op=op)
    return t.cpu().tolist()


def _world_sum(t):
    """Sum of a tensor over every rank (the replicated parameters' gradients)."""
    t = t.detach().contiguous()
    if dist.get_backend() == "gloo" and t.device.type != "cpu":
        h = t.cpu()
        dist.all_reduce(h)
        return h.to(t.device)
    t = t.clone()
    dist.all_reduce(t)
    return t


def validate_staged(dadj, D=300, heads=4, alpha=0.2, dtypes=None, reps=3, tol=1e-6,
                    tol_bf16=1e-2, seed=0, apply=True):
    """Prove the per-slice halo pipeline on this job's own ranks before it is used (SURVEY.md §8e;
    layers/layers.py:35,64, layers/att_layers.py:45-58): one HighWay layer tail
    (HaloHighwayFn), one GCN aggregation (HaloAggregateFn) and one all-head GAT layer
    (HaloGATFn), forward + backward on the same seeded inputs with exchange.STAGED off, then on,
    once per storage dtype in ``dtypes`` (default fp32 on the device, fp64 on the CPU; the bench
    passes fp32 and bf16, configs[4]'s dtype, whose staged GAT runs the bf16 64-column tables).
    The legs run with smooth activations (tanh; GAT: none): with relu, an output within rounding
    of 0 can take the other branch of relu' on one side, and the input gradient then differs by
    a whole adjacency weight at that row (the staged and unstaged forwards sum in different
    orders) — a branch decision, not an exchange error.
    Compared: outputs, input gradients and the world-summed `a` gradient, norm-relative
    ‖staged − unstaged‖∞ / ‖unstaged‖∞, the max over tensors and ranks; a dtype matches when it
    is ≤ ``tol`` (bf16: ``tol_bf16``, the bf16 storage tolerance of tests/test_gpu_scale_cfg5.py:
    the two paths round differently ordered fp32 sums to bf16) and finite on every rank (one
    all-reduce decides, so all ranks agree).  Each leg is timed both ways (median of ``reps``
    fwd + bwd after one warm-up, wall clock bracketed by barriers and device syncs, max over
    ranks).  ``apply`` (GNNEA_HALO_STAGED unset / "auto"): exchange.STAGED is left on for
    exactly the dtypes that matched (exchange.STAGED_DTYPES), off when none did; "0" keeps it
    off and "1" keeps it on for every dtype whatever the outcome (the report still says what
    matched).  Every rank must call this.  Returns the report (the same dict on every rank)."""
    import time

    from . import exchange
    part = dadj.part
    if part.g == 1:
        return {"applies": False, "reason": "one KG per rank: nothing to exchange"}
    dev = dadj.device
    if dtypes is None:
        dtypes = (torch.float64 if dev.type == "cpu" else torch.float32,)
    d_head = D // heads
    n = part.n_rows

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    def make_legs(dtype):
        # the rows are the rank's own; the parameters (bias_gate, a) are replicated on every rank
        rows_gen = torch.Generator(device=dev).manual_seed(seed * 1000 + 1 + part.rank)
        par_gen = torch.Generator(device=dev).manual_seed(seed * 1000)

        def rnd(*shape, scale=1.0, gen=rows_gen):
            return (scale * torch.randn(*shape, generator=gen, device=dev, dtype=torch.float32)
                    ).to(dtype)
        hidden, gate_pre, resid = rnd(n, D), rnd(n, D), rnd(n, D)
        bias_gate = rnd(D, scale=0.1, gen=par_gen)
        dY = rnd(n, D)
        H = rnd(n, heads * d_head, scale=0.3)
        a_all = rnd(heads, 2 * d_head, scale=0.3, gen=par_gen)
        dYg = rnd(n, heads * d_head)

        def leg_highway():
            xs = [t.clone().requires_grad_() for t in (hidden, gate_pre, resid)]
            out = dadj.highway(xs[0], xs[1], xs[2], bias_gate, torch.tanh)
            out.backward(dY)
            return [out.detach()] + [x.grad for x in xs]

        def leg_gcn():
            x = hidden.clone().requires_grad_()
            out = dadj.aggregate(x, torch.tanh)
            out.backward(dY)
            return [out.detach(), x.grad]

        def leg_gat():
            h = H.clone().requires_grad_()
            a = a_all.clone().requires_grad_()
            out = dadj.gat(h, a, heads, d_head, alpha, None)
            out.backward(dYg)
            return [out.detach(), h.grad, _world_sum(a.grad)]
        legs = {"highway": leg_highway, "gcn": leg_gcn}
        if dadj.engine.gat_staged_ok(heads, d_head) if hasattr(dadj.engine, "gat_staged_ok") \
                else False:
            legs["gat"] = leg_gat
        return legs

    def timed(fn):
        fn()
        ts = []
        for _ in range(reps):
            sync()
            dist.barrier()
            t0 = time.perf_counter()
            fn()
            sync()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) * 1e3

    keep, keep_dt = exchange.STAGED, exchange.STAGED_DTYPES
    res, ms, names = {}, {}, {}
    try:
        exchange.STAGED_DTYPES = None  # the legs run each mode for their own dtype
        for dtype in dtypes:
            legs = make_legs(dtype)
            names[dtype] = list(legs)
            for mode in (False, True):
                exchange.STAGED = mode
                for name, fn in legs.items():
                    res[(dtype, name, mode)] = [t.detach().clone() for t in fn()]
                    ms[(dtype, name, mode)] = timed(fn)
            del legs
    finally:
        exchange.STAGED, exchange.STAGED_DTYPES = keep, keep_dt
    keys = [(dt, k) for dt in dtypes for k in names[dt]]
    errs = []
    for dt, name in keys:
        e = 0.0
        for s, u in zip(res[(dt, name, True)], res[(dt, name, False)]):
            s, u = s.double(), u.double()
            if not bool(torch.isfinite(s).all()) or s.shape != u.shape:
                e = float("inf")
                break
            den = float(u.abs().max()) if u.numel() else 0.0
            num = float((s - u).abs().max()) if u.numel() else 0.0
            e = max(e, num / den if den > 0 else (0.0 if num == 0 else float("inf")))
        errs.append(e)
    res = None
    # one all-reduce: every rank's errors (max) and its leg times (max over ranks)
    times = [ms[(dt, k, m)] for dt, k in keys for m in (True, False)]
    red = _world_reduce([min(e, 1e300) for e in errs] + times, dist.ReduceOp.MAX)
    errs, times = red[:len(keys)], red[len(keys):]
    report = {"applies": True, "reps": reps, "world": part.world, "group_ranks": part.g,
              "D": D, "heads": heads, "dtypes": {},
              "method": "staged vs unstaged on the same inputs, per storage dtype: outputs, input "
                        "gradients and the world-summed attention-vector gradient, "
                        "norm-relative, max over tensors and ranks; fwd + bwd wall ms, median "
                        "of %d, max over ranks" % reps}
    matched = []
    for dt in dtypes:
        name = str(dt).replace("torch.", "")
        t_ = tol_bf16 if dt == torch.bfloat16 else tol
        rep = {"tol": t_, "legs": {}}
        e_dt = 0.0
        for i, (d2, k) in enumerate(keys):
            if d2 != dt:
                continue
            e_dt = max(e_dt, errs[i])
            rep["legs"][k] = {"err": errs[i], "staged_ms": round(times[2 * i], 4),
                              "unstaged_ms": round(times[2 * i + 1], 4)}
        rep["max_norm_rel_err"] = e_dt
        rep["match"] = bool(e_dt <= t_)
        if rep["match"]:
            matched.append(dt)
        report["dtypes"][name] = rep
    report["match"] = len(matched) == len(dtypes)
    report["staged_ms"] = round(sum(times[0::2]), 4)
    report["unstaged_ms"] = round(sum(times[1::2]), 4)
    if apply:
        if exchange.STAGED_ENV == "0":
            exchange.STAGED, exchange.STAGED_DTYPES = False, None
        elif exchange.STAGED_ENV != "1":
            exchange.STAGED = bool(matched)
            exchange.STAGED_DTYPES = set(matched) if matched else None
    report["staged_env"] = exchange.STAGED_ENV
    report["staged_in_use"] = {str(dt).replace("torch.", ""): bool(exchange.staged_for(dt))
                               for dt in dtypes}
    return report


def allreduce_grads(params, group=None):
    """Sum the parameter gradients of all ranks in ONE bucket (the weights are replicated and
    small: 3 x 300 x 300 fp32 for HGCN-EA, so one RCCL all_reduce of < 1.1 MB per step)."""
    ps = [p for p in params if p.grad is not None]
    if not ps or dist.get_world_size(group) == 1:
        return
    # summed in at least fp32: bf16 gradients (configs[4]) are rounded once, after the sum,
    # instead of at every step of the reduction
    acc = torch.float32
    for p in ps:
        acc = torch.promote_types(acc, p.grad.dtype)
    flat = torch.cat([p.grad.reshape(-1).to(acc) for p in ps])
    if dist.get_backend(group) == "gloo" and flat.device.type != "cpu":
        h = flat.cpu()
        dist.all_reduce(h, group=group)
        flat = h.to(flat.device)
    else:
        dist.all_reduce(flat, group=group)
    k = 0
    for p in ps:
        m = p.grad.numel()
        p.grad.copy_(flat[k:k + m].view_as(p.grad))
        k += m
