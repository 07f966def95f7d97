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
from .dist import Partition, make_groups, shard_coo, split_own_remote


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
        if part.g > 1:
            (ro, co, vo), (rr, cr, vr) = split_own_remote(r, c, v, part)
            self.csr_own = e.csr(ro, co, vo, part.n_rows, part.n_rows, device)
            self.csr_remote = e.csr(rr, cr, vr, part.n_rows, part.n_cols, device)
        else:
            self.csr_own = self.csr_remote = None
        self.group = make_groups(part) if part.world > 1 else None

    @classmethod
    def from_triples(cls, triples, n, t, rank, world, device, engine=None):
        """Shard of the synthetic cfg pair (gnnea.synth.kg_pair_triples layout: KG k's t triples
        at rows [k·t, (k+1)·t), entities [k·n, (k+1)·n))."""
        part = Partition(n, rank, world, "rows")
        r, c, v = shard_coo(triples, n, t, part)
        return cls(part, r, c, v, device, engine)

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
        full, _ = self.halo(hidden)
        return self.engine.highway_fwd(self.csr, full, gate_pre, resid, bias_gate, act)

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

    def highway_fwd_sliced(self, Zs, D, resid, bias_gate, act):
        from . import ops
        return ops.highway_fwd_sliced(self.csr, Zs, D, resid, bias_gate, act)

    def aggregate_t_sliced(self, gs, D, out):
        from . import ops
        return ops.spmm_sliced(self.csr.transpose(), gs, D, out=out)

    def aggregate_t(self, g, out):
        """out = (A_shardᵀ·g) summed over the KG group, this rank's rows (HighwayLayerFn's
        backward hook; out may be a column block of a wider buffer)."""
        if self.part.g == 1:
            return self.engine.spmm_t(self.csr, g, out=out)
        out.copy_(self.reduce_scatter(self.engine.spmm_t(self.csr, g)))
        return out

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
        else:
            full, work = dadj.halo(hidden, async_op=True, copy_own=False)
            out = e.spmm(dadj.csr_own, hidden, _lib.GNNEA_ACT_IDENTITY)  # overlaps the gather
            if work is not None:
                work.wait()
            e.spmm(dadj.csr_remote, full, act, out=out, beta=1.0)
        ctx.dadj, ctx.act = dadj, act
        ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, dy):
        (out,) = ctx.saved_tensors
        dadj = ctx.dadj
        return dadj.reduce_scatter(dadj.engine.act_spmm_t(dadj.csr, dy, out, ctx.act)), None, None


class HaloHighwayFn(torch.autograd.Function):
    """HighWay tail on the shard: S = act(A_shard·hidden_KG); g = sigmoid(gate_pre + b_g);
    out = g*S + (1-g)*resid (gate_pre, resid row-local)."""

    @staticmethod
    def forward(ctx, hidden, gate_pre, resid, bias_gate, dadj, act):
        full, _ = dadj.halo(hidden)
        out, S, G = dadj.engine.highway_fwd(dadj.csr, full, gate_pre, resid, bias_gate, act)
        ctx.dadj, ctx.act = dadj, act
        ctx.save_for_backward(S, G, resid)
        return out

    @staticmethod
    def backward(ctx, dy):
        S, G, resid = ctx.saved_tensors
        dadj = ctx.dadj
        e = dadj.engine
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
        full, _ = dadj.halo(H)
        row0 = dadj.part.row0 if dadj.part.g > 1 else 0
        Y, saved = dadj.engine.gat_fwd(dadj.csr, full, a_all, heads, d_head, alpha, act, row0)
        ctx.dadj, ctx.row0 = dadj, row0
        ctx.meta = (heads, d_head, float(alpha), int(act))
        ctx.saved = saved
        return Y

    @staticmethod
    def backward(ctx, dY):
        heads, d_head, alpha, act = ctx.meta
        dadj = ctx.dadj
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


def allreduce_grads(params, group=None):
    """Sum the parameter gradients of all ranks in ONE bucket (the weights are replicated and
    small: 3 x 300 x 300 fp32 for HGCN-EA, so one RCCL all_reduce of < 1.1 MB per step)."""
    ps = [p for p in params if p.grad is not None]
    if not ps or dist.get_world_size(group) == 1:
        return
    flat = torch.cat([p.grad.reshape(-1) for p in ps])
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
