"""Drop-in GCN layers backed by libgnnea (reference: layers/layers.py).

Constructor signatures, parameter creation order (hence RNG consumption under
``torch.manual_seed``), attribute names and ``state_dict`` keys are those of the reference, so
``run/train_ea.py`` and its saved models work unchanged.  The forward passes run on HIP only:
  hidden = x W^T + b          -> MFMA f32 GEMM   (gnnea_gemm_f32)
  act(A · hidden)             -> CSR gather SpMM with fused activation (gnnea_spmm_csr_f32; above
                                 the Infinity Cache the hidden is written slice-major by the GEMM
                                 and gathered by gnnea_spmm_sliced_f32)
  HighWay gate + blend        -> SpMM with fused sigmoid-gate epilogue (gnnea_spmm_highway_f32)
Handed a ``gnnea.dist_graph.DistAdj`` instead of the sparse adjacency (and the rank's own rows
of x), the same layers run row-sharded across GPUs with the RCCL halo exchange.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn.modules.module import Module

from gnnea import _lib, ops
from gnnea.dist_graph import DistAdj
from gnnea.graph import dense_of


def get_dim_act(args):
    """Per-layer dims and activations (reference layers/layers.py:8-16)."""
    act = getattr(F, args.act) if args.act else (lambda x: x)
    n = args.num_layers - 1
    return [args.feat_dim] + [args.dim] * n, [act] * n


def _propagate(adj, hidden, act):
    if isinstance(adj, DistAdj):  # row shard of a multi-GPU run (gnnea/dist_graph.py)
        return adj.aggregate(hidden, act)
    if adj.is_sparse:
        return ops.aggregate(adj, hidden, act)
    return act(ops.matmul(adj, hidden))  # dense adjacency: torch.mm branch (:37)


class GraphConvolution(Module):
    """out = act(A · dropout(x W^T + b)); forward((x, adj)) -> (out, adj)  (:19-42)."""

    def __init__(self, in_features, out_features, dropout, act, use_bias):
        super(GraphConvolution, self).__init__()
        self.dropout = dropout
        self.linear = nn.Linear(in_features, out_features, use_bias)
        self.act = act
        self.in_features = in_features
        self.out_features = out_features

    def _hidden(self, x):
        h = ops.linear(x, self.linear.weight, self.linear.bias)
        return F.dropout(h, self.dropout, training=self.training)

    def forward(self, input):
        x, adj = input
        x = dense_of(x)
        if (isinstance(adj, DistAdj) or adj.is_sparse) and \
                (self.dropout == 0 or not self.training):
            out = ops.gcn_layer(adj, x, self.linear.weight, self.linear.bias, self.act)
            if out is not None:  # hidden kept slice-major (gnnea.ops.GCNLayerFn)
                return out, adj
        return _propagate(adj, self._hidden(x), self.act), adj

    def extra_repr(self):
        return 'input_dim={}, output_dim={}'.format(self.in_features, self.out_features)


class HighWayGraphConvolution(GraphConvolution):
    """GCN layer with a HighWay gate (:45-80):
    g = sigmoid(x K_g + b_g); out = g * act(A · hidden) + (1 - g) * x.
    K_g / b_g are plain tensors (not parameters, not saved) drawn after the Linear init."""

    def __init__(self, in_features, out_features, dropout, act, use_bias, cuda, device):
        super(HighWayGraphConvolution, self).__init__(in_features, out_features, dropout, act,
                                                      use_bias)
        assert self.in_features == self.out_features
        d = self.in_features
        bound = np.sqrt(6.0 / (d + d))
        self.kernel_gate = torch.FloatTensor(d, d).uniform_(-bound, bound)
        self.bias_gate = torch.zeros([d])
        if cuda != -1:
            self.kernel_gate = self.kernel_gate.to(device)
            self.bias_gate = self.bias_gate.to(device)

    def forward(self, input):
        x, adj = input
        x = dense_of(x)
        if (isinstance(adj, DistAdj) or adj.is_sparse) and \
                (self.dropout == 0 or not self.training):
            out = ops.highway_layer(adj, x, self.linear.weight, self.linear.bias,
                                    self.kernel_gate, self.bias_gate, self.act)
            if out is not None:  # one GEMM each way (gnnea.ops.HighwayLayerFn)
                return out, adj
        hidden = self._hidden(x)
        gate_pre = ops.matmul(x, self.kernel_gate)
        if isinstance(adj, DistAdj):
            out = adj.highway(hidden, gate_pre, x, self.bias_gate, self.act)
        elif adj.is_sparse:
            out = ops.highway(adj, hidden, gate_pre, x, self.bias_gate, self.act)
        else:
            s = self.act(ops.matmul(adj, hidden))
            g = torch.sigmoid(gate_pre + self.bias_gate)
            out = g * s + (1.0 - g) * x
        return out, adj

    def extra_repr(self):
        return 'input_dim={}, output_dim={}'.format(self.in_features, self.out_features)


class Linear(Module):
    """act(dropout(x W^T + b)) (:83-96), GEMM on MFMA."""

    def __init__(self, in_features, out_features, dropout, act, use_bias):
        super(Linear, self).__init__()
        self.dropout = dropout
        self.linear = nn.Linear(in_features, out_features, use_bias)
        self.act = act

    def forward(self, x):
        code = ops.act_code(self.act)
        drop = self.training and self.dropout > 0
        # the act in the GEMM epilogue when that is the same value: always without dropout, and
        # for relu also with it (relu(s·h) = s·relu(h) for the dropout's scale s >= 0)
        if code is not None and code != _lib.GNNEA_ACT_IDENTITY and \
                (not drop or code == _lib.GNNEA_ACT_RELU):
            h = ops.linear(dense_of(x), self.linear.weight, self.linear.bias, act=code)
            return F.dropout(h, self.dropout, training=self.training)
        h = ops.linear(dense_of(x), self.linear.weight, self.linear.bias)
        return self.act(F.dropout(h, self.dropout, training=self.training))
