"""Drop-in sparse GAT layers backed by libgnnea (reference: layers/att_layers.py).

The reference runs each head separately and materialises cat(h[row], h[col]) per head
(att_layers.py:38).  Here all heads of a GraphAttentionLayer share one MFMA projection
(x · [W_0|...|W_{H-1}]) and ONE edge pass (gnnea_gat_fwd_f32) whose output is already the
head-concatenated tensor of :86.  Parameters (``attention_{i}.W``, ``attention_{i}.a``), their
xavier_normal init order and the dropout calls keep the reference's names and RNG order.
Handed a ``gnnea.dist_graph.DistAdj`` (and the rank's own rows of x) the layers run row-sharded
with the halo all-gather of the projected rows (dropout inactive).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from gnnea import ops
from gnnea.dist_graph import DistAdj
from gnnea.graph import csr_of, dense_of


def _sharded_gat(adj, H, a_all, heads, d_head, alpha, act, p, training):
    """Row shard of a multi-GPU run (gnnea.dist_graph.DistAdj): halo all-gather of H."""
    if training and p > 0.0:
        raise NotImplementedError("gnnea: edge dropout on a row-sharded adjacency")
    return adj.gat(H, a_all, heads, d_head, alpha, act)


def _edge_dropout(nnz, p, training, device, heads):
    """Per-head edge masks, drawn in head order like the per-head nn.Dropout (:51)."""
    if not training or p == 0.0:
        return None
    ones = torch.ones(nnz, dtype=torch.float32, device=device)
    return torch.stack([F.dropout(ones, p, training=True) for _ in range(heads)], dim=1)


class SpGraphAttentionLayer(nn.Module):
    """One sparse GAT head (:8-64): h' = act(softmax_j(-LeakyReLU(a·[Wx_i || Wx_j])) · Wx)."""

    def __init__(self, in_features, out_features, dropout, alpha, activation):
        super(SpGraphAttentionLayer, self).__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.alpha = alpha
        self.W = nn.Parameter(torch.zeros(size=(in_features, out_features)))
        nn.init.xavier_normal_(self.W.data, gain=1.414)
        self.a = nn.Parameter(torch.zeros(size=(1, 2 * out_features)))
        nn.init.xavier_normal_(self.a.data, gain=1.414)
        self.dropout = nn.Dropout(dropout)
        self.leakyrelu = nn.LeakyReLU(self.alpha)
        self.act = activation

    def forward(self, input, adj):
        x = dense_of(input)
        h = ops.matmul(x, self.W)
        if isinstance(adj, DistAdj):
            return _sharded_gat(adj, h, self.a.view(1, -1), 1, self.out_features, self.alpha,
                                self.act, self.dropout.p, self.training)
        csr = csr_of(adj)
        mask = _edge_dropout(csr.nnz, self.dropout.p, self.training, h.device, 1)
        return ops.gat(adj, h, self.a.view(1, -1), 1, self.out_features, self.alpha, self.act,
                       mask)

    def __repr__(self):
        return self.__class__.__name__ + ' (' + str(self.in_features) + ' -> ' + \
            str(self.out_features) + ')'


class GraphAttentionLayer(nn.Module):
    """Multi-head sparse GAT (:67-91): forward((x, adj)) -> (h, adj); concat or mean of heads."""

    def __init__(self, input_dim, output_dim, dropout, activation, alpha, nheads, concat):
        super(GraphAttentionLayer, self).__init__()
        self.dropout = dropout
        self.output_dim = output_dim
        self.attentions = [SpGraphAttentionLayer(input_dim, output_dim, dropout=dropout,
                                                 alpha=alpha, activation=activation)
                           for _ in range(nheads)]
        self.concat = concat
        for i, head in enumerate(self.attentions):
            self.add_module('attention_{}'.format(i), head)

    def forward(self, input):
        x, adj = input
        x = F.dropout(dense_of(x), self.dropout, training=self.training)
        heads = len(self.attentions)
        first = self.attentions[0]
        W_all = torch.cat([att.W for att in self.attentions], dim=1)
        a_all = torch.cat([att.a for att in self.attentions], dim=0)  # [heads, 2*d_head]
        # above the Infinity Cache the GEMM also writes H slice-major for the GAT forward
        # (a row shard exchanges row-major H: only without exchange), only when the forward
        # takes the sliced passes for this shape (ops.gat_sliced_wanted)
        H = ops.matmul(x, W_all, sliced=(not isinstance(adj, DistAdj) or adj.part.g == 1)
                       and ops.gat_sliced_wanted(x.shape[0], heads, self.output_dim, x.dtype))
        if isinstance(adj, DistAdj):
            y = _sharded_gat(adj, H, a_all, heads, self.output_dim, first.alpha, first.act,
                             self.dropout, self.training)
        else:
            mask = _edge_dropout(csr_of(adj).nnz, self.dropout, self.training, H.device, heads)
            y = ops.gat(adj, H, a_all, heads, self.output_dim, first.alpha, first.act, mask)
        if not self.concat:  # mean of the heads (:89-91), one pass each way
            y = ops.head_mean(y, heads, self.output_dim)
        y = F.dropout(y, self.dropout, training=self.training)
        return (y, adj)
