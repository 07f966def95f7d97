"""Decoder heads (drop-in for the reference models/decoders.py).

For entity alignment the GCN/GAT models decode with three dense Linear layers (MFMA GEMMs) and
HGCN decodes with one more HighWay graph convolution (a third SpMM per forward).
"""
import torch.nn as nn
import torch.nn.functional as F

from gnnea import _lib, ops

from layers.att_layers import GraphAttentionLayer
from layers.layers import GraphConvolution, HighWayGraphConvolution, Linear, dense_of


def _identity(x):
    return x


# the reference's identity act (models/decoders.py:26,45 ``lambda x: x``) is fused as the
# kernels' identity epilogue rather than applied as a torch op after the aggregation
ops.ACT_CODES[_identity] = _lib.GNNEA_ACT_IDENTITY


class Decoder(nn.Module):
    decode_adj = True

    def decode(self, x, adj):
        if not self.decode_adj:
            return self.cls.forward(x)
        probs, _ = self.cls.forward((x, adj))
        return probs


class GCNDecoder(Decoder):
    def __init__(self, args):
        super(GCNDecoder, self).__init__()
        self.cls = GraphConvolution(args.dim, args.n_classes, args.dropout, _identity, args.bias)
        self.decode_adj = True


class GATDecoder(Decoder):
    def __init__(self, args):
        super(GATDecoder, self).__init__()
        self.cls = GraphAttentionLayer(args.dim, args.n_classes, args.dropout, F.elu, args.alpha,
                                       1, True)
        self.decode_adj = True


class HGCNDecoder(Decoder):
    def __init__(self, args):
        super(HGCNDecoder, self).__init__()
        self.cls = HighWayGraphConvolution(args.dim, args.n_classes, args.dropout, _identity,
                                           args.bias, args.cuda, args.device)
        self.decode_adj = True


class MLPDecoder(Decoder):
    def __init__(self, args):
        super(MLPDecoder, self).__init__()
        widths = [args.dim, args.dim, args.dim, args.n_classes]
        acts = [F.relu, F.relu, _identity]
        self.cls = nn.Sequential(*[Linear(widths[k], widths[k + 1], args.dropout, acts[k],
                                          args.bias) for k in range(3)])
        self.decode_adj = False

    def decode(self, x, adj):
        # the three layers as one autograd node (ops.MLPChainFn: the backward masks each relu
        # layer's gradient in the epilogue of the product that produces it); per layer otherwise
        out = ops.mlp_chain(dense_of(x), self.cls)
        return out if out is not None else self.cls.forward(x)


class LinearDecoder(Decoder):
    def __init__(self, args):
        super(LinearDecoder, self).__init__()
        self.cls = nn.Sequential(Linear(2 * args.dim, args.n_classes, args.dropout, _identity,
                                        args.bias))
        self.decode_adj = False


model2decoder = {'GCN': MLPDecoder, 'GAT': MLPDecoder, 'HGCN': HGCNDecoder, 'Distill': HGCNDecoder}
