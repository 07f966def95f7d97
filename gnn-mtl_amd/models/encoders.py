"""Graph encoders (drop-in for the reference models/encoders.py).

Each encoder stacks ``num_layers - 1`` layers in an ``nn.Sequential`` called ``layers`` (so the
state_dict keys are ``layers.{i}....`` as in the reference) and exposes ``encode(x, adj)``.
"""
import torch.nn as nn

from layers.att_layers import GraphAttentionLayer
from layers.layers import GraphConvolution, HighWayGraphConvolution, Linear, get_dim_act


class Encoder(nn.Module):
    """encode(x, adj): graph encoders consume (x, adj) tuples, the MLP consumes x."""

    encode_graph = True

    def encode(self, x, adj):
        if not self.encode_graph:
            return self.layers.forward(x)
        out, _ = self.layers.forward((x, adj))
        return out


def _stack(args, make):
    assert args.num_layers > 0
    dims, acts = get_dim_act(args)
    return nn.Sequential(*[make(d_in, d_out, act)
                           for d_in, d_out, act in zip(dims[:-1], dims[1:], acts)])


class MLP(Encoder):
    encode_graph = False

    def __init__(self, args):
        super(MLP, self).__init__()
        self.layers = _stack(args, lambda i, o, act: Linear(i, o, args.dropout, act, args.bias))
        self.encode_graph = False


class GCN(Encoder):
    def __init__(self, args):
        super(GCN, self).__init__()
        self.layers = _stack(
            args, lambda i, o, act: GraphConvolution(i, o, args.dropout, act, args.bias))
        self.encode_graph = True


class HGCN(Encoder):
    def __init__(self, args):
        super(HGCN, self).__init__()
        self.layers = _stack(
            args, lambda i, o, act: HighWayGraphConvolution(i, o, args.dropout, act, args.bias,
                                                            args.cuda, args.device))
        self.encode_graph = True


class GAT(Encoder):
    def __init__(self, args):
        super(GAT, self).__init__()

        def make(i, o, act):
            assert o % args.n_heads == 0
            return GraphAttentionLayer(i, o // args.n_heads, args.dropout, act, args.alpha,
                                       args.n_heads, True)

        self.layers = _stack(args, make)
        self.encode_graph = True


model2encoder = {'GCN': GCN, 'GAT': GAT, 'HGCN': HGCN, 'Distill': HGCN}
