"""Entity-alignment models (drop-in for the reference models/models_ea.py).

The hard-negative search (get_neg), the metrics (compute_metrics -> get_hits) and the
pseudo-pair search (generate_pairs) run on the device through the L1 kernels (gnnea.l1): fp64
cityblock distances equal to scipy's, selections ordered by (distance, index).  The reference
copies the embeddings to the host and builds the full t x n distance matrix with scipy for each of
them (models/models_ea.py:19-30, 63-64, 143-167).
"""
import random

import numpy as np
import torch
import torch.nn as nn

from gnnea import dist_search, l1, margin
from gnnea.dist_graph import DistAdj
from gnnea.dist_loss import sharded_margin_loss
from models.decoders import model2decoder
from models.encoders import model2encoder
from utils.eval_utils import get_hits
from utils.ot_loss import sinkhorn


def _index(idx, device, n_rows):
    """Checked device int64 copy of a host index array, cached per array (negatives are
    regenerated every 50 epochs; the loss reads them, and views data[split][:, 0] of the same
    pair array, every epoch): gnnea.margin._idx_cached."""
    return margin._idx_cached(idx, device, n_rows)


def margin_loss(outputs, left, right, neg_left, neg_right, neg2_left, neg2_right, t, k):
    """models/models_ea.py:105-124 (fused gather-L1-hinge kernels, gnnea.margin)."""
    if neg_right is None or neg2_left is None:
        raise ValueError("get_loss: negatives are not set (get_neg runs every 50 epochs)")
    n, dev = outputs.shape[0], outputs.device
    idx = [_index(a, dev, n) for a in (left, right, neg_left, neg_right, neg2_left, neg2_right)]
    return margin.margin_loss(outputs, *idx, t, k, checked=True)


class BaseModel(nn.Module):
    """models/models_ea.py:10-85"""

    def __init__(self, args):
        super(BaseModel, self).__init__()
        self.n_nodes = args.n_nodes
        self.device = args.device

    def _shard(self, output):
        """The DistAdj of the last encode when ``output`` is this rank's rows of a row-sharded
        output (several ranks), else None (a gathered or single-GPU output)."""
        dadj = getattr(self, "_dadj", None)
        if dadj is not None and dadj.part.world > 1 and output.shape[0] == dadj.part.n_rows:
            return dadj
        return None

    def get_neg(self, ILL, output, k):
        """The k L1-nearest entities of each ILL entity, nearest first, the entity itself (rank 0)
        excluded; flattened to t*k (models/models_ea.py:19-30).  On a row-sharded output (the
        rank's rows after a DistAdj encode): every rank searches its own rows, the per-rank lists
        are merged (gnnea.dist_search; index-exact with the single-GPU search)."""
        dadj = self._shard(output) if self is not None else None
        if dadj is not None:
            return dist_search.get_neg(ILL, output, dadj.part, k)
        out = output.detach()
        if not out.is_cuda and torch.cuda.is_available():
            out = out.to("cuda")
        rows = _index(np.asarray(ILL), out.device, out.shape[0])
        neg = l1.topk(out[rows], out, k + 1, skip=1)
        return neg.reshape(-1).cpu().numpy()

    def get_neg_triplet(self, triples, head, tail, ids):
        """models/models_ea.py:32-55 (host sampling; unused by the training scripts)."""
        neg = []
        for (h, r, t) in triples:
            h2, t2 = h, t
            in_scope, tries = True, 0
            while True:
                if random.randint(0, 999) < 500:
                    h2 = random.sample(head[r], 1)[0] if in_scope else \
                        random.sample(range(ids), 1)[0]
                else:
                    t2 = random.sample(tail[r], 1)[0] if in_scope else \
                        random.sample(range(ids), 1)[0]
                if (h2, r, t2) not in triples:
                    break
                tries += 1
                if tries > 10:
                    in_scope = False
            neg.append((h2, r, t2))
        return neg

    def compute_metrics(self, outputs, data, split):
        pair = data["train"] if split == "train" else data["test"]
        dadj = self._shard(outputs) if self is not None else None
        if dadj is not None:  # row-sharded output: per-rank candidate blocks, counts summed
            return dist_search.get_hits(outputs, dadj.part, pair, top_k=[1])
        return get_hits(outputs, pair, top_k=[1])

    def has_improved(self, m1, m2):
        return (m1["Hits@10_l"] < m2["Hits@10_l"]) or (m1["Hits@10_r"] < m2["Hits@10_r"])

    def init_metric_dict(self):
        return {"Hits@1_l": -1, "Hits@10_l": -1, "Hits@50_l": -1, "Hits@100_l": -1,
                "Hits@1_r": -1, "Hits@10_r": -1, "Hits@50_r": -1, "Hits@100_r": -1}


def _repeat_col(col, k):
    """np.ones((t, k)) * col[:, None] flattened (float64, as the reference builds it)."""
    t = len(col)
    return (np.ones((t, k)) * np.asarray(col).reshape((t, 1))).reshape((t * k,))


class EAModel(BaseModel):
    """models/models_ea.py:88-124"""

    def __init__(self, args):
        super(EAModel, self).__init__(args)
        self.encoder = model2encoder[args.model](args)
        self.decoder = model2decoder[args.model](args)
        ILL = args.data["train"]
        self.neg_num = args.neg_num
        self.neg_left = _repeat_col(ILL[:, 0], self.neg_num)
        self.neg2_right = _repeat_col(ILL[:, 1], self.neg_num)
        self.neg_right = None
        self.neg2_left = None

    def encode(self, x, adj):
        # a row-sharded adjacency of several ranks (gnnea.dist_graph.DistAdj): get_loss then
        # evaluates the loss column-sharded on the rank's output rows (gnnea.dist_loss)
        self._dadj = adj if isinstance(adj, DistAdj) and adj.part.world > 1 else None
        return self.encoder.encode(x, adj)

    def decode(self, h, adj):
        return self.decoder.decode(h, adj)

    def get_loss(self, outputs, data, split):
        ILL = data[split]
        dadj = getattr(self, "_dadj", None)
        if dadj is not None and outputs.shape[0] == dadj.part.n_rows:
            return sharded_margin_loss(outputs, dadj, ILL[:, 0], ILL[:, 1], self.neg_left,
                                       self.neg_right, self.neg2_left, self.neg2_right, len(ILL),
                                       self.neg_num)
        return margin_loss(outputs, ILL[:, 0], ILL[:, 1], self.neg_left, self.neg_right,
                           self.neg2_left, self.neg2_right, len(ILL), self.neg_num)


class UEAModel(BaseModel):
    """models/models_ea.py:127-235 (unsupervised: pseudo pairs from mutual L1 nearest
    neighbours, optional Wasserstein / Gromov-Wasserstein terms)."""

    def __init__(self, args):
        super(UEAModel, self).__init__(args)
        self.ILL = None
        self.encoder = model2encoder[args.model](args)
        self.decoder = model2decoder[args.model](args)

    def encode(self, x, adj):
        return self.encoder.encode(x, adj)

    def decode(self, h, adj):
        return self.decoder.decode(h, adj)

    def generate_pairs(self, outputs, data, bsz):
        """Mutual nearest neighbours of the two entity sets under L1, best bsz by distance
        (pairs are (left position, right position), as the reference stores them)."""
        e1, e2 = data["e1"], data["e2"]
        index1, index2 = data["index1"], data["index2"]
        out = outputs.detach()
        if not out.is_cuda and torch.cuda.is_available():
            out = out.to("cuda")
        dev = out.device
        Lx = out[torch.as_tensor([index1[i] for i in range(e1)], dtype=torch.int64, device=dev)]
        Rx = out[torch.as_tensor([index2[i] for i in range(e2)], dtype=torch.int64, device=dev)]
        idx_l2r, v_l2r = l1.nearest(Lx, Rx)
        idx_r2l, _ = l1.nearest(Rx, Lx)
        left = torch.arange(e1, device=dev)
        mutual = idx_r2l[idx_l2r] == left
        pairs = torch.stack([left[mutual], idx_l2r[mutual]], 1)
        scores = v_l2r[mutual]
        print("generate {} pairs by the L1 distance".format(min(len(pairs), bsz)))
        order = torch.sort(scores, stable=True).indices[:bsz]
        self.ILL = pairs[order].cpu().numpy()

    def generate_neg(self, outputs, k):
        t = len(self.ILL)
        self.neg_num = k
        self.neg_left = _repeat_col(self.ILL[:, 0], k)
        self.neg2_right = _repeat_col(self.ILL[:, 1], k)
        self.neg_right = self.get_neg(self.ILL[:, 0], outputs, k)
        self.neg2_left = self.get_neg(self.ILL[:, 1], outputs, k)
        assert len(self.neg_right) == t * k

    def get_loss(self, outputs):
        return margin_loss(outputs, self.ILL[:, 0], self.ILL[:, 1], self.neg_left,
                           self.neg_right, self.neg2_left, self.neg2_right, len(self.ILL),
                           self.neg_num)

    @staticmethod
    def _sample(data, bsz, outputs):
        e1, e2 = data["e1"], data["e2"]
        index1, index2 = data["index1"], data["index2"]
        L = np.array([index1[i] for i in np.random.permutation(e1)[:bsz]])
        R = np.array([index2[i] for i in np.random.permutation(e2)[:bsz]])
        return outputs[L], outputs[R]

    def get_loss_wassertein(self, outputs, data, bsz):
        """models/models_ea.py:185-205, including its one-hot of argmax(zeros) (column 0)."""
        X, Y = self._sample(data, bsz, outputs)
        device = outputs.device
        a, b = torch.ones(bsz).to(device), torch.ones(bsz).to(device)
        M = torch.cdist(X, Y, p=2)
        T, _ = sinkhorn(a, b, M.detach(), reg=0.01)
        newT = torch.zeros_like(T).to(device)
        newT[torch.arange(len(newT)), torch.argmax(newT, dim=1)] = 1
        return torch.sum(newT * M)

    def get_loss_gromove_wassertein(self, outputs, data, bsz):
        """models/models_ea.py:207-225 (GW solver from SinkhornOT, §8f #3)."""
        from SinkhornOT import gw_iterative_1
        X, Y = self._sample(data, bsz, outputs)
        device = outputs.device
        a, b = torch.ones(bsz).to(device), torch.ones(bsz).to(device)
        M = torch.cdist(X, Y, p=1)
        C1 = torch.cdist(X, X, p=1).detach()
        C2 = torch.cdist(Y, Y, p=1).detach()
        T, gwdist = gw_iterative_1(C1, C2, a, b, epsilon=0.01, max_iter=1000)
        newT = torch.zeros_like(T[0]).to(device)
        newT[torch.arange(len(newT)), torch.argmax(newT, dim=1)] = 1
        return torch.sum(newT * M)
