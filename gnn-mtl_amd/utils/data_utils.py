"""Entity-alignment input pipeline (reference utils/data_utils.py:51-57, 272-455; §8f #4).

The adjacency builders (``get_matrix``, ``get_sparse_tensor``, ``get_sparse_tensor_for_one_graph``,
``sparse_mx_to_torch_sparse_tensor``) and the EA loaders (``loadfile``, ``rfunc``,
``get_features``, ``load_data_ea``, ``load_seperate_data_ea``, ``load_data``) keep the reference's
signatures and outputs; the per-line / per-triple Python loops are replaced by the C++ host
library (gnnea.ingest: parallel parsing, counting-sort adjacency in the reference's dict order)
and vectorised numpy / scipy.  Entry order and fp32 values of the adjacency are bit-identical
(tests/test_adjacency.py, tests/test_ingest.py).  The other task loaders of the reference module
(node classification, text) are out of scope.
"""
import json

import numpy as np
import scipy.sparse as sp
import torch
import torch.nn.functional as F

from gnnea import ingest, synth

# dense rfunc incidence matrices above this many entries are returned as scipy CSR instead
DENSE_INCIDENCE_LIMIT = 1 << 28


def sparse_mx_to_torch_sparse_tensor(sparse_mx):
    """scipy sparse -> uncoalesced torch sparse COO (int64 indices, fp32 values), order kept."""
    sparse_mx = sparse_mx.tocoo()
    indices = torch.from_numpy(np.vstack((sparse_mx.row, sparse_mx.col)).astype(np.int64))
    values = torch.from_numpy(np.asarray(sparse_mx.data).astype(np.float32))
    return torch.sparse_coo_tensor(indices, values, torch.Size(sparse_mx.shape))


def get_matrix(e, KG):
    """(M, degree) dicts as the reference builds them (:296-321)."""
    tr = np.asarray(KG, dtype=np.int64).reshape(-1, 3)
    row, col, _ = synth.adjacency_coo(tr, int(max(e, tr[:, [0, 2]].max() + 1 if len(tr) else 0)))
    M = {(int(r), int(c)): 1 for r, c in zip(row.tolist(), col.tolist())}
    h, t = tr[:, 0], tr[:, 2]
    ns = h != t
    ents, first = np.unique(np.stack([h, t], 1).reshape(-1), return_index=True)
    ents = ents[np.argsort(first, kind="stable")]
    cnt = np.bincount(np.concatenate([h[ns], t[ns]]), minlength=int(ents.max()) + 1 if len(ents) else 0)
    degree = {int(i): 1 + int(cnt[i]) for i in ents.tolist()}
    return M, degree


def get_sparse_tensor(e, KG):
    """Normalised adjacency as a scipy COO matrix (:325-336), built by the C++ host library."""
    print('getting a sparse tensor...')
    tr = np.asarray(KG, dtype=np.int64).reshape(-1, 3)
    row, col, val = ingest.adjacency(tr, e, reference_order=True)
    return sp.coo_matrix((val.astype(np.float64), (row, col)), shape=(e, e))


def get_sparse_tensor_for_one_graph(e, KG, index_R):
    """Single-KG adjacency with ids remapped by index_R (:339-350)."""
    tr = np.asarray(KG, dtype=np.int64).reshape(-1, 3)
    n_raw = int(tr[:, [0, 2]].max()) + 1 if len(tr) else 0
    row, col, val = synth.adjacency_coo(tr, n_raw)
    lut = np.full(n_raw, -1, dtype=np.int64)
    for k, v in index_R.items():
        if k < n_raw:
            lut[k] = v
    return sp.coo_matrix((val.astype(np.float64), (lut[row], lut[col])), shape=(e, e))


def loadfile(fn, num=1):
    """(:362-372) list of int tuples, one per line (parsed by the C++ host library)."""
    print('loading a file...' + fn)
    return [tuple(r) for r in ingest.loadfile_array(fn, num).tolist()]


def rfunc(e, KG):
    """(:272-293) per-relation head / tail lists (relations in order of first appearance, triples
    in order) and the entity x relation incidence indicators head_r / tail_r.  The indicators are
    dense float64 as in the reference up to DENSE_INCIDENCE_LIMIT entries, scipy CSR beyond."""
    tr = np.asarray(KG, dtype=np.int64).reshape(-1, 3)
    n_rel_ids = int(tr[:, 1].max()) + 1 if len(tr) else 0
    ptr, heads, tails = ingest.relation_groups(tr, n_rel_ids)
    rels, first = np.unique(tr[:, 1], return_index=True)
    order = rels[np.argsort(first, kind="stable")]
    head = {int(r): heads[ptr[r]:ptr[r + 1]].tolist() for r in order.tolist()}
    tail = {int(r): tails[ptr[r]:ptr[r + 1]].tolist() for r in order.tolist()}
    r_num = len(head)
    if int(e) * r_num <= DENSE_INCIDENCE_LIMIT:
        head_r = np.zeros((e, r_num))
        tail_r = np.zeros((e, r_num))
        head_r[tr[:, 0], tr[:, 1]] = 1
        tail_r[tr[:, 2], tr[:, 1]] = 1
    else:
        ones = np.ones(len(tr))
        head_r = sp.csr_matrix((ones, (tr[:, 0], tr[:, 1])), shape=(e, r_num))
        tail_r = sp.csr_matrix((ones, (tr[:, 2], tr[:, 1])), shape=(e, r_num))
        head_r.data[:] = 1
        tail_r.data[:] = 1
    return head, tail, head_r, tail_r


def get_features(lang):
    """(:353-358) row-normalised entity vectors of data/dbp15k/{lang}_en/{lang}_vectorList.json."""
    print('adding the primal input layer...')
    with open(file='data/dbp15k/' + lang + '_en/' + lang + '_vectorList.json', mode='r',
              encoding='utf-8') as f:
        embedding_list = json.load(f)
        print(len(embedding_list), 'rows,', len(embedding_list[0]), 'columns.')
    ent_embeddings = torch.Tensor(embedding_list)
    return sp.coo_matrix(F.normalize(ent_embeddings, 2, 1))


def _relation_features(feat, tr, r):
    """features_r[rel] = (sum feat[tails of rel] - sum feat[heads of rel]) / #triples of rel
    (:404-406) with sparse incidence products instead of a Python loop over relations."""
    n = feat.shape[0]
    cnt = np.bincount(tr[:, 1], minlength=r).astype(np.float32)
    ones = np.ones(len(tr), dtype=np.float32)
    Ht = sp.csr_matrix((ones, (tr[:, 1], tr[:, 0])), shape=(r, n))
    Tt = sp.csr_matrix((ones, (tr[:, 1], tr[:, 2])), shape=(r, n))
    f = feat.numpy()
    out = (np.asarray(Tt @ f) - np.asarray(Ht @ f)) / cnt[:, None]
    return torch.from_numpy(out.astype(np.float32))


def load_data_ea(args):
    """(:375-413) DBP15K-format entity-alignment data of args.dataset."""
    lang = args.dataset  # zh_en | ja_en | fr_en
    base = 'data/dbp15k/' + lang + '/'
    e = len(set(loadfile(base + 'ent_ids_1', 1)) | set(loadfile(base + 'ent_ids_2', 1)))
    r = len(set(loadfile(base + 'rel_ids_1', 1)) | set(loadfile(base + 'rel_ids_2', 1)))
    ILL = loadfile(base + 'ref_ent_ids', 2)
    illL = len(ILL)
    np.random.shuffle(ILL)
    train = np.array(ILL[:illL // 10 * 3])
    test = np.array(ILL[illL // 10 * 3:])
    test_r = loadfile(base + 'ref_r_ids', 2)
    KG = loadfile(base + 'triples_1', 3) + loadfile(base + 'triples_2', 3)
    tr = np.asarray(KG, dtype=np.int64).reshape(-1, 3)

    features = sparse_mx_to_torch_sparse_tensor(get_features(lang[0:2]))
    M = sparse_mx_to_torch_sparse_tensor(get_sparse_tensor(e, KG))
    head, tail, head_r, tail_r = rfunc(e, KG)
    features_r = _relation_features(features.to_dense(), tr, r).to_sparse()
    data = {'x': features, 'adj': M, 'r': features_r, 'train': train, 'test': test,
            'test_r': test_r, 'triple': KG, 'head': head, 'tail': tail, 'head_r': head_r,
            'tail_r': tail_r, 'idx_x': torch.LongTensor(range(features.shape[0])),
            'idx_r': torch.LongTensor(range(features_r.shape[0]))}
    if args.model == 'Distill':
        print('loading TransE embeddings...')
        data['emb'] = torch.from_numpy(np.load(f'data/dbp15k/{args.dataset}/TransE_embeddings.npy'))
        print(data['emb'].shape[0], 'rows', data['emb'].shape[1], 'columns')
    return data


def load_seperate_data_ea(args):
    """(:416-455) the two KGs separately (unsupervised / GW alignment) plus the joint graph."""
    lang = args.dataset
    base = 'data/dbp15k/' + lang + '/'
    index1, index1_R, index2, index2_R = {}, {}, {}, {}
    for i, v in enumerate(loadfile(base + 'ent_ids_1', 1)):
        index1[i] = v[0]
        index1_R[v[0]] = i
    for i, v in enumerate(loadfile(base + 'ent_ids_2', 1)):
        index2[i] = v[0]
        index2_R[v[0]] = i
    E1, E2 = len(index1), len(index2)
    KG1, KG2 = loadfile(base + 'triples_1', 3), loadfile(base + 'triples_2', 3)
    KG = KG1 + KG2
    M1 = sparse_mx_to_torch_sparse_tensor(get_sparse_tensor_for_one_graph(E1, KG1, index1_R))
    M2 = sparse_mx_to_torch_sparse_tensor(get_sparse_tensor_for_one_graph(E2, KG2, index2_R))
    M = sparse_mx_to_torch_sparse_tensor(get_sparse_tensor(E1 + E2, KG))
    ILL = loadfile(base + 'ref_ent_ids', 2)
    illL = len(ILL)
    np.random.shuffle(ILL)
    train = np.array(ILL[:illL // 10 * 3])
    test = np.array(ILL[illL // 10 * 3:])
    features = sparse_mx_to_torch_sparse_tensor(get_features(lang[0:2]))
    return {'x': features, 'adj': M, 'e1': E1, 'e2': E2, 'adj1': M1, 'adj2': M2,
            'train': train, 'test': test, "index1": index1, "index2": index2,
            "index1_R": index1_R, "index2_R": index2_R}


def load_data(args):
    """(:17-26) task dispatch; only the entity-alignment task is on this tier's path."""
    if args.task == 'ea':
        return load_data_ea(args)
    raise NotImplementedError("gnnea: only task 'ea' is rebuilt (the reference's NC / LP / text "
                              "loaders are out of scope, DESIGN.md §7); got task %r" % args.task)
