"""Writes a small DBP15K-format dataset (the files utils/data_utils.py:375-455 read) under
<root>/data/dbp15k/: ent_ids_1/2, rel_ids_1/2, ref_ent_ids, ref_r_ids, triples_1/2 and
zz_en/zz_vectorList.json.  Deterministic (seeded); used by tests/golden/gen_golden.py to run
the reference loaders and by tests/test_ingest.py to run the drop-in ones on the same files."""
import json
import os

import numpy as np

LANG = "zz_en"


def write(root, seed=0):
    rng = np.random.default_rng(seed)
    d = os.path.join(root, "data", "dbp15k", LANG)
    os.makedirs(d, exist_ok=True)
    n1, n2, r1, r2 = 300, 280, 20, 15
    e1 = np.arange(n1)
    e2 = np.arange(n1, n1 + n2)
    rel1 = np.arange(r1)
    rel2 = np.arange(r1, r1 + r2)

    def lines(path, rows):
        with open(os.path.join(d, path), "w", encoding="utf-8") as f:
            for row in rows:
                f.write("\t".join(str(x) for x in row) + "\n")

    lines("ent_ids_1", [(i, "http://kg1/e%d" % i) for i in e1])
    lines("ent_ids_2", [(i, "http://kg2/e%d" % i) for i in e2])
    lines("rel_ids_1", [(i, "http://kg1/r%d" % i) for i in rel1])
    lines("rel_ids_2", [(i, "http://kg2/r%d" % i) for i in rel2])

    def triples(ents, rels, t):
        h = rng.choice(ents, t)
        tt = rng.choice(ents, t)
        r = rng.choice(rels, t)
        tr = np.stack([h, r, tt], 1)
        tr[5] = (tr[5, 0], tr[5, 1], tr[5, 0])   # a self-loop triple
        tr[9] = tr[3]                             # a repeated triple (multi-edge degree)
        tr[11] = (tr[3, 2], tr[11, 1], tr[3, 0])  # the reverse of another
        return tr

    lines("triples_1", triples(e1, rel1, 900))
    lines("triples_2", triples(e2, rel2, 800))
    pairs = np.stack([rng.permutation(e1)[:200], rng.permutation(e2)[:200]], 1)
    lines("ref_ent_ids", pairs)
    lines("ref_r_ids", np.stack([rel1[:10], rel2[:10]], 1))
    vec = rng.standard_normal((n1 + n2, 16))
    with open(os.path.join(root, "data", "dbp15k", "zz_vectorList.json"), "w") as f:
        json.dump(vec.tolist(), f)
    # get_features reads data/dbp15k/{lang[0:2]}_en/{lang[0:2]}_vectorList.json
    os.replace(os.path.join(root, "data", "dbp15k", "zz_vectorList.json"),
               os.path.join(d, "zz_vectorList.json"))
    return LANG


def flatten(data, sep):
    """Flatten the loaders' outputs into arrays (shared with tests/test_ingest.py)."""
    out = {}
    adj = data["adj"]
    out["adj_idx"] = adj._indices().numpy()
    out["adj_val"] = adj._values().numpy()
    out["x"] = data["x"].to_dense().numpy()
    out["r"] = data["r"].to_dense().numpy()
    out["train"], out["test"] = np.asarray(data["train"]), np.asarray(data["test"])
    out["test_r"] = np.asarray(data["test_r"])
    out["triple"] = np.asarray(data["triple"])
    out["head_keys"] = np.array(list(data["head"].keys()))
    out["head_flat"] = np.concatenate([np.asarray(v) for v in data["head"].values()])
    out["tail_flat"] = np.concatenate([np.asarray(v) for v in data["tail"].values()])
    out["head_r"] = np.asarray(data["head_r"])
    out["tail_r"] = np.asarray(data["tail_r"])
    for k in ("adj", "adj1", "adj2"):
        out["sep_%s_idx" % k] = sep[k]._indices().numpy()
        out["sep_%s_val" % k] = sep[k]._values().numpy()
    out["sep_train"], out["sep_test"] = sep["train"], sep["test"]
    out["sep_e"] = np.array([sep["e1"], sep["e2"]])
    out["sep_index1"] = np.array([sep["index1"][i] for i in range(sep["e1"])])
    out["sep_index2"] = np.array([sep["index2"][i] for i in range(sep["e2"])])
    return out
