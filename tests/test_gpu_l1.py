"""§8f #1 parity: device L1 searches (gnnea_l1_*, gnnea_topk_rows_f32) vs the reference's
scipy-based get_neg / get_hits / eval_at_1 / generate_pairs (golden fixtures) and vs the oracle.

Distances are compared bit-exactly (fp64 sums of exact terms); index outputs bit-exactly.
"""
import types

import numpy as np
import pytest
import torch

from oracle import l1 as ol1

pytestmark = pytest.mark.gpu


def _fixture(golden, device):
    f = golden("l1_search")
    return f, torch.from_numpy(f["vec"]).to(device)


def test_get_neg_vs_reference(golden, device):
    from models.models_ea import BaseModel
    f, vec = _fixture(golden, device)
    tr = f["train"]
    assert (BaseModel.get_neg(None, tr[:, 0], vec, 25) == f["neg_right"]).all()
    assert (BaseModel.get_neg(None, tr[:, 1], vec, 25) == f["neg2_left"]).all()
    # the reference passes host tensors: same result after the upload
    assert (BaseModel.get_neg(None, tr[:, 0], vec.cpu(), 25) == f["neg_right"]).all()


def test_get_hits_vs_reference(golden, device):
    from utils.eval_utils import eval_at_1, get_hits
    f, vec = _fixture(golden, device)
    for split in ("train", "test"):
        m = get_hits(vec, f[split])
        assert list(m) == list(f["hits_%s_keys" % split])
        assert list(m.values()) == list(f["hits_%s_vals" % split])
    m = get_hits(vec.cpu(), f["test"], top_k=[1])
    assert m == {"Hits@1_l": f["hits_test_vals"][0], "Hits@1_r": f["hits_test_vals"][4]}
    assert abs(float(eval_at_1(vec, {"test": f["test"]})) - float(f["eval_at_1"])) < 1e-4


def test_generate_pairs_vs_reference(golden, device):
    from models.models_ea import UEAModel
    f, vec = _fixture(golden, device)
    e1 = len(f["gp_index1"])
    data = {"e1": e1, "e2": e1, "index1": dict(enumerate(f["gp_index1"].tolist())),
            "index2": dict(enumerate(f["gp_index2"].tolist()))}
    for key, bsz in (("gp_ILL", 200), ("gp_ILL30", 30)):
        holder = types.SimpleNamespace(ILL=None)
        UEAModel.generate_pairs(holder, vec, data, bsz)
        assert (holder.ILL == f[key]).all()


def test_distances_bit_exact(device):
    from gnnea import l1
    rng = np.random.default_rng(3)
    for nq, nx, D in ((1, 1, 1), (5, 70, 3), (130, 257, 300), (64, 64, 33), (77, 1000, 100)):
        A = rng.standard_normal((nq, D)).astype(np.float32) * rng.uniform(0.01, 3)
        B = rng.standard_normal((nx, D)).astype(np.float32)
        ref = ol1.cityblock(A, B)
        k = l1.keys(torch.from_numpy(A).to(device), torch.from_numpy(B).to(device)).cpu().numpy()
        assert (k == ref.astype(np.float32)).all()
        n = min(nq, nx)
        d = l1.pairs(torch.from_numpy(A[:n]).to(device), torch.from_numpy(B[:n]).to(device))
        assert (d.cpu().numpy() == np.diag(ref[:n, :n])).all()


@pytest.mark.parametrize("nq,nx,D,K,skip", [(40, 3000, 300, 26, 1), (7, 513, 64, 1, 0),
                                            (300, 2000, 100, 512, 0), (3, 600, 5, 600 // 2, 2)])
def test_topk_vs_oracle(device, nq, nx, D, K, skip):
    from gnnea import l1
    rng = np.random.default_rng(nq + nx)
    X = (0.1 * rng.standard_normal((nx, D))).astype(np.float32)
    Q = X[rng.integers(0, nx, nq)] + (0.05 * rng.standard_normal((nq, D))).astype(np.float32)
    S = ol1.cityblock(Q, X)
    order = np.argsort(S, axis=1, kind="stable")[:, skip:K]
    idx, dist = l1.topk(torch.from_numpy(Q).to(device), torch.from_numpy(X).to(device), K,
                        skip, want_dist=True)
    assert (idx.cpu().numpy() == order).all()
    assert (dist.cpu().numpy() == np.take_along_axis(S, order, 1)).all()
    assert int(l1.topk.last_overflow.item()) == 0


def test_topk_ties_and_duplicates(device):
    """Exact duplicate rows and an all-equal (collapsed) embedding: lowest indices first."""
    from gnnea import l1
    rng = np.random.default_rng(9)
    X = (0.1 * rng.standard_normal((500, 16))).astype(np.float32)
    X[100:140] = X[7]  # 41 copies of row 7
    Q = X[[7, 100, 3]]
    S = ol1.cityblock(Q, X)
    order = np.argsort(S, axis=1, kind="stable")[:, :60]
    idx = l1.topk(torch.from_numpy(Q).to(device), torch.from_numpy(X).to(device), 60)
    assert (idx.cpu().numpy() == order).all()
    Z = np.zeros((3000, 8), np.float32)  # every distance 0: ties beyond the candidate cap
    idx = l1.topk(torch.from_numpy(Z[:4]).to(device), torch.from_numpy(Z).to(device), 11, 1)
    assert (idx.cpu().numpy() == np.arange(1, 11)[None, :]).all()
    assert int(l1.topk.last_overflow.item()) == 4


def test_hits_ranks_with_ties(device):
    from gnnea import l1
    rng = np.random.default_rng(4)
    L = np.round(rng.standard_normal((300, 4)), 1).astype(np.float32)  # many equal distances
    R = np.round(L + 0.3 * rng.standard_normal((300, 4)), 1).astype(np.float32)
    vec = np.concatenate([L, R])
    pairs = np.stack([np.arange(300), np.arange(300) + 300], 1)
    lr_ref, rl_ref = ol1.hit_ranks(vec, pairs)
    lr, rl = l1.hits_ranks(torch.from_numpy(L).to(device), torch.from_numpy(R).to(device))
    assert (lr.cpu().numpy() == lr_ref).all() and (rl.cpu().numpy() == rl_ref).all()


def test_l1_rejects_bad_shapes(device):
    from gnnea import _lib, l1
    X = torch.zeros(10, 4, device=device)
    with pytest.raises(ValueError):
        l1.topk(X, X, 11)
    with pytest.raises(_lib.GnneaError):
        l1.topk(torch.zeros(2, 4, device=device), torch.zeros(2000, 4, device=device), 600)


# ---------------- §8f #2 margin loss ----------------
def test_margin_loss_vs_reference(golden, device):
    """EAModel.get_loss through the fused kernels vs the reference (fp32; tolerance 1e-5
    norm-relative: the reference's fp32 sums are reduced in another order)."""
    from conftest import rel_err
    from models.models_ea import EAModel
    f, vec = _fixture(golden, device)
    tr, k = f["train"], 25
    holder = types.SimpleNamespace(neg_num=k, neg_right=f["neg_right"], neg2_left=f["neg2_left"])
    holder.neg_left = (np.ones((len(tr), k)) * tr[:, 0:1]).reshape(-1)
    holder.neg2_right = (np.ones((len(tr), k)) * tr[:, 1:2]).reshape(-1)
    x = vec.clone().requires_grad_(True)
    loss = EAModel.get_loss(holder, x, {"train": tr}, "train")
    loss.backward()
    assert abs(float(loss.detach()) - float(f["margin_loss"])) <= 1e-5 * float(f["margin_loss"])
    assert rel_err(x.grad.cpu().numpy(), f["margin_grad"]) < 1e-5


@pytest.mark.parametrize("N,D,t,k,anchored", [(500, 300, 60, 7, True), (300, 37, 40, 5, False),
                                              (2000, 1024, 16, 33, True), (50, 8, 30, 9, False),
                                              (40, 64, 300, 30, False)])  # hub rows: chunks
def test_margin_vs_oracle(device, N, D, t, k, anchored):
    """Active and inactive hinge terms, repeated rows, non-anchored negatives, scalar and float4
    paths; fp32 kernel vs fp64 oracle."""
    from conftest import rel_err
    from gnnea.margin import margin_loss
    from oracle import margin as om
    rng = np.random.default_rng(D + k)
    vec = (rng.standard_normal((N, D)) / np.sqrt(D)).astype(np.float32)
    left = rng.integers(0, N, t)
    right = rng.integers(0, N, t)
    vec[right[: t // 2]] = vec[left[: t // 2]] + 0.01 * rng.standard_normal((t // 2, D))
    if anchored:
        nl1, nr2 = np.repeat(left, k), np.repeat(right, k)
    else:
        nl1, nr2 = rng.integers(0, N, t * k), rng.integers(0, N, t * k)
    nr1, nl2 = rng.integers(0, N, t * k), rng.integers(0, N, t * k)
    x = torch.from_numpy(vec).to(device).requires_grad_(True)
    loss = margin_loss(x, left, right, nl1, nr1, nl2, nr2, t, k)
    loss.backward()
    ref_loss, ref_grad = om.margin_loss_and_grad(vec, left, right, nl1, nr1, nl2, nr2, t, k)
    assert 0 < ref_loss
    assert abs(float(loss) - ref_loss) <= 1e-5 * ref_loss
    assert rel_err(x.grad.cpu().numpy(), ref_grad) < 1e-5


def test_margin_rejects_bad_indices(device):
    from gnnea.margin import margin_loss
    x = torch.zeros(10, 4, device=device)
    with pytest.raises(IndexError):
        margin_loss(x, [0], [10], [0], [1], [2], [3], 1, 1)
    with pytest.raises(ValueError):
        margin_loss(x, [0], [1], [0], None, [2], [3], 1, 1)


def test_margin_backward_deterministic(device):
    """The incidence-gather backward has no atomics: gradients are bit-identical run to run."""
    from gnnea.margin import margin_loss
    rng = np.random.default_rng(1)
    N, D, t, k = 3000, 300, 200, 40
    vec = torch.from_numpy((0.05 * rng.standard_normal((N, D))).astype(np.float32)).to(device)
    idx = [rng.integers(0, 50, t), rng.integers(0, N, t)] + \
        [rng.integers(0, 50 if i % 2 == 0 else N, t * k) for i in range(4)]  # hub rows
    grads = []
    for _ in range(3):
        x = vec.clone().requires_grad_(True)
        margin_loss(x, *idx, t, k).backward()
        grads.append(x.grad.cpu().numpy())
    assert (grads[0] == grads[1]).all() and (grads[0] == grads[2]).all()


@pytest.mark.parametrize("N,D,t,k", [(3000, 300, 200, 40), (500, 1024, 30, 9), (60, 8, 50, 6),
                                     (40, 64, 300, 30), (80, 300, 4, 300)])  # k > 255: int32 path
def test_margin_sign_codes_match_row_gather(device, N, D, t, k):
    """The sign-code backward (the forward stores 2 bits per column, the backward reads them)
    gives the row-gather backward's gradient bit for bit: hub rows (chunked items), tied columns
    (duplicate rows: code 00) and every float4 width."""
    from gnnea import margin
    rng = np.random.default_rng(D * 7 + k)
    vec = (0.05 * rng.standard_normal((N, D))).astype(np.float32)
    vec[: N // 4, : D // 2] = vec[N // 4: 2 * (N // 4), : D // 2]  # exact ties in half the columns
    x0 = torch.from_numpy(vec).to(device)
    idx = [rng.integers(0, N // 2, t), rng.integers(0, N, t)] + \
        [rng.integers(0, 40 if i % 2 == 0 else N // 2, t * k) for i in range(4)]
    out = []
    try:
        for codes in (True, False):
            margin.CODES = codes
            x = x0.clone().requires_grad_(True)
            loss = margin.margin_loss(x, *idx, t, k)
            loss.backward()
            out.append((float(loss), x.grad.cpu().numpy()))
    finally:
        margin.CODES = True
    assert out[0][0] == out[1][0]
    assert (out[0][1] == out[1][1]).all()
    assert np.abs(out[0][1]).sum() > 0


@pytest.mark.parametrize("N,D,t,k", [(3000, 300, 200, 40), (500, 1024, 30, 9), (60, 8, 50, 6),
                                     (40, 64, 300, 30), (80, 300, 4, 300), (300, 37, 40, 5)])
def test_margin_bf16_rows_match_fp32_copy(device, N, D, t, k):
    """bf16 embeddings (cfg-5 storage): the sign-code kernels read the bf16 rows and write a bf16
    gradient.  Loss and gradient are bit-identical to the fp32 kernels on out.float() with the
    gradient cast back (the path without the bf16 kernels): hub rows (chunked items, k > 255 on
    the int32 path), tied columns; D = 37 takes the fp32-copy fallback."""
    from gnnea.margin import margin_loss
    rng = np.random.default_rng(N + D + k)
    vec = torch.from_numpy((0.05 * rng.standard_normal((N, D))).astype(np.float32))
    vec[1] = vec[0]  # a tied pair: code 00 in every column
    xb = vec.to(device).bfloat16()
    idx = [rng.integers(0, N, t), rng.integers(0, N, t)] + \
        [rng.integers(0, 20 if i % 2 == 0 else N, t * k) for i in range(4)]  # hub rows
    idx[0][0], idx[1][0] = 0, 1
    x1 = xb.clone().requires_grad_(True)
    l1 = margin_loss(x1, *idx, t, k)
    l1.backward()
    x2 = xb.clone().requires_grad_(True)
    l2 = margin_loss(x2.float(), *idx, t, k)
    l2.backward()
    assert x1.grad.dtype == torch.bfloat16
    assert float(l1) == float(l2)
    assert torch.equal(x1.grad, x2.grad)


def test_l1_ties_vs_reference(golden, device):
    """The drop-in get_neg / get_hits on the tie-heavy fixture the reference produced: equal to
    the reference up to the order among exactly equal distances (tests/tie_rules.py), and index
    for index equal to the stable-order oracle (ties by index, the documented rule)."""
    import tie_rules
    from models.models_ea import BaseModel
    from oracle import l1 as l1o
    from utils.eval_utils import get_hits
    f = golden("l1_ties")
    vec, train, test = f["vec"], f["train"], f["test"]
    out = torch.from_numpy(vec).to(device)
    for col, key in ((0, "neg_right"), (1, "neg2_left")):
        got = BaseModel.get_neg(None, train[:, col], out, 25)
        tie_rules.check_neg(vec, train[:, col], got, f[key], 25)
        assert np.array_equal(got, l1o.get_neg(train[:, col], vec, 25))
    for split, pairs in (("train", train), ("test", test)):
        got = get_hits(out, pairs)
        tie_rules.check_hits(vec, pairs, got, f["hits_%s_keys" % split],
                             f["hits_%s_vals" % split])
        assert got == l1o.get_hits(vec, pairs)
