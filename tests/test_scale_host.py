"""Host-side checks of the BASELINE-size test infrastructure (CPU only).

  * the vectorised adjacency builder reproduces the reference's COO at DBP15K scale (order and
    values, by the digest the reference run stored in tests/golden/dbp15k.npz);
  * the neighbourhood oracle (oracle/local.py) equals the whole-graph oracle (oracle/gnn.py) on
    the rows it samples, outputs and input gradients, for the three layer kinds;
  * the seeded inputs are reproducible.
"""
import hashlib

import numpy as np
import pytest
import torch

import scale_inputs as si


def test_dbp15k_adjacency_matches_reference(golden):
    f = golden("dbp15k")
    tr, N, r, c, v = si.dbp15k_graph()
    assert r.size == int(f["nnz"]) == 229940
    idx = np.stack([r, c]).astype(np.int64)
    assert hashlib.sha256(idx.tobytes() + v.tobytes()).hexdigest() == str(f["adj_sha256"])


def _small_graph(n=300, t=1200, seed=3):
    from gnnea import synth
    tr = synth.kg_pair_triples(n, t, 20, seed=seed)
    r, c, v = synth.adjacency_coo(tr, 2 * n, reference_order=True)
    return 2 * n, r, c, v


@pytest.mark.parametrize("kind", ["gcn", "highway", "gat"])
def test_local_oracle_equals_whole_graph(kind):
    from oracle import gnn
    from oracle.local import LocalGraph, sampled_input_grads, sampled_outputs
    N, r, c, v = _small_graph()
    rng = np.random.default_rng(1)
    x = rng.standard_normal((N, 32)) * 0.3
    R = rng.standard_normal((N, 32))
    if kind == "gcn":
        params = [torch.randn(32, 32, dtype=torch.float64) * 0.2, torch.randn(32).double() * 0.1]
        fn = lambda xx, W, b: gnn.gcn_layer(xx, W, b, r, c, v)  # noqa: E731
        full_params = params
    elif kind == "highway":
        W, b, Kg = (torch.randn(32, 32).double() * 0.2, torch.randn(32).double() * 0.1,
                    torch.randn(32, 32).double() * 0.2)
        params = [W, b, Kg, None]
        fn = lambda xx, W_, b_: gnn.highway_layer(xx, W_, b_, Kg, r, c, v)  # noqa: E731
        full_params = [W, b]
    else:
        Ws = torch.randn(2, 32, 16).double() * 0.3
        As = torch.randn(2, 1, 32).double() * 0.3
        params = [Ws, As]
        fn = lambda xx, Ws_, As_: gnn.gat_layer(xx, Ws_, As_, r, c)  # noqa: E731
        full_params = params
    out, dx, _ = gnn.layer_with_grads(fn, x, full_params, R)
    g = LocalGraph(r, c, v, N)
    rows = np.array([0, 5, 17, 299, 300, 301, 598, 599])
    S, o = sampled_outputs(kind, g, x, rows, params)
    assert np.array_equal(S, rows)
    np.testing.assert_allclose(o.numpy(), out[rows].numpy(), rtol=1e-12, atol=1e-13)
    T, d = sampled_input_grads(kind, g, x, R, rows, params)
    np.testing.assert_allclose(d.numpy(), dx[rows].numpy(), rtol=1e-11, atol=1e-12)


def test_relu_branch_band_follows_tested_output():
    from oracle.local import _relu_hybrid
    pre = torch.tensor([[1.0, -1.0, 1e-9, -1e-9]], dtype=torch.float64)
    tested = np.array([[1.0, 0.0, 0.0, 2e-9]])  # the tested path took the other side twice
    y = _relu_hybrid(pre, tested)
    assert y.tolist() == [[1.0, -0.0, 0.0, -1e-9]]


def test_seeded_inputs_reproducible():
    a = si.sinkhorn_cost(300)
    b = si.sinkhorn_cost(300)
    assert a.dtype == torch.float32 and torch.equal(a, b) and float(a.max()) == 1.0
    assert np.array_equal(si.negatives(100, 5, 3, 1), si.negatives(100, 5, 3, 1))
    p = si.ea_pairs(1000, 50)
    assert p.shape == (50, 2) and np.all(p[:, 1] == p[:, 0] + 1000)


def test_fp64_device_reference_equals_oracle():
    """tests/fp64_ref.py (the whole-graph fp64 restatement the BASELINE-size GPU tests run on
    the device) equals the CPU oracle's autograd gradients; run here on host tensors."""
    import fp64_ref
    from oracle import gnn
    N, r, c, v = _small_graph()
    rng = np.random.default_rng(2)
    x = torch.from_numpy(rng.standard_normal((N, 32)) * 0.3)
    R = torch.from_numpy(rng.standard_normal((N, 32)))
    W, b, Kg = (torch.randn(32, 32).double() * 0.2, torch.randn(32).double() * 0.1,
                torch.randn(32, 32).double() * 0.2)
    rt, ct, vt = torch.from_numpy(r), torch.from_numpy(c), torch.from_numpy(v).double()
    _, _, (dW, db) = gnn.layer_with_grads(lambda xx, W_, b_: gnn.gcn_layer(xx, W_, b_, r, c, v),
                                          x, [W, b], R)
    gW, gb = fp64_ref.gcn_grads(rt, ct, vt, x, W, b, R, None)
    np.testing.assert_allclose(gW.numpy(), dW.numpy(), rtol=1e-11, atol=1e-12)
    np.testing.assert_allclose(gb.numpy(), db.numpy(), rtol=1e-11, atol=1e-12)
    _, _, (dW, db) = gnn.layer_with_grads(
        lambda xx, W_, b_: gnn.highway_layer(xx, W_, b_, Kg, r, c, v), x, [W, b], R)
    gW, gb = fp64_ref.highway_grads(rt, ct, vt, x, W, b, Kg, R, None)
    np.testing.assert_allclose(gW.numpy(), dW.numpy(), rtol=1e-11, atol=1e-12)
    np.testing.assert_allclose(gb.numpy(), db.numpy(), rtol=1e-11, atol=1e-12)
    # the differentiable layer (EA-step reference) against the oracle's forward
    xx = x.clone().requires_grad_(True)
    y = fp64_ref.highway_layer(xx, W, b, Kg, rt, ct, vt, relu=True)
    np.testing.assert_allclose(y.detach().numpy(),
                               gnn.highway_layer(x, W, b, Kg, r, c, v).numpy(), rtol=1e-12,
                               atol=1e-13)
