"""The Linear layer's act fused into the GEMM (layers/layers.py:111-122, the MLPDecoder's relu
layers at models/decoders.py:57-63): gnnea_gemm_x3_act_f32 / gnnea_gemm_bf16_act (relu in the
weight-resident kernels' epilogue, other acts in place after the product) and
gnnea_act_bwd_colsum_* (the act's backward and the bias gradient in one pass).

Checks:
  * the fused forward equals the unfused one (the same GEMM, then F.relu) bit for bit, and the
    fused backward's input / weight gradients equal the unfused ones bit for bit (the act's
    derivative is 0 / 1, so G is exact either way);
  * against an fp64 restatement (fp32 tolerance 1e-5 norm-relative for the x3 GEMM; the relu
    branch of the backward taken from the tested output, whose elements inside the rounding band
    of 0 are ~1e-7 of the norm);
  * the one-pass act backward + column sums vs fp64 on row-major, strided (column block of a
    wider buffer), unvectorised (D % 4 != 0), > 1024-wide and empty inputs.
"""
import pytest
import torch
import torch.nn.functional as F

from conftest import rel_err

pytestmark = pytest.mark.gpu
TOL32 = 1e-5


def _inputs(device, M, K, N, dtype=torch.float32, seed=0):
    g = torch.Generator(device=device).manual_seed(seed)
    x = torch.randn(M, K, device=device, generator=g).to(dtype)
    W = (torch.randn(N, K, device=device, generator=g) / K ** 0.5).to(dtype)
    b = (0.1 * torch.randn(N, device=device, generator=g)).to(dtype)
    R = torch.randn(M, N, device=device, generator=g)
    return x, W, b, R


def _run(fn, x, W, b, R):
    x = x.clone().requires_grad_(True)
    W = W.clone().requires_grad_(True)
    b = b.clone().requires_grad_(True)
    y = fn(x, W, b)
    (y.float() * R).sum().backward()
    return y.detach(), x.grad, W.grad, b.grad


@pytest.mark.parametrize("M,K,N", [(70000, 300, 300),   # weight-resident ring: relu epilogue
                                   (70000, 600, 300),   # k_gemm_x3p, act in place after
                                   (1000, 300, 300)])   # small: exact-f32 GEMM + act pass
def test_linear_relu_fused_vs_unfused_and_fp64(device, M, K, N):
    from gnnea import _lib, ops
    x, W, b, R = _inputs(device, M, K, N)
    relu = _lib.GNNEA_ACT_RELU
    yf, dxf, dWf, dbf = _run(lambda x, W, b: ops.linear(x, W, b, act=relu), x, W, b, R)
    yu, dxu, dWu, dbu = _run(lambda x, W, b: F.relu(ops.linear(x, W, b)), x, W, b, R)
    assert torch.equal(yf, yu)
    assert torch.equal(dxf, dxu) and torch.equal(dWf, dWu)
    assert rel_err(dbf.cpu(), dbu.cpu()) < 1e-6
    x64, W64, b64, R64 = x.double(), W.double(), b.double(), R.double()
    y64 = torch.relu(x64 @ W64.t() + b64)
    assert rel_err(yf.cpu(), y64.cpu()) < TOL32
    G = R64 * (yf > 0).double()  # the branch of the tested output
    assert rel_err(dxf.cpu(), (G @ W64).cpu()) < TOL32
    assert rel_err(dWf.cpu(), (G.t() @ x64).cpu()) < TOL32
    assert rel_err(dbf.cpu(), G.sum(0).cpu()) < TOL32


@pytest.mark.parametrize("act", ["elu", "tanh", "sigmoid", "leaky_relu"])
def test_linear_other_acts_vs_fp64(device, act):
    from gnnea import ops
    fn = {"elu": F.elu, "tanh": torch.tanh, "sigmoid": torch.sigmoid,
          "leaky_relu": F.leaky_relu}[act]
    code = ops.act_code(fn)
    x, W, b, R = _inputs(device, 70000, 300, 300, seed=3)
    yf, dxf, dWf, dbf = _run(lambda x, W, b: ops.linear(x, W, b, act=code), x, W, b, R)
    x64, W64, b64, R64 = (t.double() for t in (x, W, b, R))
    h64 = x64 @ W64.t() + b64
    y64 = fn(h64)
    assert rel_err(yf.cpu(), y64.cpu()) < TOL32
    if act == "leaky_relu":  # a jump in the derivative at 0: the branch of the tested output
        G = R64 * torch.where(yf > 0, 1.0, 0.01).double()
    else:
        h64.requires_grad_(True)
        (fn(h64) * R64).sum().backward()
        G = h64.grad
    assert rel_err(dxf.cpu(), (G @ W64).cpu()) < 3 * TOL32
    assert rel_err(dWf.cpu(), (G.t() @ x64).cpu()) < 3 * TOL32
    assert rel_err(dbf.cpu(), G.sum(0).cpu()) < 3 * TOL32


def test_linear_relu_bf16_fused_vs_unfused(device):
    """cfg-5 storage: bf16 x / W, the weight-resident bf16 kernel's relu epilogue."""
    from gnnea import _lib, ops
    x, W, b, R = _inputs(device, 70000, 300, 300, dtype=torch.bfloat16, seed=5)
    relu = _lib.GNNEA_ACT_RELU
    yf, dxf, dWf, dbf = _run(lambda x, W, b: ops.linear(x, W, b, act=relu), x, W, b, R)
    yu, dxu, dWu, dbu = _run(lambda x, W, b: F.relu(ops.linear(x, W, b)), x, W, b, R)
    assert yf.dtype == torch.bfloat16 and dxf.dtype == torch.bfloat16
    assert torch.equal(yf, yu)  # relu commutes with the one bf16 rounding
    assert torch.equal(dxf, dxu) and torch.equal(dWf, dWu)
    G = (R.bfloat16().double() * (yf > 0).double())
    assert rel_err(dbf.float().cpu(), G.sum(0).cpu()) < 1e-2  # the bf16 bias gradient's rounding


@pytest.mark.parametrize("n,D,ld,dtype", [(50000, 300, 300, torch.float32),
                                          (50000, 300, 600, torch.float32),   # column block
                                          (3001, 30, 30, torch.float32),      # D % 4 != 0
                                          (2000, 1100, 1100, torch.float32),  # > 1024 wide
                                          (50000, 300, 300, torch.bfloat16),
                                          (777, 302, 302, torch.bfloat16),
                                          (0, 300, 300, torch.float32)])
def test_act_bwd_colsum_vs_fp64(device, n, D, ld, dtype):
    from gnnea import _lib, ops
    g = torch.Generator(device=device).manual_seed(n + D)
    buf_y = torch.randn(n, ld, device=device, generator=g).to(dtype)
    buf_d = torch.randn(n, ld, device=device, generator=g).to(dtype)
    y, dy = buf_y[:, :D], buf_d[:, :D]
    for act in (_lib.GNNEA_ACT_RELU, _lib.GNNEA_ACT_TANH):
        G, db = ops.act_bwd_colsum(dy, y, act)
        y64, dy64 = y.double(), dy.double()
        d = (y64 > 0).double() if act == _lib.GNNEA_ACT_RELU else 1 - y64 * y64
        G64 = dy64 * d
        tol = 1e-2 if dtype == torch.bfloat16 else 1e-6
        assert G.shape == (n, D) and db.shape == (D,) and db.dtype == torch.float32
        if n == 0:
            assert torch.all(db == 0)
            continue
        assert rel_err(G.double().cpu(), G64.cpu()) < tol
        # the column sums are of the stored G (exactly what the bias gradient sums)
        assert rel_err(db.cpu(), G.double().sum(0).cpu()) < 1e-6
        G2, db2 = ops.act_bwd_colsum(dy, y, act)
        assert torch.equal(G, G2) and torch.equal(db, db2)  # deterministic


@pytest.mark.parametrize("dtype,M", [(torch.bfloat16, 70000),   # masked backward products
                                     (torch.bfloat16, 1000),    # small: the two-step fallback
                                     (torch.float32, 70000),    # fp32: the ring's sign bits
                                     (torch.float32, 1000)])    # fp32 small: two steps
def test_mlp_chain_vs_per_layer(device, dtype, M):
    """MLPDecoder's three Linear layers (relu, relu, identity; models/decoders.py) as one
    MLPChainFn against the per-layer LinearActFn / LinearFn path: output, dx and every dW bit
    for bit (gemm_dmask's masked product = the product then act_bwd's G), db to 1e-6 (the same
    values summed in another order; bf16 biases round each sum) -- and the fused path is the one
    that ran (tall)."""
    import torch.nn as nn
    from gnnea import ops
    from layers.layers import Linear
    from models.decoders import _identity
    torch.manual_seed(5)
    layers = nn.Sequential(Linear(300, 300, 0.0, F.relu, True), Linear(300, 300, 0.0, F.relu, True),
                           Linear(300, 300, 0.0, _identity, True)).to(device).to(dtype)
    g = torch.Generator(device=device).manual_seed(6)
    x0 = torch.randn(M, 300, device=device, generator=g).to(dtype)
    R = torch.randn(M, 300, device=device, generator=g).to(dtype)
    calls = []
    orig = ops.gemm_dmask

    def spy(*a):
        out = orig(*a)
        calls.append(out is not None and a[3] is not None)  # (from the forward's sign bits)
        return out

    def run(fused):
        layers.zero_grad()
        x = x0.clone().requires_grad_(True)
        y = ops.mlp_chain(x, layers) if fused else layers(x)
        assert y is not None
        (y.float() * R.float()).sum().backward()
        return [y.detach(), x.grad] + [p.grad.clone() for p in layers.parameters()]
    import pytest as _pt
    mp = _pt.MonkeyPatch()
    mp.setattr(ops, "gemm_dmask", spy)
    try:
        got = run(True)
    finally:
        mp.undo()
    ref = run(False)
    assert calls == [M >= 65536] * 2
    names = ["y", "dx", "dW0", "db0", "dW1", "db1", "dW2", "db2"]
    for nm, a, b in zip(names, got, ref):
        if nm.startswith("db"):  # (bf16 biases: each sum rounded to bf16, a 2^-8 step apart)
            tol = 1e-6 if dtype == torch.float32 else 8e-3
            assert rel_err(a.float().cpu(), b.float().cpu()) < tol, nm
        else:
            assert torch.equal(a, b), nm


def test_relu_mask_bits_and_dmask_forms(device):
    """gemm_relu_mask: y bit-identical to the relu GEMM, the sign bits = (y > 0) in the documented
    layout (byte 20 t + 4 u + g of a row: columns 160 t + 32 u + 8 g + 0..7); gemm_dmask from the
    bits = from y = the product then act_bwd, bit for bit (ragged rows, N = 300 in two tiles)."""
    from gnnea import _lib, ops
    g0 = torch.Generator(device=device).manual_seed(9)
    M = 70001
    x = torch.randn(M, 300, device=device, generator=g0).bfloat16()
    W = (torch.randn(300, 300, device=device, generator=g0) / 17).bfloat16()
    b = (0.1 * torch.randn(300, device=device, generator=g0)).bfloat16()
    y, mask = ops.gemm_relu_mask(x, W, b)
    assert torch.equal(y, ops.gemm(x, W, trans_b=True, bias=b, act=_lib.GNNEA_ACT_RELU))
    cols = torch.arange(300, device=device)
    byte = 20 * (cols // 160) + (cols % 160) // 8
    bits = (mask[:, byte] >> (cols % 8).to(torch.uint8)) & 1
    assert torch.equal(bits.bool(), y > 0)
    dy = torch.randn(M, 300, device=device, generator=g0).bfloat16()
    W2 = (torch.randn(300, 300, device=device, generator=g0) / 17).bfloat16()
    ref = ops.act_bwd(ops.gemm(dy, W2), y, _lib.GNNEA_ACT_RELU)
    assert torch.equal(ops.gemm_dmask(dy, W2, y), ref)
    assert torch.equal(ops.gemm_dmask(dy, W2, y, mask), ref)


def test_relu_mask_bits_f32(device):
    """The fp32 forms (the f16x2 ring's epilogue): y bit-identical to the relu GEMM, the bits =
    (y > 0) in the documented layout (byte 16 t + 2 j + h: columns 112 t + 16 j + 8 h + 0..7),
    gemm_dmask from them = the product then act_bwd, bit for bit (ragged rows, three tiles)."""
    from gnnea import _lib, ops
    g0 = torch.Generator(device=device).manual_seed(10)
    M = 70001
    x = torch.randn(M, 300, device=device, generator=g0)
    W = torch.randn(300, 300, device=device, generator=g0) / 17
    b = 0.1 * torch.randn(300, device=device, generator=g0)
    y, mask = ops.gemm_relu_mask(x, W, b)
    assert torch.equal(y, ops.gemm(x, W, trans_b=True, bias=b, act=_lib.GNNEA_ACT_RELU))
    cols = torch.arange(300, device=device)
    byte = 16 * (cols // 112) + (cols % 112) // 8
    bits = (mask[:, byte] >> (cols % 8).to(torch.uint8)) & 1
    assert torch.equal(bits.bool(), y > 0)
    dy = torch.randn(M, 300, device=device, generator=g0)
    W2 = torch.randn(300, 300, device=device, generator=g0) / 17
    ref = ops.act_bwd(ops.gemm(dy, W2), y, _lib.GNNEA_ACT_RELU)
    assert ops.gemm_dmask(dy, W2, y) is None  # (fp32: from the bits only)
    assert torch.equal(ops.gemm_dmask(dy, W2, y, mask), ref)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("K,M,N,block", [(200003, 300, 300, False),   # K tail, 2 column tiles
                                         (70000, 300, 300, True),     # dh a column block (ld 2M)
                                         (70000, 128, 100, False),    # one tile, M < 160
                                         (70000, 300, 296, False),    # N % 8 == 0 (bf16 chunk)
                                         (70000, 300, 320, False)])   # no padding column: None
def test_gemm_ta_db_vs_separate(device, K, M, N, block, dtype):
    """gemm_ta_db: a layer's dW = dhᵀ·x bit-identical to gemm(dh, x, trans_a=True) (the same
    kernel; bf16: bf16 out as the Linear's bf16 weight) and db = column sums of dh from the
    kernel's ones column, against fp64 of the same (stored) values (fp32 sums of K = 2e5 terms:
    1e-6 norm-relative) and against colsum."""
    from gnnea import ops
    g0 = torch.Generator(device=device).manual_seed(11)
    big = torch.randn(K, 2 * M if block else M, device=device, generator=g0).to(dtype)
    dh = big[:, :M]
    x = torch.randn(K, N, device=device, generator=g0).to(dtype)
    od = torch.bfloat16 if dtype == torch.bfloat16 else None
    r = ops.gemm_ta_db(dh, x, od)
    if N % 160 == 0:
        assert r is None
        return
    dw, db = r
    assert torch.equal(dw, ops.gemm(dh, x, trans_a=True, out_dtype=od))
    ref = dh.double().sum(0)
    assert rel_err(db.cpu(), ref.cpu()) < 1e-6
    assert rel_err(db.cpu(), ops.colsum(dh, torch.float32).cpu()) < 1e-6
