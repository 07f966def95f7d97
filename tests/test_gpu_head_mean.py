"""The non-concatenated GAT layer's head mean (layers/att_layers.py:89-91,
torch.mean(torch.stack(heads), dim=2)) on gnnea_head_mean_*: forward and backward against torch's
mean of the same tensor, fp32 (1e-6) and bf16 (one bf16 rounding: at most one ulp apart), on
row-major and column-block inputs, heads 1 / 3 / 4, d_head 75 (cfg-5) and 8."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,heads,dh,ld", [(200000, 4, 75, 300), (1001, 3, 8, 24),
                                           (5000, 4, 75, 320), (777, 1, 16, 16)])
def test_head_mean_vs_torch(device, dtype, n, heads, dh, ld):
    from gnnea import ops
    g = torch.Generator(device=device).manual_seed(n + heads)
    buf = torch.randn(n, ld, device=device, generator=g).to(dtype)
    x = buf[:, :heads * dh]
    xr = x.detach().clone().requires_grad_(True)
    xg = x.detach().clone().requires_grad_(True)
    R = torch.randn(n, dh, device=device, generator=g).to(dtype)
    y_ref = xr.view(-1, heads, dh).mean(dim=1) if ld == heads * dh else \
        xr.contiguous().view(-1, heads, dh).mean(dim=1)
    (y_ref.float() * R.float()).sum().backward()
    y = ops.head_mean(xg, heads, dh)
    (y.float() * R.float()).sum().backward()
    assert y.shape == (n, dh) and y.dtype == dtype
    if dtype == torch.float32:
        assert torch.allclose(y, y_ref, rtol=1e-6, atol=1e-6)
        assert torch.allclose(xg.grad, xr.grad, rtol=1e-6, atol=1e-6)
    else:
        ulp = (y_ref.float().abs() * 2.0 ** -7).clamp(min=1e-30)
        assert torch.all((y.float() - y_ref.float()).abs() <= ulp + 1e-30)
        assert torch.equal(xg.grad, xr.grad) or \
            torch.allclose(xg.grad.float(), xr.grad.float(), rtol=2 ** -7, atol=0)
