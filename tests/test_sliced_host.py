"""Host-side logic of the slice-major tables (no GPU): when the sliced path applies, the table
shapes, and the element map (c // W)·sstride + r·W + c % W restated on the CPU."""
import torch

from gnnea import ops


def _slice_cpu(x, W):
    """CPU restatement of gnnea_slice_pack_*: [n, D] -> [ceil(D/W), n, W] (zero padded)."""
    n, D = x.shape
    S = (D + W - 1) // W
    out = torch.zeros(S, n, W, dtype=x.dtype)
    for s in range(S):
        w = min(W, D - s * W)
        out[s, :, :w] = x[:, s * W:s * W + w]
    return out


def test_slice_widths():
    assert ops.slice_w(torch.float32) == 64
    assert ops.slice_w(torch.bfloat16) == 128


def test_use_sliced_thresholds(monkeypatch):
    # cfg-4: one KG of 1M rows x 300 columns is far above the Infinity Cache
    assert ops.use_sliced(1_000_000, 300, torch.float32)
    assert ops.use_sliced(1_000_000, 300, torch.bfloat16)
    assert ops.use_sliced(1_000_000, 152, torch.float32)      # 4-GPU feature slice
    assert not ops.use_sliced(1_000_000, 76, torch.float32)   # 8-GPU slice stays row-major
    assert not ops.use_sliced(1_000_000, 152, torch.bfloat16)  # < two 256-B slices
    assert not ops.use_sliced(30_000, 300, torch.float32)     # DBP15K: cache resident
    assert not ops.use_sliced(1_000_000, 302, torch.float32)  # D % 4
    assert not ops.use_sliced(1_000_000, 300, torch.float64)
    monkeypatch.setattr(ops, "SLICED", False)
    assert not ops.use_sliced(1_000_000, 300, torch.float32)


def test_sliced_table_shape_and_map():
    t = ops.sliced_empty(10, 300, "cpu")
    assert t.shape == (5, 10, 64) and t.dtype == torch.float32
    tb = ops.sliced_empty(10, 300, "cpu", torch.bfloat16)
    assert tb.shape == (3, 10, 128)
    x = torch.arange(7 * 132, dtype=torch.float32).view(7, 132)
    xs = _slice_cpu(x, 64)
    flat = xs.reshape(-1)
    sstride = 7 * 64
    for r in range(7):
        for c in (0, 63, 64, 100, 131):
            assert flat[(c // 64) * sstride + r * 64 + c % 64] == x[r, c]
    # the test-side inverse used by the GPU tests
    assert torch.equal(xs.permute(1, 0, 2).reshape(7, -1)[:, :132], x)


def test_gat_sliced_wanted_slice_size_limit(monkeypatch):
    # the sliced GAT passes address a 64-column slice with 32-bit offsets (gat_sliced.hip
    # load_piece): below 4 GB per slice they apply above the Infinity Cache, beyond it the
    # head-grouped row-major passes take the table
    monkeypatch.setattr(ops, "GAT_SLICED", True)
    assert ops.gat_sliced_wanted(2_000_000, 4, 75, torch.float32)        # cfg-4: 512 MB slices
    assert not ops.gat_sliced_wanted(30_000, 4, 75, torch.float32)       # cache resident
    assert ops.gat_sliced_wanted(16_000_000, 4, 75, torch.float32)       # 4.1e9 B < 2^32 - 2^24
    assert not ops.gat_sliced_wanted(17_000_000, 4, 75, torch.float32)   # 4.35e9 B
