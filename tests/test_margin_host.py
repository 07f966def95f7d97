"""Host side of the fused margin loss (no GPU): the device copies of the reference's numpy index
arrays are cached per array, so the per-step loss reuses them (and the incidence CSR built on
them) until the negatives are reassigned (run/train_ea.py:61-62)."""
import numpy as np
import pytest
import torch

from gnnea import margin


def test_index_copies_cached_per_array():
    cpu = torch.device("cpu")
    ILL = np.arange(40).reshape(20, 2)
    a1 = margin._idx_cached(ILL[:, 0], cpu, 100)  # a fresh view object every epoch ...
    a2 = margin._idx_cached(ILL[:, 0], cpu, 100)
    assert a1 is a2                                # ... maps to the same device copy
    assert torch.equal(a1, torch.arange(0, 40, 2))
    b = margin._idx_cached(ILL[:, 1], cpu, 100)    # other column: other pointer
    assert b is not a1 and torch.equal(b, torch.arange(1, 40, 2))
    neg = np.ones((20 * 3,)) * 7.0                 # the reference's float64 np.ones products
    n1 = margin._idx_cached(neg, cpu, 100)
    assert n1 is margin._idx_cached(neg, cpu, 100) and n1.dtype == torch.int64
    neg2 = neg.copy()                              # reassigned negatives: a new array
    assert margin._idx_cached(neg2, cpu, 100) is not n1
    with pytest.raises(IndexError):
        margin._idx_cached(np.array([0, 100]), cpu, 100)
