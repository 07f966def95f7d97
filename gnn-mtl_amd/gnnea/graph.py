"""Device CSR of the reference's adjacency (SURVEY.md §8a a1, §8b "CSR cache").

The reference hands every layer the same torch sparse COO object (``data['adj']``,
utils/data_utils.py:398-399, moved to the device at run/train_ea.py:42-44): uncoalesced,
int64 indices, fp32 values.  ``torch.spmm`` coalesces it on every call (layers/layers.py:35) and
GAT calls ``adj.coalesce()`` once per head per forward (layers/att_layers.py:31).  Here it is
converted once, on the device, to an int32 CSR (and lazily its transpose for the backward pass)
and cached per adjacency object.
"""
import weakref

import torch

from . import _lib


class DeviceCSR:
    """int32 CSR on a HIP device: rowptr[n_rows+1], col[nnz], val[nnz] sorted by (row, col).

    ``transpose()`` returns the CSR of A^T with ``perm`` mapping each transposed entry to its
    position in this CSR (used by the GAT backward to find dz of edge (i, j) from row j).
    """

    def __init__(self, rowptr, col, val, n_rows, n_cols, perm=None):
        self.rowptr = rowptr
        self.col = col
        self.val = val
        self.n_rows = int(n_rows)
        self.n_cols = int(n_cols)
        self.nnz = int(col.numel())
        self.perm = perm
        self._t = None
        self.device = rowptr.device

    @staticmethod
    def from_coo(row, col, val, n_rows, n_cols, want_perm=False):
        """Coalescing COO -> CSR conversion on the device (gnnea_coo_to_csr)."""
        _lib.require_device(row, col)
        dev = row.device
        L = _lib.lib()
        nnz = int(row.numel())
        if col.dtype != row.dtype or row.dtype not in (torch.int32, torch.int64):
            raise ValueError("gnnea: COO indices must be int32 or int64 of one dtype")
        row = row.contiguous()
        col = col.contiguous()
        if val is not None:
            val = val.to(device=dev, dtype=torch.float32).contiguous()
        ws_bytes = int(L.gnnea_coo_to_csr_ws_bytes(nnz, n_rows, n_cols))
        if ws_bytes < 0:
            _lib.check(ws_bytes)
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        rowptr = torch.empty(n_rows + 1, dtype=torch.int32, device=dev)
        col_out = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)
        val_out = torch.empty(max(nnz, 1), dtype=torch.float32, device=dev)
        perm = torch.empty(max(nnz, 1), dtype=torch.int64, device=dev) if want_perm else None
        nnz_out = torch.zeros(1, dtype=torch.int64, device=dev)
        with _lib.on_device(dev):
            _lib.check(L.gnnea_coo_to_csr(
                _lib.ptr(row), _lib.ptr(col), row.element_size(), _lib.ptr(val), nnz, n_rows,
                n_cols, _lib.ptr(rowptr), _lib.ptr(col_out), _lib.ptr(val_out), _lib.ptr(perm),
                _lib.ptr(nnz_out), _lib.ptr(ws), ws_bytes, _lib.stream_of(dev)))
        n = int(nnz_out.item())  # one-time setup sync
        if n < 0:
            raise ValueError("gnnea: COO index out of range for shape (%d, %d)" % (n_rows, n_cols))
        del ws
        return DeviceCSR(rowptr, col_out[:n], val_out[:n], n_rows, n_cols,
                         perm[:n] if perm is not None else None)

    def row_ids(self):
        L = _lib.lib()
        rows = torch.empty(max(self.nnz, 1), dtype=torch.int32, device=self.device)
        with _lib.on_device(self.device):
            _lib.check(L.gnnea_csr_expand_rows(_lib.ptr(self.rowptr), self.n_rows, self.nnz,
                                               _lib.ptr(rows), _lib.stream_of(self.device)))
        return rows[:self.nnz]

    def transpose(self):
        if self._t is None:
            rows = self.row_ids()
            self._t = DeviceCSR.from_coo(self.col, rows, self.val, self.n_cols, self.n_rows,
                                         want_perm=True)
        return self._t

    def tpos(self):
        """Position in transpose() of every entry of this CSR (inverse of transpose().perm)."""
        if getattr(self, "_tpos", None) is None:
            t = self.transpose()
            inv = torch.empty(max(self.nnz, 1), dtype=torch.int64, device=self.device)
            with _lib.on_device(self.device):
                _lib.check(_lib.lib().gnnea_perm_invert(_lib.ptr(t.perm), self.nnz,
                                                        _lib.ptr(inv),
                                                        _lib.stream_of(self.device)))
            self._tpos = inv[:self.nnz]
        return self._tpos

    def degrees(self):
        return (self.rowptr[1:] - self.rowptr[:-1])

    MIN_BLOCK_ROWS = 1 << 18  # a block must still fill the chip (256 CUs x 4 waves x 256 rows)

    def row_blocks(self):
        """Row ranges [r0, r1) of the diagonal blocks of a block-diagonal matrix (the two KGs of
        the EA adjacency: KG1 rows only reference KG1 columns), merged to >= MIN_BLOCK_ROWS rows.
        Launching the blocks one after another keeps the gathered rows of one block only in
        flight, so the Infinity Cache holds a larger share of them (one setup sync, cached)."""
        if getattr(self, "_blocks", None) is None:
            n = self.n_rows
            blocks = [(0, n)]
            if n >= 2 * self.MIN_BLOCK_ROWS and self.nnz > 0 and self.n_cols == n:
                rp = self.rowptr.long()
                nonempty = rp[1:] > rp[:-1]
                last = self.col[(rp[1:] - 1).clamp(min=0)].long()
                first = self.col[rp[:-1].clamp(max=self.nnz - 1)].long()
                maxc = torch.where(nonempty, last, torch.full_like(last, -1))
                minc = torch.where(nonempty, first, torch.full_like(first, n))
                pmax = torch.cummax(maxc, 0).values
                smin = torch.flip(torch.cummin(torch.flip(minc, [0]), 0).values, [0])
                r = torch.arange(n, device=self.device)
                # split before row s: rows < s only reference cols < s, rows >= s cols >= s
                ok = (pmax[:-1] <= r[:-1]) & (smin[1:] >= r[1:])
                cuts = (torch.nonzero(ok).flatten() + 1).tolist()
                blocks, start = [], 0
                for c in cuts:
                    if c - start >= self.MIN_BLOCK_ROWS and n - c >= self.MIN_BLOCK_ROWS:
                        blocks.append((start, c))
                        start = c
                blocks.append((start, n))
            self._blocks = blocks
        return self._blocks


_CACHE = {}


def _evict(key):
    _CACHE.pop(key, None)


def csr_of(adj):
    """CSR of a torch sparse COO adjacency, built once per tensor object (weakly cached)."""
    if isinstance(adj, DeviceCSR):
        return adj
    if not adj.is_sparse:
        raise TypeError("gnnea: csr_of expects a torch sparse COO tensor")
    key = id(adj)
    hit = _CACHE.get(key)
    if hit is not None:
        ref, csr, version = hit
        if ref() is adj and version == adj._values()._version:
            return csr
    _lib.require_device(adj)
    n_rows, n_cols = adj.shape
    idx = adj._indices()
    csr = DeviceCSR.from_coo(idx[0], idx[1], adj._values(), n_rows, n_cols)
    try:
        ref = weakref.ref(adj, lambda _r, k=key: _evict(k))
    except TypeError:  # pragma: no cover - tensors support weakrefs
        ref = lambda: adj  # noqa: E731
    _CACHE[key] = (ref, csr, adj._values()._version)
    return csr


_DENSE = {}


def dense_of(x):
    """Dense view of a (possibly sparse-COO) feature matrix, densified once per object.

    The reference stores the features as a sparse COO tensor with fully dense content
    (utils/data_utils.py:352-358, 396-397) and multiplies it with ``nn.Linear`` every epoch.
    """
    if not x.is_sparse:
        return x
    key = id(x)
    hit = _DENSE.get(key)
    if hit is not None and hit[0]() is x:
        return hit[1]
    d = x.to_dense()
    _DENSE[key] = (weakref.ref(x, lambda _r, k=key: _DENSE.pop(k, None)), d)
    return d
