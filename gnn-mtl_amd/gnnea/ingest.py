"""ctypes binding of libgnnea_host.so: KG ingestion on the host (include/gnnea_host.h, §8f #4).

The reference's loaders parse files line by line and build the adjacency with Python dicts
(utils/data_utils.py:272-372); these calls do the same work in parallel C++ and hand back numpy
arrays.  Pure host code: no GPU, no torch types.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgnnea_host.so")

_p = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64

SIGNATURES = {
    "gnnea_h_loadfile": (_i64, [ctypes.c_char_p, _i32, _p, _i64]),
    "gnnea_h_adjacency": (_i64, [_p, _i64, _i64, _i32, _p, _p, _p, _i64]),
    "gnnea_h_relation_groups": (_i64, [_p, _i64, _i64, _p, _p, _p]),
}

_ERR = {-1: "bad argument", -2: "cannot read file", -3: "line does not hold the integer fields",
        -4: "output capacity too small"}
_LIB = None


class IngestError(RuntimeError):
    pass


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise IngestError("gnnea: host library %s is not built (make -C gnn-mtl_amd/csrc)"
                              % LIB_PATH)
        h = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = h
    return _LIB


def _check(rc, what):
    if rc < 0:
        raise IngestError("gnnea ingest %s: %s" % (what, _ERR.get(int(rc), str(rc))))
    return int(rc)


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def loadfile_array(fn, num=1):
    """int64 [rows, num] of loadfile(fn, num) (utils/data_utils.py:362-372)."""
    L = lib()
    path = os.fsencode(fn)
    n = _check(L.gnnea_h_loadfile(path, num, None, 0), fn)
    out = np.empty((n, num), dtype=np.int64)
    _check(L.gnnea_h_loadfile(path, num, _ptr(out), n), fn)
    return out


def adjacency(triples, n_ent, reference_order=True):
    """(row int64, col int64, val float32) of get_sparse_tensor(n_ent, triples)."""
    tr = np.ascontiguousarray(np.asarray(triples, dtype=np.int64).reshape(-1, 3))
    L = lib()
    nnz = _check(L.gnnea_h_adjacency(_ptr(tr), len(tr), n_ent, int(reference_order), None, None,
                                     None, 0), "adjacency")
    row = np.empty(nnz, dtype=np.int64)
    col = np.empty(nnz, dtype=np.int64)
    val = np.empty(nnz, dtype=np.float32)
    _check(L.gnnea_h_adjacency(_ptr(tr), len(tr), n_ent, int(reference_order), _ptr(row),
                               _ptr(col), _ptr(val), nnz), "adjacency")
    return row, col, val


def relation_groups(triples, n_rel):
    """(rel_ptr [n_rel+1], heads, tails): the triples grouped by relation, triple order kept."""
    tr = np.ascontiguousarray(np.asarray(triples, dtype=np.int64).reshape(-1, 3))
    ptr = np.empty(n_rel + 1, dtype=np.int64)
    heads = np.empty(len(tr), dtype=np.int64)
    tails = np.empty(len(tr), dtype=np.int64)
    _check(lib().gnnea_h_relation_groups(_ptr(tr), len(tr), n_rel, _ptr(ptr), _ptr(heads),
                                         _ptr(tails)), "relation groups")
    return ptr, heads, tails
