"""gnnea — MI355X-native hot path of the GNN entity-alignment engine.

Host package around libgnnea.so (include/gnnea.h): device CSR cache (graph), HIP ops and their
autograd wrappers (ops), the Sinkhorn host driver (sinkhorn), synthetic inputs (synth) and the
multi-GPU node sharding (dist).  The drop-in mirrors of the reference modules live next to this
package (layers/, models/, utils/, SinkhornOT/) and call into it.
"""
from . import _lib  # noqa: F401
from ._lib import GnneaError, lib  # noqa: F401

__all__ = ["GnneaError", "lib", "release"]


def release():
    """Drop every device / pinned buffer the package caches (CSR and dense-feature caches, GEMM
    workspaces, sliced copies, margin incidences) and hand torch's cached device and pinned
    blocks back to the HIP runtime, after the queue has drained.  For a deterministic teardown
    at the end of a run: nothing is left for the runtime's own exit handlers to free."""
    import gc
    import sys

    import torch
    for name, attrs in (("gnnea.graph", ("_CACHE", "_DENSE")),
                        ("gnnea.ops", ("_WS", "_SLICED_COPIES", "_ONES")),
                        ("gnnea.margin", ("_DEV_IDX", "_INCIDENCE"))):
        mod = sys.modules.get(name)
        for a in attrs if mod is not None else ():
            getattr(mod, a).clear()
    gc.collect()
    if torch.cuda.is_initialized():
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        host_empty = getattr(torch._C, "_host_emptyCache", None)
        if host_empty is not None:
            host_empty()
