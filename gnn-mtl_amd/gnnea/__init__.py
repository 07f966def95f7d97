"""gnnea — MI355X-native hot path of the GNN entity-alignment engine.

Host package around libgnnea.so (include/gnnea.h): device CSR cache (graph), HIP ops and their
autograd wrappers (ops), the Sinkhorn host driver (sinkhorn), synthetic inputs (synth) and the
multi-GPU node sharding (dist).  The drop-in mirrors of the reference modules live next to this
package (layers/, models/, utils/, SinkhornOT/) and call into it.
"""
from . import _lib  # noqa: F401
from ._lib import GnneaError, lib  # noqa: F401

__all__ = ["GnneaError", "lib"]
