# Drop-in package: sinkhorn_loss.py here runs the solvers on HIP; the reference's GW / FGW outer
# loops (SinkhornOT/iterative_projection.py, cderivation.py) are found further down sys.path when
# the reference is installed, and then call these solvers through their relative imports.
from pkgutil import extend_path

__path__ = extend_path(__path__, __name__)

from .sinkhorn_loss import (forward_relax_sinkhorn_iteration, gsinkhorn_iteration,  # noqa: E402,F401
                            kl_div, sinkhorn_iteration)

try:  # optional upstream GW / FGW outer loops (SURVEY.md §8f #3 — not rebuilt yet)
    from .cderivation import cos_dist_mat, get_inter_sim, get_intra_sim  # noqa: F401
    from .iterative_projection import gw_iterative_1, rgw_iterative_1  # noqa: F401
except ImportError:
    pass
