# Drop-in package: sinkhorn_loss.py runs the solvers on HIP, cderivation.py /
# iterative_projection.py are the GW / FGW outer loops on device GEMMs around them.  Modules not
# rebuilt here (fgw.py, which needs the un-vendored UMH package) are found further down sys.path
# when the reference is installed.
from pkgutil import extend_path

__path__ = extend_path(__path__, __name__)

from .sinkhorn_loss import (forward_relax_sinkhorn_iteration, gsinkhorn_iteration,  # noqa: E402,F401
                            kl_div, sinkhorn_iteration)
from .cderivation import cos_dist_mat, get_inter_sim, get_intra_sim  # noqa: E402,F401
from .iterative_projection import (fgw_iterative_1, gw_iterative_1,  # noqa: E402,F401
                                   rfgw_iterative_1, rgw_iterative_1)
