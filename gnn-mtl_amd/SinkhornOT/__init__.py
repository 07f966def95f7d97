from .sinkhorn_loss import (forward_relax_sinkhorn_iteration, gsinkhorn_iteration,  # noqa: F401
                            kl_div, sinkhorn_iteration)
