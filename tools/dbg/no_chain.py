"""A/B of the fused MLP decoder (ops.MLPChainFn): tools/dist_step.py with ops.mlp_chain disabled, so
the decoder runs layer by layer (LinearActFn / LinearFn) -- debug tool, same arguments as
dist_step.py."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))
sys.path.insert(0, ROOT)

from gnnea import ops  # noqa: E402

ops.mlp_chain = lambda x, layers: None

from tools import dist_step  # noqa: E402

if __name__ == "__main__":
    dist_step.main()
