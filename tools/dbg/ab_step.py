"""A/B of step-level fusions: tools/dist_step.py with some of them disabled (debug tool):
    python tools/dbg/ab_step.py --off chain[,tadb] <dist_step.py arguments>
chain: ops.mlp_chain off (the MLP decoder layer by layer, LinearActFn / LinearFn);
tadb:  ops.gemm_ta_db off (dW and db as a product and a separate column-sum pass);
gcnbits: the GCN layer's relu backward from Y instead of the forward's sign bits."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))
sys.path.insert(0, ROOT)

from gnnea import ops  # noqa: E402

off = []
if "--off" in sys.argv:
    i = sys.argv.index("--off")
    off = sys.argv[i + 1].split(",")
    del sys.argv[i:i + 2]
if "chain" in off:
    ops.mlp_chain = lambda x, layers: None
if "tadb" in off:
    ops.gemm_ta_db = lambda a, b, out_dtype=None: None
if "gcnbits" in off:  # (the GCN layer keeps Y for its relu backward)
    ops.spmm_sliced_m = lambda csr, xs, D: (lambda y: (y, y))(
        ops.spmm_sliced(csr, xs, D, ops._lib.GNNEA_ACT_RELU))
    ops.act_bwd_sliced_bits = lambda dy, y, D: ops.act_bwd_sliced(dy, y, ops._lib.GNNEA_ACT_RELU)

from tools import dist_step  # noqa: E402

if __name__ == "__main__":
    dist_step.main()
