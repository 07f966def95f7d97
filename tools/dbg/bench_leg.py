"""Run one side leg of bench.py on cuda:0 and print its JSON (debug tool):
python tools/dbg/bench_leg.py {bf16|anchors|fgw|sinkhorn|sinkhorn_large} [libgnnea_<variant>.so]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))
from gnnea import _lib  # noqa: E402
if len(sys.argv) > 2:  # an A/B build of the library, loaded instead of the default one
    _lib.LIB_PATH = os.path.join(os.path.dirname(_lib.LIB_PATH), sys.argv[2])
import bench  # noqa: E402

dev = torch.device("cuda:0")
leg = sys.argv[1]
fn = {"bf16": lambda: bench.bf16_rate(dev, 20), "anchors": lambda: bench.anchors(dev),
      "fgw": lambda: bench.fgw_rate(dev), "sinkhorn": lambda: bench.sinkhorn_rate(dev),
      "sinkhorn_large": lambda: bench.sinkhorn_large(dev)}[leg]
print(json.dumps({leg: fn()}), flush=True)
