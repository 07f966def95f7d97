"""Sinkhorn iters/s at the EA batch through each KNOPP device path (A/B of k_sk_res vs the
resident-K sweep): python tools/sk_bench.py [B ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
import torch  # noqa: E402
from gnnea import _lib  # noqa: E402

dev = torch.device("cuda", 0)
for B in [int(x) for x in sys.argv[1:]] or [3000]:
    for fl in (0, _lib.GNNEA_SK_NO_ONCHIP):
        r = bench.sinkhorn_rate(dev, B=B, flags=fl)
        print(json.dumps({"B": B, "onchip": fl == 0, **r["iters_per_s"]}), flush=True)
if os.environ.get("SK_LOG"):
    r = bench.sinkhorn_rate(dev, B=15000, n0=20, n1=120, variant=1)
    print(json.dumps({"B": 15000, "logdomain": True, **r["iters_per_s"]}), flush=True)
