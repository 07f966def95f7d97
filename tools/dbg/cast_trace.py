"""Where do the bf16 <-> fp32 casts of the cfg-5 GAT-EA step come from?  Runs a few steps of
tools/dist_step.measure (GAT, bf16) on a small graph under a TorchFunctionMode that records every
dtype conversion of a large tensor with the repo frames of its call stack.
    python tools/dbg/cast_trace.py [entities]"""
import collections
import json
import os
import sys
import traceback

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))
sys.path.insert(0, ROOT)

SEEN = collections.Counter()


ON = [False]


def _record(src, out):
    if ON[0] and isinstance(src, torch.Tensor) and isinstance(out, torch.Tensor) and \
            src.dtype != out.dtype and out.numel() >= 100000 and \
            {src.dtype, out.dtype} <= {torch.float32, torch.bfloat16}:
        frames = [f for f in traceback.extract_stack()[:-2] if ROOT in f.filename]
        key = "%s -> %s %s | %s" % (src.dtype, out.dtype, tuple(out.shape), " < ".join(
            "%s:%d" % (os.path.relpath(f.filename, ROOT), f.lineno)
            for f in reversed(frames[-4:])))
        SEEN[key] += 1


def _wrap(name):
    orig = getattr(torch.Tensor, name)

    def f(self, *a, **k):
        out = orig(self, *a, **k)
        _record(self, out)
        return out
    setattr(torch.Tensor, name, f)


for _n in ("to", "float", "bfloat16", "type", "type_as"):
    _wrap(_n)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    from tools.dist_step import measure
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    measure("GAT", n, 0, 1, dev, 1, 1, torch.bfloat16, attribute=0)  # warm (lazy setup)
    SEEN.clear()
    ON[0] = True
    measure("GAT", n, 0, 1, dev, 1, 1, torch.bfloat16, attribute=0)
    ON[0] = False
    for k, v in SEEN.most_common():
        print(json.dumps({"calls": v, "cast": k}))


if __name__ == "__main__":
    main()
