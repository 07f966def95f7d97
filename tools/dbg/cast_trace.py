"""Where do the bf16 <-> fp32 casts of the cfg-5 GAT-EA step come from?  Runs a few steps of
tools/dist_step.measure (GAT, bf16) on a small graph under a TorchDispatchMode that records every
aten dtype conversion (and fill) of a large tensor with the repo frames of its call stack.
    python tools/dbg/cast_trace.py [entities]"""
import collections
import json
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gnn-mtl_amd"))
sys.path.insert(0, ROOT)

SEEN = collections.Counter()
ON = [False]
_CASTS = {"aten._to_copy.default", "aten.copy_.default", "aten.to.dtype", "aten.fill_.Scalar",
          "aten.zeros_like.default", "aten.zero_.default", "aten.zeros.default",
          "aten.add.Tensor", "aten.add_.Tensor", "aten.new_zeros.default",
          "aten.empty_like.default", "aten.fill_.Tensor"}


class Trace(TorchDispatchMode):
    """Every aten op that changes dtype (or fills) a large tensor, with the repo frames of the
    Python stack (empty for ops the autograd engine issues from its own thread)."""

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = str(func)
        if ON[0] and name in _CASTS and isinstance(out, torch.Tensor) and out.numel() >= 100000:
            src = args[1] if name == "aten.copy_.default" else args[0]
            sd = src.dtype if isinstance(src, torch.Tensor) else None
            if name.startswith("aten.fill") or name.startswith("aten.zero") or \
                    name.startswith("aten.add") or name.startswith("aten.new_zeros") or sd != out.dtype:
                frames = [f for f in traceback.extract_stack()[:-1] if ROOT in f.filename]
                key = "%s %s -> %s %s | %s" % (name, sd, out.dtype, tuple(out.shape), " < ".join(
                    "%s:%d" % (os.path.relpath(f.filename, ROOT), f.lineno)
                    for f in reversed(frames[-4:])))
                SEEN[key] += 1
        return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    from tools.dist_step import measure
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    measure("GAT", n, 0, 1, dev, 1, 1, torch.bfloat16, attribute=0)  # warm (lazy setup)
    SEEN.clear()
    ON[0] = True
    # the backward on this thread (the autograd engine's device threads do not see the mode)
    with torch.autograd.set_multithreading_enabled(False), Trace():
        measure("GAT", n, 0, 1, dev, 1, 1, torch.bfloat16, attribute=0)
    ON[0] = False
    for k, v in SEEN.most_common():
        print(json.dumps({"calls": v, "cast": k}))


if __name__ == "__main__":
    main()
