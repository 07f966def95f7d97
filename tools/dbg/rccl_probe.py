"""Probe: can two RCCL ranks share ONE device (the 1-GPU box)?  Each rank inits the nccl backend
on cuda:0, runs an all_reduce and one batch_isend_irecv exchange, prints what it saw.

    python tools/dbg/rccl_probe.py          (launches 2 ranks itself)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

if "WORLD_SIZE" not in os.environ:
    from tools import launch
    sys.exit(launch.spawn(2, os.path.abspath(__file__), []))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

rank = int(os.environ["RANK"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
try:
    dist.init_process_group("nccl", device_id=dev)
    t = torch.full((4,), float(rank + 1), device=dev)
    dist.all_reduce(t)
    peer = 1 - rank
    s = torch.full((1024,), float(rank), device=dev)
    r = torch.empty(1024, device=dev)
    for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, s, peer), dist.P2POp(dist.irecv, r, peer)]):
        w.wait()
    torch.cuda.synchronize()
    print("rank %d: all_reduce %s, recv %s" % (rank, t.tolist(), r[:2].tolist()), flush=True)
    dist.destroy_process_group()
except Exception as e:  # the probe reports, the launcher sees the status
    print("rank %d: %r" % (rank, e), flush=True)
    sys.exit(3)
