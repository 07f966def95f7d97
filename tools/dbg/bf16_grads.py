"""Debug: per-parameter cosine of bf16 vs fp32 model gradients (GPU)."""
import sys, os
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "gnn-mtl_amd"), os.path.join(ROOT, "tests"), ROOT]
from models.decoders import model2decoder
from models.encoders import model2encoder
from gnnea.margin import margin_loss
from test_dropin_cpu import make_args
g = np.load(os.path.join(ROOT, "tests/golden/graph_cfg1.npz"))
device = torch.device("cuda:0")
for model in sys.argv[1:]:
    a = make_args(model); a.cuda, a.device = 0, device
    torch.manual_seed(10086)
    enc = model2encoder[model](a).to(device); dec = model2decoder[model](a).to(device)
    idx = torch.from_numpy(np.stack([g["row"], g["col"]]).astype(np.int64))
    adj = torch.sparse_coo_tensor(idx, torch.from_numpy(g["val"]), (2000, 2000)).to(device)
    x = torch.from_numpy(g["X"]).to(device)
    rng = np.random.default_rng(0)
    t, k = 200, 5
    left, right = rng.integers(0, 1000, t), rng.integers(1000, 2000, t)
    negs = [rng.integers(0, 2000, t * k) for _ in range(4)]
    res = {}
    for dtype in (torch.float32, torch.bfloat16):
        e, d = enc.to(dtype), dec.to(dtype)
        e.zero_grad(); d.zero_grad()
        out = d.decode(e.encode(x.to(dtype), adj), adj)
        loss = margin_loss(out, left, right, np.repeat(left, k), negs[0], negs[1], np.repeat(right, k), t, k)
        loss.backward()
        res[dtype] = {n: p.grad.float().cpu().clone() for n, p in list(e.named_parameters()) + [("dec." + n, p) for n, p in d.named_parameters()]}
    for n in res[torch.float32]:
        p32, p16 = res[torch.float32][n], res[torch.bfloat16][n]
        cos = float(torch.nn.functional.cosine_similarity(p16.flatten().double(), p32.flatten().double(), dim=0))
        print(model, n, tuple(p32.shape), "cos %.4f" % cos, "n32 %.3e n16 %.3e" % (p32.norm(), p16.norm()))
