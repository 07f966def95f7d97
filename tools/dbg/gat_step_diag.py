"""Diagnose the GAT-EA step's last-layer weight gradient at DBP15K scale (debug tool, GPU).

Splits the error of decoder.cls.2.linear.weight.grad vs the reference's fp64 step into
  (1) the margin backward given our fp32 outputs (our kernel vs fp64 autograd of the reference
      formula at the same outputs), and
  (2) the sensitivity of the sign pattern to the forward's rounding.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "gnn-mtl_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import fp64_ref  # noqa: E402
import scale_inputs as si  # noqa: E402
from conftest import rel_err  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    f = dict(np.load(os.path.join(ROOT, "tests/golden/dbp15k.npz")))
    tr, N, r, c, v = si.dbp15k_graph()
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.stack([r, c])), torch.from_numpy(v),
                                  (N, N)).to(dev)
    X = si.features(N)
    from models.models_ea import EAModel
    from test_dropin_cpu import make_args
    train = f["train"]
    t, k = train.shape[0], 125
    model = sys.argv[1] if len(sys.argv) > 1 else "GAT"
    a = make_args(model)
    a.cuda, a.device = 0, dev
    a.n_nodes, a.neg_num, a.data = N, k, {"train": train}
    torch.manual_seed(10086)
    m = EAModel(a).to(dev)
    m.train()
    saved = {}
    last = m.decoder.cls[2] if model in ("GCN", "GAT") else m.decoder.cls
    last.register_forward_hook(lambda mod, inp, out: saved.__setitem__("h2", inp[0]))
    xs = torch.from_numpy(X).to_sparse().to(dev)
    outputs = m.decode(m.encode(xs, adj), adj)
    outputs.retain_grad()
    m.neg_right = si.negatives(N, t, k, 31)
    m.neg2_left = si.negatives(N, t, k, 32)
    loss = m.get_loss(outputs, {"train": train}, "train")
    loss.backward()
    G = outputs.grad.double()
    o64 = outputs.detach().double().requires_grad_(True)
    ix = [torch.from_numpy(np.asarray(z, dtype=np.int64)).to(dev) for z in
          (train[:, 0], train[:, 1], m.neg_left, m.neg_right, m.neg2_left, m.neg2_right)]
    L64 = fp64_ref.margin_loss(o64, *ix, t, k)
    L64.backward()
    print("loss ours %.9g fp64-at-ours %.9g ref32 %.9g ref64 %.9g" %
          (float(loss), float(L64), float(f[model + "_loss"]), float(f[model + "_loss64"])))
    print("dL/dout: ours vs fp64 autograd at our outputs: rel %.3e" % rel_err(G.cpu(), o64.grad.cpu()))
    h2 = saved["h2"][0] if isinstance(saved["h2"], tuple) else saved["h2"]
    h2 = h2.detach().double()
    name = [n for n, p in m.named_parameters()][-2]
    ref64 = f["%s_grad64.%s" % (model, name)]
    ref32 = f["%s_grad.%s" % (model, name)]
    ours = dict(m.named_parameters())[name].grad.double().cpu().numpy()
    dW_from64G = (o64.grad.t() @ h2).cpu().numpy() if model in ("GCN", "GAT") else None
    print(name)
    print("  ours vs ref64 %.3e   ref32 vs ref64 %.3e   ours vs ref32 %.3e" %
          (rel_err(ours, ref64), rel_err(ref32, ref64), rel_err(ours, ref32)))
    if dW_from64G is not None:
        print("  fp64 G at our outputs x our h2 vs ours %.3e, vs ref64 %.3e" %
              (rel_err(dW_from64G, ours), rel_err(dW_from64G, ref64)))
    rows = torch.from_numpy(f["rows"]).to(dev)
    print("  sampled outputs ours vs ref32 %.3e" % rel_err(outputs.detach()[rows].cpu(),
                                                         f[model + "_out"]))
    # near-tie statistics of the term differences
    od = outputs.detach()
    for nm, (aa, bb) in (("pos", (ix[0], ix[1])), ("neg1", (ix[2], ix[3])), ("neg2", (ix[4], ix[5]))):
        d = (od[aa] - od[bb]).abs()
        scale = od.abs().max()
        print("  %s terms: exact zero diffs %d, |d| < 1e-6*max %d, < 1e-5*max %d of %d" %
              (nm, int((d == 0).sum()), int((d < 1e-6 * scale).sum()),
               int((d < 1e-5 * scale).sum()), d.numel()))
    print("  outputs: exact zeros %d of %d, max |out| %.3e" % (int((od == 0).sum()), od.numel(),
                                                             float(od.abs().max())))
    print("  h2: exact zeros %d of %d" % (int((h2 == 0).sum()), h2.numel()))


if __name__ == "__main__":
    main()
