"""fp64 restatement of the EA margin loss (§8f #2) — TEST INFRASTRUCTURE ONLY.

models/models_ea.py:103-123 (EAModel.get_loss): A = |x[left] - x[right]|_1,
B_s = |x[nl_s] - x[nr_s]|_1, loss = (sum relu(A + 1 - B_1) + sum relu(A + 1 - B_2)) / (2 t k);
gradient by torch autograd in fp64.
"""
import numpy as np
import torch


def margin_loss_and_grad(vec, left, right, nl1, nr1, nl2, nr2, t, k):
    x = torch.tensor(np.asarray(vec, np.float64), requires_grad=True)

    def ix(a):
        return torch.as_tensor(np.asarray(a).astype(np.int64))

    A = torch.sum(torch.abs(x[ix(left)] - x[ix(right)]), 1).reshape(t, 1) + 1.0
    B1 = torch.sum(torch.abs(x[ix(nl1)] - x[ix(nr1)]), 1).reshape(t, k)
    B2 = torch.sum(torch.abs(x[ix(nl2)] - x[ix(nr2)]), 1).reshape(t, k)
    loss = (torch.relu(A - B1).sum() + torch.relu(A - B2).sum()) / (2.0 * t * k)
    loss.backward()
    return float(loss.detach()), x.grad.numpy()
