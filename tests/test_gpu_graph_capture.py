"""A whole EA training iteration (encode + decode + margin loss + backward + Adam) captured as one
HIP graph through the drop-in modules replays bit-identically to the eager iteration
(tools/graph_step.py; run/train_ea.py:55-66): every libgnnea launch takes the caller's current
stream, allocates nothing the capture cannot own and syncs nothing with the host after warm-up."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("model", ["GCN", "HGCN", "GAT"])
def test_ea_iteration_graph_replay_matches_eager(model):
    from tools.graph_step import run
    r = run(model, 1000, 2500, 5, torch.device("cuda", 0))  # cfg-1 sized pair
    p = r["parity"]
    assert p["loss_rel"] == 0.0 and p["grad_max_rel"] == 0.0 and p["param_max_rel"] == 0.0, p
    assert r["graph_ms"] > 0 and r["eager_ms"] > 0
