"""bench.py --gpus N launches its own N ranks when no launcher did (tools/launch.py): rank
environment, relayed rank-0 line, non-zero exit when a rank fails, and a parent that never
initialises HIP."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tools import launch  # noqa: E402

STUB = r'''
import json, os, sys, time
r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
mode = sys.argv[1]
if mode == "fail" and r == 1:
    sys.exit(7)
if mode == "fail":
    time.sleep(60)  # a rank left waiting for a peer that died
if mode == "gloo":
    import torch, torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.tensor([float(r)])
    dist.all_reduce(t)
    dist.destroy_process_group()
    if r == 0:
        print(json.dumps({"n_gpus": w, "sum": t.item(),
                          "addr": os.environ["MASTER_ADDR"]}), flush=True)
    sys.exit(0)
if r == 0:
    print(json.dumps({"n_gpus": w, "local": os.environ["LOCAL_RANK"],
                      "addr": os.environ["MASTER_ADDR"], "argv": sys.argv[1:]}), flush=True)
'''


@pytest.fixture
def stub(tmp_path):
    p = tmp_path / "stub.py"
    p.write_text(STUB)
    return str(p)


def test_requested_ranks_and_need():
    assert launch.requested_ranks(["--steps", "3"]) == 1
    assert launch.requested_ranks(["--gpus", "8", "--steps", "3"]) == 8
    assert launch.requested_ranks(["--gpus=4"]) == 4
    assert launch.needs_launch(["--gpus", "2"], environ={})
    assert not launch.needs_launch(["--gpus", "2"], environ={"WORLD_SIZE": "2"})
    assert not launch.needs_launch(["--gpus", "1"], environ={})


def _run_parent(code, timeout=120):
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                          timeout=timeout, cwd=ROOT,
                          env={k: v for k, v in os.environ.items()
                               if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})


def test_bench_parent_launches_ranks_without_hip(stub):
    """bench.self_launch starts the children and returns their status; the parent process has
    not initialised HIP (torch.cuda stays uninitialised)."""
    code = ("import sys, json; sys.path.insert(0, %r); import bench, torch; "
            "rc = bench.self_launch(['--gpus', '3', 'ok'], script=%r); "
            "print('PARENT', json.dumps({'rc': rc, 'cuda_init': torch.cuda.is_initialized()}))"
            % (ROOT, stub))
    r = _run_parent(code)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    child = json.loads([ln for ln in lines if not ln.startswith("PARENT")][0])
    parent = json.loads([ln for ln in lines if ln.startswith("PARENT")][0].split(" ", 1)[1])
    assert child["n_gpus"] == 3 and child["local"] == "0" and child["addr"] == "127.0.0.1"
    assert child["argv"] == ["--gpus", "3", "ok"]
    assert parent == {"rc": 0, "cuda_init": False}


def test_bench_is_a_rank_under_a_launcher():
    import bench
    os.environ["WORLD_SIZE"] = "2"
    try:
        assert bench.self_launch(["--gpus", "2"]) is None
    finally:
        del os.environ["WORLD_SIZE"]
    assert bench.self_launch(["--gpus", "1"]) is None


def test_failing_rank_stops_the_run(stub):
    t0 = time.time()
    rc = launch.spawn(2, stub, ["fail"], environ={k: v for k, v in os.environ.items()
                                                  if k != "WORLD_SIZE"})
    assert rc == 7
    assert time.time() - t0 < 40  # the waiting rank was terminated, not waited for


def test_launched_ranks_rendezvous_gloo(stub, capfd):
    rc = launch.spawn(2, stub, ["gloo"])
    assert rc == 0
    out = capfd.readouterr().out
    line = json.loads([ln for ln in out.splitlines() if ln.startswith("{")][0])
    assert line == {"n_gpus": 2, "sum": 1.0, "addr": "127.0.0.1"}
