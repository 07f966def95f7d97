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
if mode == "ignore_term":  # a rank that survives SIGTERM (stuck in a collective, say)
    import signal
    signal.signal(signal.SIGTERM, signal.SIG_IGN)
    open(sys.argv[2] + ".%d" % r, "w").write(str(os.getpid()))
    time.sleep(120)
    sys.exit(0)
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


def _alive(pid):
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    try:  # a zombie (exited, not yet reaped by its new parent) is not running
        with open("/proc/%d/stat" % pid) as f:
            return f.read().split(")")[-1].split()[0] != "Z"
    except OSError:
        return False


def test_signal_to_parent_kills_ranks_that_ignore_sigterm(stub, tmp_path):
    """An outer time limit's SIGTERM to the launching process is forwarded to the ranks; ranks
    still running after the grace period (here: ignoring SIGTERM) are SIGKILLed before the
    parent exits with 128 + SIGTERM."""
    import signal
    marker = str(tmp_path / "pid")
    code = ("import sys; sys.path.insert(0, %r); from tools import launch; "
            "sys.exit(launch.spawn(2, %r, ['ignore_term', %r], grace_s=2.0))"
            % (ROOT, stub, marker))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    parent = subprocess.Popen([sys.executable, "-c", code], cwd=ROOT, env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    try:
        t0 = time.time()
        while not all(os.path.exists(marker + ".%d" % r) for r in range(2)):
            assert parent.poll() is None and time.time() - t0 < 60, parent.communicate()
            time.sleep(0.1)
        pids = [int(open(marker + ".%d" % r).read()) for r in range(2)]
        t1 = time.time()
        parent.send_signal(signal.SIGTERM)
        rc = parent.wait(timeout=60)
        assert rc == 128 + signal.SIGTERM, parent.communicate()
        assert time.time() - t1 < 30  # the grace period, then SIGKILL: not the ranks' 120 s
        t2 = time.time()
        while any(_alive(p) for p in pids) and time.time() - t2 < 10:
            time.sleep(0.1)
        assert not any(_alive(p) for p in pids), pids
    finally:
        if parent.poll() is None:
            parent.kill()
