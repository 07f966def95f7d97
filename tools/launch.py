"""One process per GPU for `bench.py --gpus N` when no launcher set the rank environment.

The driver may start the bench either as ``python -m torch.distributed.run --nproc-per-node N
bench.py --gpus N`` (RANK / WORLD_SIZE already set: nothing here runs) or as a plain
``python bench.py --gpus N``.  In the second case the parent process starts N fresh Python
children running the same script with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT set (rendezvous on 127.0.0.1), relays their output (the children inherit stdout /
stderr; only rank 0 prints the JSON line), and returns the first non-zero child exit status.

The parent never touches HIP: this module imports only the standard library, and bench.py calls
it before ``import torch``.  A child that fails ends the run: the remaining children (the exact
PIDs started here) get SIGTERM, then SIGKILL after a grace period, so no rank is left waiting in
a collective for a peer that is gone.
"""
import os
import signal
import socket
import subprocess
import sys
import time

GRACE_S = 15.0


def requested_ranks(argv):
    """The --gpus value of an argument list (1 when absent or malformed)."""
    for i, a in enumerate(argv):
        if a == "--gpus" and i + 1 < len(argv):
            v = argv[i + 1]
        elif a.startswith("--gpus="):
            v = a.split("=", 1)[1]
        else:
            continue
        try:
            return max(1, int(v))
        except ValueError:
            return 1
    return 1


def needs_launch(argv, environ=None):
    """True when N > 1 ranks are asked for and no launcher has set the rank environment."""
    env = os.environ if environ is None else environ
    return requested_ranks(argv) > 1 and "WORLD_SIZE" not in env


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _stop(procs, sig):
    for p in procs:
        if p.poll() is None:
            try:
                p.send_signal(sig)
            except ProcessLookupError:
                pass


def _stop_all(procs, sig, grace_s, poll_s=0.1):
    """Send ``sig`` to the children still running, wait up to ``grace_s`` for them to exit, then
    SIGKILL the rest and reap them (a child that ignores or handles SIGTERM cannot outlive it)."""
    _stop(procs, sig)
    deadline = time.monotonic() + grace_s
    while any(p.poll() is None for p in procs) and time.monotonic() < deadline:
        time.sleep(poll_s)
    _stop(procs, signal.SIGKILL)
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            pass


def spawn(nprocs, script, argv, environ=None, poll_s=0.2, log=None, grace_s=None):
    """Run ``python -u script argv`` as ranks 0..nprocs-1 and wait for all of them.

    Returns 0 when every rank exits 0, else the first failing rank's status (128 + signal for a
    rank killed by a signal).  A SIGTERM / SIGINT to this process is forwarded to the ranks; the
    ones still running ``grace_s`` (default GRACE_S) later are killed, then this process exits
    with 128 + the signal."""
    grace_s = GRACE_S if grace_s is None else grace_s
    base = dict(os.environ if environ is None else environ)
    base.setdefault("MASTER_ADDR", "127.0.0.1")
    base["MASTER_PORT"] = str(free_port())
    log = log or (lambda msg: print(msg, file=sys.stderr, flush=True))
    procs = []
    for r in range(nprocs):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs),
                   LOCAL_WORLD_SIZE=str(nprocs), GROUP_RANK="0", NODE_RANK="0")
        procs.append(subprocess.Popen([sys.executable, "-u", script] + list(argv), env=env))
    log("launch: %d ranks (pids %s), rendezvous 127.0.0.1:%s"
        % (nprocs, " ".join(str(p.pid) for p in procs), base["MASTER_PORT"]))

    # a SIGTERM / SIGINT to the parent (an outer time limit) goes to the children first; any
    # still running after the grace period are killed before the parent exits
    def forward(signum, _frame):
        log("launch: signal %d; stopping the ranks" % signum)
        _stop_all(procs, signum, grace_s)
        raise SystemExit(128 + signum)
    old = {s: signal.signal(s, forward) for s in (signal.SIGTERM, signal.SIGINT)}
    first_bad, deadline = None, None
    try:
        while True:
            states = [p.poll() for p in procs]
            if first_bad is None:
                for r, st in enumerate(states):
                    if st not in (None, 0):
                        first_bad = (r, st)
                        log("launch: rank %d exited with %d; stopping the other ranks" % (r, st))
                        _stop(procs, signal.SIGTERM)
                        deadline = time.monotonic() + grace_s
                        break
            if all(st is not None for st in states):
                break
            if deadline is not None and time.monotonic() > deadline:
                _stop(procs, signal.SIGKILL)
                deadline = None
            time.sleep(poll_s)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    if first_bad is None:
        return 0
    st = first_bad[1]
    return 128 - st if st < 0 else st
