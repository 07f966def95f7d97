"""Attribution of a training step's GPU time without a profiler (tools/dist_step.py, bench.py
``train_step``): per-kernel-class HIP-event totals and the GFX clock sampled while it runs.

  KernelClassTimer   while active, every libgnnea entry point is bracketed by two HIP events on
                     the caller's current stream (the stream every gnnea launch goes to), and its
                     GPU time is summed by class: gemm (the MFMA projections / gradients),
                     aggregation (SpMM, HighWay, activation backward, slice packs), gat (the
                     attention passes and their column sums), loss (margin / L1), sinkhorn,
                     csr (graph construction).  What the step spends outside libgnnea -- torch
                     elementwise kernels, copies, collectives, idle gaps -- is the remainder.
  ClockSampler       a host thread reading the GFX clock (torch.cuda.clock_rate -> amdsmi) every
                     few milliseconds; median / min / max over the region.

Both are measurement aids: the timed steps of a run are taken without the event brackets (they
add host work per launch), the attributed steps after them.
"""
import threading
import time

import torch

from . import _lib

CLASSES = (
    ("gemm", ("gnnea_gemm",)),
    ("aggregation", ("gnnea_spmm", "gnnea_slice_pack", "gnnea_act_bwd", "gnnea_highway")),
    ("gat", ("gnnea_gat", "gnnea_colsum")),
    ("loss", ("gnnea_margin", "gnnea_l1")),
    ("sinkhorn", ("gnnea_sinkhorn",)),
    ("csr", ("gnnea_coo", "gnnea_csr", "gnnea_perm")),
)


def kernel_class(name):
    for cls, prefixes in CLASSES:
        if name.startswith(prefixes):
            return cls
    return "other_gnnea"


class KernelClassTimer:
    """``with KernelClassTimer() as t: step()`` then ``t.totals_ms()`` (synchronises)."""

    def __init__(self):
        self._pending = []
        self._orig = {}

    def __enter__(self):
        lib = _lib.lib()
        for name in _lib.SIGNATURES:
            if name.endswith(("_ws_bytes", "_version", "_string", "_path", "_pair_len")):
                continue  # host-only queries
            fn = getattr(lib, name)
            self._orig[name] = fn
            setattr(lib, name, self._wrap(name, fn))
        return self

    def __exit__(self, *exc):
        lib = _lib.lib()
        for name, fn in self._orig.items():
            setattr(lib, name, fn)
        self._orig = {}
        return False

    def _wrap(self, name, fn):
        cls = kernel_class(name)
        pending = self._pending

        def call(*args):
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            rc = fn(*args)
            b.record()
            pending.append((cls, a, b))
            return rc
        return call

    def totals_ms(self):
        torch.cuda.synchronize()
        out = {}
        for cls, a, b in self._pending:
            out[cls] = out.get(cls, 0.0) + a.elapsed_time(b)
        self._pending.clear()
        return out


class ClockSampler:
    """Samples the GFX clock (MHz) of ``device`` from a host thread while active."""

    def __init__(self, device, period_s=0.005):
        self.device, self.period = device, period_s
        self.samples = []
        self._stop = threading.Event()
        self._thread = None

    def _run(self):
        while not self._stop.is_set():
            try:
                self.samples.append(float(torch.cuda.clock_rate(self.device)))
            except Exception:  # no SMI on this host: report nothing rather than guess
                return
            time.sleep(self.period)

    def __enter__(self):
        self._thread = threading.Thread(target=self._run, daemon=True)
        self._thread.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        self._thread.join()
        return False

    def summary(self):
        if not self.samples:
            return None
        s = sorted(self.samples)
        return {"median_mhz": s[len(s) // 2], "min_mhz": s[0], "max_mhz": s[-1],
                "samples": len(s), "source": "torch.cuda.clock_rate (amdsmi GFX clock)"}
