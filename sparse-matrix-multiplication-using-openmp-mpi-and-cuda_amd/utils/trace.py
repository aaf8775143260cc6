"""Phase tracing: HIP-event timers + roctx ranges.

The reference computes chrono timers around symbolic / pack / H2D / kernel /
D2H phases and then comments every print out (sparse_matrix_mult.cu:160-274);
the report's Table 2 phase breakdown comes from that instrumentation.  Here:

* ``PhaseTimer.phase(name)`` records a HIP event pair on the current stream
  (device time, no synchronisation inside the phase) and a host wall-clock
  pair, and opens a roctx range so rocprofv3 traces (``--marker-trace``) show
  the phase;
* ``summary()`` synchronises once and returns per-phase totals (ms) — the
  structure behind the ``--metrics-json`` output of the CLIs.
"""
from __future__ import annotations

import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Dict, List, Optional, Tuple

import torch


def _roctx():
    try:
        from torch.cuda import nvtx  # roctx on ROCm builds

        return nvtx
    except Exception:  # pragma: no cover
        return None


class PhaseTimer:
    def __init__(self, device: Optional[torch.device] = None, enabled: bool = True):
        self.device = device if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.enabled = enabled
        self._events: List[Tuple[str, object, object]] = []
        self._host: Dict[str, float] = defaultdict(float)
        self._counts: Dict[str, int] = defaultdict(int)
        self._nvtx = _roctx() if self.device.type == "cuda" else None

    @contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        gpu = self.device.type == "cuda"
        if self._nvtx is not None:
            self._nvtx.range_push(name)
        if gpu:
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
        t0 = time.perf_counter()
        try:
            yield
        finally:
            if gpu:
                e.record()
                self._events.append((name, s, e))
            self._host[name] += time.perf_counter() - t0
            self._counts[name] += 1
            if self._nvtx is not None:
                self._nvtx.range_pop()

    def summary(self) -> Dict[str, Dict[str, float]]:
        dev_ms: Dict[str, float] = defaultdict(float)
        if self._events:
            torch.cuda.synchronize(self.device)
            for name, s, e in self._events:
                dev_ms[name] += s.elapsed_time(e)
        out = {}
        for name in self._host:
            out[name] = dict(host_ms=self._host[name] * 1e3, count=self._counts[name])
            if name in dev_ms:
                out[name]["device_ms"] = dev_ms[name]
        return out
