"""Pipeline-stage tracing and profiling.

The reference has no tracer: its observability is ``explain`` (``PlanAnalyzer.scala:46-130``),
which this framework keeps unchanged in ``plananalysis``.  On MI355X the executor and the index
build additionally mark every pipeline stage two ways:

* **roctx ranges** (``csrc/runtime/hs_trace.cpp``) so ``rocprofv3 --marker-trace --kernel-trace``
  nests each kernel under the stage that launched it (decode+H2D, hash, all-to-all, sort, gather,
  D2H+encode, span search, probe, final reduction).  Enabled by
  ``spark.hyperspace.mi.trace.roctx.enabled`` or ``HS_ROCTX=1``.
* **stage timers** (``spark.hyperspace.mi.profile.enabled`` or ``HS_PROFILE=1``): host wall time
  plus device time from a pair of HIP events on the current stream.  ``report()`` folds them into
  per-stage totals; ``Hyperspace.profile()`` returns that table.

Both are off by default and cost one attribute check per stage when off.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
import threading
import time
from collections import OrderedDict
from typing import Dict, List, Optional

ROCTX_ENABLED = "spark.hyperspace.mi.trace.roctx.enabled"
PROFILE_ENABLED = "spark.hyperspace.mi.profile.enabled"


class _Record:
    __slots__ = ("name", "host_s", "ev0", "ev1")

    def __init__(self, name, host_s, ev0, ev1):
        self.name, self.host_s, self.ev0, self.ev1 = name, host_s, ev0, ev1


class Tracer:
    """Process-wide stage tracer.  Thread-safe: staging/IO threads may record stages too."""

    def __init__(self):
        self.roctx = False
        self.profile = False
        self._lib = None
        self._lock = threading.Lock()
        self._records: List[_Record] = []
        self._depth = threading.local()

    # -- configuration -----------------------------------------------------------------------
    def _native(self):
        if self._lib is None:
            from ..exec.jit import runtime
            L = runtime()
            L.hs_trace_enable.restype = C.c_int
            L.hs_trace_enable.argtypes = [C.c_int]
            L.hs_trace_push.restype = C.c_int
            L.hs_trace_push.argtypes = [C.c_char_p]
            L.hs_trace_pop.restype = C.c_int
            L.hs_trace_pop.argtypes = []
            L.hs_trace_mark.restype = None
            L.hs_trace_mark.argtypes = [C.c_char_p]
            L.hs_trace_depth.restype = C.c_int64
            L.hs_trace_depth.argtypes = []
            self._lib = L
        return self._lib

    def set_roctx(self, on: bool) -> bool:
        """Turns roctx markers on/off; returns whether a roctx library was found."""
        found = bool(self._native().hs_trace_enable(1 if on else 0))
        self.roctx = bool(on) and found
        return found

    def set_profile(self, on: bool) -> None:
        self.profile = bool(on)

    def configure(self, conf) -> None:
        from .conf import _b
        roctx = _b(conf.get(ROCTX_ENABLED, "false")) or os.environ.get("HS_ROCTX") == "1"
        prof = _b(conf.get(PROFILE_ENABLED, "false")) or os.environ.get("HS_PROFILE") == "1"
        if roctx != self.roctx:
            try:
                self.set_roctx(roctx)
            except (OSError, RuntimeError):
                self.roctx = False
        self.profile = prof

    # -- recording ---------------------------------------------------------------------------
    @contextlib.contextmanager
    def stage(self, name: str, device: bool = True):
        if not (self.roctx or self.profile):
            yield
            return
        if self.roctx:
            self._lib.hs_trace_push(name.encode())
        ev0 = ev1 = None
        if self.profile and device:
            ev0 = _event()
        t0 = time.perf_counter()
        try:
            yield
        finally:
            host = time.perf_counter() - t0
            if ev0 is not None:
                ev1 = _event()
            if self.roctx:
                self._lib.hs_trace_pop()
            if self.profile:
                with self._lock:
                    self._records.append(_Record(name, host, ev0, ev1))

    def mark(self, name: str) -> None:
        if self.roctx:
            self._lib.hs_trace_mark(name.encode())

    def open_ranges(self) -> int:
        return int(self._native().hs_trace_depth()) if self._lib is not None else 0

    # -- reporting ---------------------------------------------------------------------------
    def report(self, reset: bool = True) -> "OrderedDict[str, Dict[str, float]]":
        """Per-stage totals: ``{stage: {calls, host_ms, device_ms}}`` in first-seen order.
        ``device_ms`` is the HIP-event time on the stream that was current at stage entry."""
        with self._lock:
            recs = list(self._records)
            if reset:
                self._records.clear()
        if any(r.ev1 is not None for r in recs):
            import torch
            torch.cuda.synchronize()
        out: "OrderedDict[str, Dict[str, float]]" = OrderedDict()
        for r in recs:
            d = out.setdefault(r.name, {"calls": 0, "host_ms": 0.0, "device_ms": 0.0})
            d["calls"] += 1
            d["host_ms"] += r.host_s * 1e3
            if r.ev0 is not None and r.ev1 is not None:
                d["device_ms"] += r.ev0.elapsed_time(r.ev1)
        for d in out.values():
            d["host_ms"] = round(d["host_ms"], 4)
            d["device_ms"] = round(d["device_ms"], 4)
        return out

    def reset(self) -> None:
        with self._lock:
            self._records.clear()


def _event():
    try:
        import torch
        if not torch.cuda.is_available():
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e
    except Exception:  # noqa: BLE001 - profiling must never break a query
        return None


TRACER = Tracer()


_OFF = contextlib.nullcontext()


def stage(name: str, device: bool = True):
    """``with stage("join.probe"): ...`` — the module-level shortcut used by the executors
    (a shared no-op context while tracing is off: it sits on every query's host path)."""
    if not (TRACER.roctx or TRACER.profile):
        return _OFF
    return TRACER.stage(name, device)


def format_report(rep: Dict[str, Dict[str, float]]) -> str:
    lines = [f"{'stage':<28}{'calls':>7}{'host ms':>12}{'device ms':>12}"]
    for k, d in rep.items():
        lines.append(f"{k:<28}{d['calls']:>7}{d['host_ms']:>12.3f}{d['device_ms']:>12.3f}")
    return "\n".join(lines)


def active() -> Optional[Tracer]:
    return TRACER if (TRACER.roctx or TRACER.profile) else None
