"""Request spans + per-stage timestamps, exported as JSON / Chrome trace; roctx ranges on GPU.

The reference wraps sync execution and async thread launch in
``self.tracer.span(name=trace_name or api_path)`` (``APIs/1.0/base-py/ai4e_service.py:158-178``)
via an OpenCensus tracer; mesh-level B3 spans go to App Insights
(``Cluster/monitoring/application-insights-istio-adapter/configuration.yaml``).  Here a ``Tracer``
offers the same ``span(name=...)`` context manager, propagates B3-style ids
(``x-b3-traceid``/``x-b3-spanid``) and records the task pipeline stages
(accept -> enqueue -> batch-form -> h2d -> compute -> d2h -> complete).  When running on the GPU it
also pushes ``roctx`` ranges so rocprofv3 kernel traces line up with request spans.
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
import random
import threading
import time
from typing import Dict, List, Optional

_roctx = None


def _load_roctx():
    global _roctx
    if _roctx is None:
        _roctx = False
        for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePop.restype = ctypes.c_int
                _roctx = lib
                break
            except OSError:
                continue
    return _roctx or None


def _hexid(bits: int) -> str:
    return f"{random.getrandbits(bits):0{bits // 4}x}"


class Span:
    __slots__ = ("name", "trace_id", "span_id", "parent_id", "start", "end", "attrs", "tid")

    def __init__(self, name: str, trace_id: str, parent_id: Optional[str], attrs: Optional[dict] = None):
        self.name = name
        self.trace_id = trace_id
        self.span_id = _hexid(64)
        self.parent_id = parent_id
        self.start = time.time()
        self.end: Optional[float] = None
        self.attrs = dict(attrs or {})
        self.tid = threading.get_ident()

    def add_attribute(self, k, v) -> None:
        self.attrs[k] = v

    def to_dict(self) -> dict:
        return {"name": self.name, "trace_id": self.trace_id, "span_id": self.span_id,
                "parent_id": self.parent_id, "start": self.start, "end": self.end,
                "duration_ms": None if self.end is None else (self.end - self.start) * 1e3, "attrs": self.attrs}


class Tracer:
    def __init__(self, max_spans: int = 100000, roctx: Optional[bool] = None):
        self.spans: List[Span] = []
        self._max = max_spans
        self._local = threading.local()
        self._mu = threading.Lock()
        self.use_roctx = (os.environ.get("AI4E_ROCTX", "0") == "1") if roctx is None else roctx

    def _stack(self) -> list:
        st = getattr(self._local, "stack", None)
        if st is None:
            st = self._local.stack = []
        return st

    @contextlib.contextmanager
    def span(self, name: str, trace_id: Optional[str] = None, **attrs):
        st = self._stack()
        parent = st[-1] if st else None
        tid = trace_id or (parent.trace_id if parent else _hexid(128))
        sp = Span(name, tid, parent.span_id if parent else None, attrs)
        st.append(sp)
        rx = _load_roctx() if self.use_roctx else None
        if rx:
            rx.roctxRangePushA(name.encode())
        try:
            yield sp
        finally:
            if rx:
                rx.roctxRangePop()
            sp.end = time.time()
            st.pop()
            with self._mu:
                self.spans.append(sp)
                if len(self.spans) > self._max:
                    del self.spans[: len(self.spans) - self._max]

    def current(self) -> Optional[Span]:
        st = self._stack()
        return st[-1] if st else None

    def export_json(self) -> List[dict]:
        with self._mu:
            return [s.to_dict() for s in self.spans]

    def export_chrome_trace(self, path: str) -> None:
        with self._mu:
            events = [{"name": s.name, "ph": "X", "ts": s.start * 1e6,
                       "dur": ((s.end or s.start) - s.start) * 1e6, "pid": os.getpid(), "tid": s.tid % 100000,
                       "args": {**s.attrs, "trace_id": s.trace_id}} for s in self.spans]
        with open(path, "w") as f:
            json.dump({"traceEvents": events}, f)

    def clear(self) -> None:
        with self._mu:
            self.spans.clear()


_TRACER: Optional[Tracer] = None


def get_tracer() -> Tracer:
    global _TRACER
    if _TRACER is None:
        _TRACER = Tracer()
    return _TRACER


class StageClock:
    """Per-task stage timestamps (monotonic) — the new framework's hot-path trace record."""

    STAGES = ("accept", "enqueue", "batch_form", "h2d", "compute", "d2h", "complete")

    def __init__(self):
        self.t: Dict[str, float] = {}

    def mark(self, stage: str, t: Optional[float] = None) -> None:
        self.t[stage] = time.monotonic() if t is None else t

    def durations_ms(self) -> Dict[str, float]:
        out = {}
        prev = None
        for s in self.STAGES:
            if s in self.t:
                if prev is not None:
                    out[f"{prev}->{s}"] = (self.t[s] - self.t[prev]) * 1e3
                prev = s
        return out
