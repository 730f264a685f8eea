"""Request spans + per-stage timestamps, exported as JSON / Chrome trace; roctx ranges on GPU.

The reference wraps sync execution and async thread launch in
``self.tracer.span(name=trace_name or api_path)`` (``APIs/1.0/base-py/ai4e_service.py:158-178``)
via an OpenCensus tracer; mesh-level B3 spans go to App Insights
(``Cluster/monitoring/application-insights-istio-adapter/configuration.yaml``).  Here a ``Tracer``
offers the same ``span(name=...)`` context manager, propagates B3-style ids
(``x-b3-traceid``/``x-b3-spanid``) and records the task pipeline stages
(accept -> batch-form -> worker -> h2d -> compute -> complete, :class:`StageClock` over the native
task record).  When running on the GPU it
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


# ---------------------------------------------------------------------------- B3 propagation
B3_HEADERS = ("x-b3-traceid", "x-b3-spanid", "x-b3-parentspanid", "x-b3-sampled")


def b3_from_headers(headers) -> Dict[str, str]:
    """Incoming B3 context (the Istio mesh headers the reference's adapter reads,
    ``application-insights-istio-adapter/configuration.yaml``); a fresh trace when absent. The gateway
    is the next hop, so it opens a child span of the caller's span."""
    get = (lambda k: headers.get(k) or headers.get(k.upper()) or "") if headers is not None else (lambda k: "")
    trace_id = get("x-b3-traceid") or _hexid(128)
    parent = get("x-b3-spanid")
    return {"x-b3-traceid": trace_id, "x-b3-spanid": _hexid(64), "x-b3-parentspanid": parent,
            "x-b3-sampled": get("x-b3-sampled") or "1"}


def b3_pack(ctx: Dict[str, str]) -> str:
    """Compact form stored in the native task record: traceid/spanid/parentspanid."""
    return f"{ctx['x-b3-traceid']}/{ctx['x-b3-spanid']}/{ctx.get('x-b3-parentspanid', '')}"


def b3_unpack(s: str) -> Dict[str, str]:
    parts = (s or "").split("/")
    parts += [""] * (3 - len(parts))
    return {"x-b3-traceid": parts[0], "x-b3-spanid": parts[1], "x-b3-parentspanid": parts[2]}


# ---------------------------------------------------------------------------- per-task stages
class StageClock:
    """Per-task stage timestamps (CLOCK_MONOTONIC) of the hot path.

    The native store keeps accept (``t_created``), dispatch (``t_running``) and finish times per task;
    the GPU worker reports, per batch, when it received and launched the batch, when the GPU results
    were ready and the GPU-side H2D / compute durations (``TaskStore.trace``). ``from_trace`` turns one
    such record into the stage sequence accept -> enqueue(d) -> batch_form -> h2d -> compute -> d2h ->
    complete, which ``GET /v1/taskmanagement/task/{id}/trace`` returns.
    """

    STAGES = ("accept", "batch_form", "worker_recv", "launch", "h2d_done", "gpu_done", "complete")

    def __init__(self):
        self.t: Dict[str, float] = {}

    def mark(self, stage: str, t: Optional[float] = None) -> None:
        self.t[stage] = time.monotonic() if t is None else t

    @classmethod
    def from_trace(cls, tr: dict) -> "StageClock":
        c = cls()
        if tr.get("t_created"):
            c.mark("accept", tr["t_created"])
        if tr.get("t_running"):
            c.mark("batch_form", tr["t_running"])
        if tr.get("t_worker_recv"):
            c.mark("worker_recv", tr["t_worker_recv"])
        if tr.get("t_worker_launch"):
            c.mark("launch", tr["t_worker_launch"])
            if tr.get("gpu_h2d_ms"):
                c.mark("h2d_done", tr["t_worker_launch"] + tr["gpu_h2d_ms"] / 1e3)
        if tr.get("t_worker_done"):
            c.mark("gpu_done", tr["t_worker_done"])
        if tr.get("t_finished"):
            c.mark("complete", tr["t_finished"])
        return c

    def durations_ms(self) -> Dict[str, float]:
        out = {}
        prev = None
        for s in self.STAGES:
            if s in self.t:
                if prev is not None:
                    out[f"{prev}->{s}"] = round((self.t[s] - self.t[prev]) * 1e3, 4)
                prev = s
        return out

    def to_dict(self) -> dict:
        base = min(self.t.values()) if self.t else 0.0
        return {"stages_ms_from_accept": {k: round((v - base) * 1e3, 4) for k, v in self.t.items()},
                "durations_ms": self.durations_ms()}
