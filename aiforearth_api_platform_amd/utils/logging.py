"""Structured JSON logging with the reference's telemetry fields.

Every line carries ``service_owner, service_name, service_version, service_cluster, uri, task_id``
like ``ProcessManager/Libraries/AppInsightsLogger.cs:43-95``; ``log_exception(exc, taskId)`` and
``tracer`` match what ``APIs/1.0/base-py/ai4e_service.py:53-54,189-195`` expects from the external
``AI4EAppInsights`` logger, so user code written against the reference keeps working.
"""
from __future__ import annotations

import json
import logging
import sys
import threading
import time
import traceback
import zlib
from typing import Any, Optional

from ..config import get_config
from .tracing import Tracer, get_tracer


class TelemetrySampler:
    """Adaptive sampling of telemetry items, as Application Insights does for the reference's Function apps
    (``samplingSettings: {isEnabled, maxTelemetryItemsPerSecond: 50}``, ``ProcessManager/CacheManager/host.json:3-9``)
    and its Istio adapter (adaptive sampling limit, ``application-insights-istio-mixer-adapter-deployment.yaml:36``):

    * the sampling ratio is re-estimated every ``interval_s`` from the offered rate of the previous interval,
      ``ratio = min(1, max_per_s / offered_per_s)``, so the emitted rate tracks ``max_per_s`` at any load;
    * items of one task are kept or dropped together (the decision hashes the task id against the ratio, App
      Insights' per-operation sampling), so a kept task's log lines stay complete; items without a task id are
      sampled by a deterministic counter;
    * within an interval at most twice the interval's budget of SAMPLED items is kept (a sudden burst is cut before
      the next re-estimate; the one place a task can lose some of its lines);
    * ERROR items are always kept (rare, and the ones an operator needs; a deviation from App Insights, which would
      sample exceptions too): they count toward the offered rate but not toward the burst cap, so an error burst does
      not starve the INFO / WARN lines of the same tasks;
    * sampling applies to the EXPORTED stream only (the telemetry sink, here the JSON lines on the stream); the
      service's own recent-records ring (``AI4ELogger.records``, /v1/platform/logs) stays complete, as App Insights
      sampling never touches the application's local view;
    * every emitted item carries ``sample_rate`` = 1 / ratio (App Insights' itemCount) so counts can be re-weighted.
    """

    def __init__(self, max_per_s: float = 50.0, interval_s: float = 1.0, clock=time.monotonic):
        self.max_per_s, self.interval_s, self.clock = float(max_per_s), float(interval_s), clock
        self.ratio = 1.0
        self.seen = self.kept = 0
        self._t0 = clock()
        self._n = 0          # items offered in the current interval
        self._k = 0          # items kept in the current interval
        self._untagged = 0.0
        self._mu = threading.Lock()

    def _roll(self, now: float) -> None:
        dt = now - self._t0
        if dt < self.interval_s:
            return
        offered = self._n / dt
        self.ratio = 1.0 if offered <= self.max_per_s else self.max_per_s / offered
        self._t0, self._n, self._k = now, 0, 0

    def keep(self, task_id: str = "", always: bool = False) -> bool:
        if self.max_per_s <= 0:
            return True
        with self._mu:
            self._roll(self.clock())
            self._n += 1
            self.seen += 1
            if always:
                self.kept += 1
                return True
            if self._k >= 2.0 * self.max_per_s * self.interval_s:
                ok = False
            elif self.ratio >= 1.0:
                ok = True
            elif task_id:
                ok = (zlib.crc32(task_id.encode()) & 0xFFFFFFFF) < self.ratio * 4294967296.0
            else:
                self._untagged += self.ratio
                ok = self._untagged >= 1.0
                if ok:
                    self._untagged -= 1.0
            self.kept += ok
            self._k += ok
            return ok


class AI4ELogger:
    """Drop-in for the reference container logger (``AI4EAppInsights``/``AzureMonitorLogger``)."""

    def __init__(self, service_name: Optional[str] = None, service_version: Optional[str] = None,
                 service_cluster: Optional[str] = None, stream=None, level: int = logging.INFO,
                 tracer: Optional[Tracer] = None):
        cfg = get_config()
        self.fields = {
            "service_owner": cfg.service_owner,
            "service_name": service_name or cfg.service_name,
            "service_version": service_version or cfg.service_version,
            "service_cluster": service_cluster or cfg.service_cluster,
        }
        self.level = level
        self.stream = stream if stream is not None else sys.stderr
        self.tracer = tracer if tracer is not None else get_tracer()
        self.records = []  # last N records kept for /v1/platform/logs and tests
        self._keep = 1000
        self.sampler = TelemetrySampler(getattr(cfg, "telemetry_max_per_s", 50.0))

    def _emit(self, level: str, msg: str, uri: str = "", task_id: str = "", **extra: Any) -> None:
        rec = {"ts": time.time(), "level": level, "message": msg, **self.fields, "uri": uri,
               "task_id": task_id, **extra}
        self.records.append(rec)  # the local view is complete: sampling is an export decision
        if len(self.records) > self._keep:
            del self.records[: len(self.records) - self._keep]
        if logging.getLevelName(level) < self.level or self.stream is None:
            return
        if not self.sampler.keep(task_id, always=level in ("ERROR", "CRITICAL")):
            return
        if self.sampler.ratio < 1.0:
            rec = dict(rec, sample_rate=round(1.0 / self.sampler.ratio, 3))
        self.stream.write(json.dumps(rec, default=str) + "\n")

    def log_debug(self, msg: str, uri: str = "", task_id: str = "", **kw) -> None:
        self._emit("DEBUG", msg, uri, task_id, **kw)

    def log_info(self, msg: str, uri: str = "", task_id: str = "", **kw) -> None:
        self._emit("INFO", msg, uri, task_id, **kw)

    LogInformation = log_info

    def log_warn(self, msg: str, uri: str = "", task_id: str = "", **kw) -> None:
        self._emit("WARNING", msg, uri, task_id, **kw)

    LogWarning = log_warn

    def log_error(self, msg: str, uri: str = "", task_id: str = "", **kw) -> None:
        self._emit("ERROR", msg, uri, task_id, **kw)

    def LogError(self, exc: BaseException, uri: str = "", task_id: str = "") -> None:
        self._emit("ERROR", f"{type(exc).__name__}: {exc}", uri, task_id)

    def log_exception(self, exc: Any = None, taskId: str = "", uri: str = "") -> None:
        et, ev, tb = sys.exc_info()
        desc = str(exc if exc is not None else et)
        self._emit("ERROR", desc, uri, taskId or "",
                   traceback="".join(traceback.format_exception(et, ev, tb)) if et else "")

    def LogMetric(self, name: str, value: float, uri: str = "") -> None:
        from .metrics import REGISTRY

        REGISTRY.gauge(name).set(value)
        self._emit("DEBUG", f"metric {name}={value}", uri, metric=name, value=value)


_DEFAULT: Optional[AI4ELogger] = None


def get_logger() -> AI4ELogger:
    global _DEFAULT
    if _DEFAULT is None:
        _DEFAULT = AI4ELogger(level=logging.WARNING)
    return _DEFAULT
