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
import time
import traceback
from typing import Any, Optional

from ..config import get_config
from .tracing import Tracer, get_tracer


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

    def _emit(self, level: str, msg: str, uri: str = "", task_id: str = "", **extra: Any) -> None:
        rec = {"ts": time.time(), "level": level, "message": msg, **self.fields, "uri": uri,
               "task_id": task_id, **extra}
        self.records.append(rec)
        if len(self.records) > self._keep:
            del self.records[: len(self.records) - self._keep]
        if logging.getLevelName(level) >= self.level and self.stream is not None:
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
