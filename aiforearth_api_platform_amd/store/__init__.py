"""Task store + dispatch queue (the reference's Redis cache + Service Bus queue, in-process).

``TaskStore`` / ``DispatchQueue`` resolve to the native C++ core (``csrc/core/ai4e_core.cpp``)
unless ``AI4E_STORE_BACKEND=python`` selects the pure-Python reference implementation.
"""
from __future__ import annotations

import os

from . import pystore
from .schema import (BACKEND_STATES, STATE_COMPLETED, STATE_CREATED, STATE_FAILED, STATE_RUNNING,
                     APITask, queue_name_for_endpoint)

try:
    from .. import _ai4e_core as native  # type: ignore
except ImportError:  # not built yet
    native = None


def backend_module(name: str | None = None):
    name = (name or os.environ.get("AI4E_STORE_BACKEND", "native")).lower()
    if name == "python":
        return pystore
    if native is None:
        raise ImportError("native core _ai4e_core is not built: run `python -m aiforearth_api_platform_amd._build` "
                          "or set AI4E_STORE_BACKEND=python")
    return native


def make_store(journal_path: str = "", backend: str | None = None):
    return backend_module(backend).TaskStore(journal_path)


def make_queue(name: str, max_delivery_count: int = 1440, lock_duration_s: float = 300.0, max_size: int = 0,
               backend: str | None = None):
    return backend_module(backend).DispatchQueue(name, max_delivery_count, lock_duration_s, max_size)


__all__ = ["APITask", "BACKEND_STATES", "STATE_CREATED", "STATE_RUNNING", "STATE_COMPLETED", "STATE_FAILED",
           "queue_name_for_endpoint", "make_store", "make_queue", "backend_module", "native", "pystore"]
