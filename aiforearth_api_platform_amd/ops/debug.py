"""Breadcrumbs (``AI4E_BREADCRUMBS=1``): named progress counters that kernels inside a captured graph bump in
host-mapped memory (csrc/kernels/breadcrumbs.hip), readable from the host while the GPU runs. After a replay
stops (a fault or a hang), the counters before the stopping point are one ahead of those after it. Diagnostic
only: with the variable unset ``crumb`` is a no-op and nothing is launched."""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional

import torch

from . import _ext


class Breadcrumbs:
    def __init__(self, n: int = 64):
        host, dev = ctypes.c_void_p(), ctypes.c_void_p()
        _ext.call("ai4e_crumbs_alloc", n, ctypes.addressof(host), ctypes.addressof(dev))
        self.n, self.dev = n, dev.value
        self.arr = (ctypes.c_int * n).from_address(host.value)
        self.names: Dict[str, int] = {}

    def mark(self, name: str, device: torch.device) -> None:
        idx = self.names.setdefault(name, len(self.names))
        if idx >= self.n:
            raise ValueError("breadcrumbs: too many names")
        _ext.call("ai4e_crumb", self.dev, idx, _ext.stream_ptr(device))

    def read(self) -> Dict[str, int]:
        return {k: int(self.arr[i]) for k, i in self.names.items()}


_CRUMBS: Optional[Breadcrumbs] = None


def crumbs() -> Optional[Breadcrumbs]:
    global _CRUMBS
    if _CRUMBS is None and os.environ.get("AI4E_BREADCRUMBS", "0") == "1" and torch.cuda.is_available():
        _CRUMBS = Breadcrumbs()
    return _CRUMBS


def crumb(name: str, t: torch.Tensor) -> None:
    """Bump counter ``name`` on ``t``'s device, on the current stream (captured into a graph like any kernel)."""
    c = crumbs()
    if c is not None and t.is_cuda:
        c.mark(name, t.device)
