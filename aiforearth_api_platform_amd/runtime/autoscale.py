"""Queue-depth autoscaler for a worker pool — the HPA analogue.

The reference scales model pods with a HorizontalPodAutoscaler on CPU plus the App-Insights custom
metric ``CURRENT_REQUESTS/<cluster><path>`` (``APIs/Charts/templates/async-gpu/autoscaler.yaml:1-21``:
``minReplicas 1``, ``maxReplicas 10``, Pods metric ``targetAverageValue 1``;
``APIs/Charts/templates/appinsights-metric.yaml:1-7``), fed every 30 s by the queue-length timer
(``TaskProcessLogger/TaskQueueLogger.cs:19-27``). Here the replicas are GPU worker processes and the
metric is read directly from the native scheduler: requests waiting in the endpoint's queue plus
batches in flight, in units of full batches.

Policy (the HPA v2 algorithm): ``desired = ceil(load / target_per_worker)`` clamped to
``[min_workers, max_workers]``; scale-up applies at once, scale-down only after the lower value held
for ``down_stabilization`` consecutive periods (HPA's stabilization window), so bursty arrival does
not churn processes (a worker restart costs graph capture).
"""
from __future__ import annotations

import math
import threading
import time
from typing import List, Optional, Tuple

from ..utils.metrics import REGISTRY


class QueueDepthAutoscaler:
    def __init__(self, pool, min_workers: int = 1, max_workers: Optional[int] = None, target_per_worker: float = 2.0,
                 period_s: float = 5.0, down_stabilization: int = 3, clock=time.monotonic):
        self.pool = pool
        self.min = max(0, int(min_workers))
        self.max = int(max_workers or len(pool.devices))
        self.target = float(target_per_worker)
        self.period = float(period_s)
        self.down_need = max(1, int(down_stabilization))
        self.clock = clock
        self._below = 0
        self.decisions: List[Tuple[float, float, int, int]] = []  # (t, load, current, desired)
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._g_desired = REGISTRY.gauge(f"autoscale_desired_workers{getattr(pool, 'endpoint', '')}")
        self._g_load = REGISTRY.gauge(f"autoscale_load_batches{getattr(pool, 'endpoint', '')}")

    def load(self) -> float:
        """Pending work in full batches: queued requests + batches running on the GPUs."""
        q = self.pool.queue.stats()
        mb = max(1, int(self.pool.spec.max_batch))
        queued = (q["ready"] + q["scheduled"]) / mb
        inflight = sum(int(w.stats.get("outstanding", 0)) for w in self.pool.workers if not w.stop.is_set())
        return queued + inflight

    def desired(self, load: float, current: int) -> int:
        want = int(math.ceil(load / self.target)) if self.target > 0 else current
        want = max(self.min, min(self.max, want))
        if want >= current:
            self._below = 0
            return want
        self._below += 1
        if self._below >= self.down_need:
            self._below = 0
            return want
        return current

    def step(self) -> int:
        if hasattr(self.pool, "refresh"):
            self.pool.refresh()
        cur = self.pool.active()
        load = self.load()
        want = self.desired(load, cur)
        self.decisions.append((self.clock(), load, cur, want))
        self._g_desired.set(want)
        self._g_load.set(load)
        if want != cur:
            self.pool.resize(want)
        return want

    def _loop(self) -> None:
        while not self._stop.wait(self.period):
            try:
                self.step()
            except Exception:  # pragma: no cover - never kill the serving process over scaling
                pass

    def start(self) -> "QueueDepthAutoscaler":
        self._thread = threading.Thread(target=self._loop, daemon=True, name="ai4e-autoscaler")
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(5)
