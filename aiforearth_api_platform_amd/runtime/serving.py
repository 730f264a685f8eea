"""GPU batch worker: dispatch queue -> dynamic batch -> engine -> task completion.

This is the in-process replacement for the reference's per-endpoint ``BackendQueueProcessor``
(``ProcessManager/BackendQueueProcessor/BackendQueueProcessor.cs:27-81``) *plus* the model
container's async thread (``APIs/1.0/base-py/ai4e_service.py:180-213``): instead of one HTTP POST
and one OS thread per request, a worker pinned to one MI355X pulls up to ``max_batch`` peek-locked
messages at once (``receive(max_n, timeout, linger)`` — the dynamic batcher, max batch / max
delay), marks them ``running`` in one store call, runs them as one batch, and completes them in one
store call. A failed batch is abandoned with the retry delay (redelivery, bounded by the queue's
max delivery count; exhausted tasks are failed with a reason).
"""
from __future__ import annotations

import collections
import threading
import time
from typing import Deque, Dict, List, Optional, Tuple

import numpy as np

from ..store import STATE_COMPLETED, STATE_FAILED, STATE_RUNNING
from ..utils.metrics import REGISTRY


class ResultStore:
    """Task results kept as per-batch arrays (no per-task Python objects on the hot path)."""

    def __init__(self, max_tasks: int = 1_000_000):
        self._rows: Dict[str, Tuple[int, int]] = {}
        self._batches: Dict[int, Tuple[np.ndarray, np.ndarray]] = {}
        self._order: Deque[Tuple[int, List[str]]] = collections.deque()
        self._n = 0
        self._bid = 0
        self._max = max_tasks
        self._mu = threading.Lock()

    def put_batch(self, ids: List[str], top_idx: np.ndarray, top_prob: np.ndarray) -> None:
        with self._mu:
            bid = self._bid
            self._bid += 1
            self._batches[bid] = (top_idx, top_prob)
            for r, tid in enumerate(ids):
                self._rows[tid] = (bid, r)
            self._order.append((bid, ids))
            self._n += len(ids)
            while self._n > self._max and self._order:
                old, oids = self._order.popleft()
                self._batches.pop(old, None)
                for t in oids:
                    self._rows.pop(t, None)
                self._n -= len(oids)

    def get(self, task_id: str) -> Optional[dict]:
        with self._mu:
            loc = self._rows.get(task_id)
            if loc is None:
                return None
            idx, prob = self._batches[loc[0]]
            r = loc[1]
            return {"classes": idx[r].tolist(), "probabilities": [float(x) for x in prob[r]]}


class GpuBatchWorker:
    def __init__(self, control_plane, endpoint: str, engine, ring, results: Optional[ResultStore] = None,
                 max_batch: Optional[int] = None, max_delay_s: Optional[float] = None, retry_delay_s: float = 0.0,
                 poll_s: float = 0.05):
        self.cp = control_plane
        self.endpoint = endpoint
        self.queue = control_plane.queue_for(endpoint)
        self.store = control_plane.store
        self.engine = engine
        self.ring = ring
        self.results = results if results is not None else ResultStore()
        self.max_batch = max_batch or engine.max_batch
        self.max_delay_s = (control_plane.cfg.max_batch_delay_ms / 1e3) if max_delay_s is None else max_delay_s
        self.retry_delay_s = retry_delay_s
        self.poll_s = poll_s
        self.pending: Deque = collections.deque()
        self.batches = 0
        self.images = 0
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.phase_s = collections.defaultdict(float)  # host time per worker phase (diagnostics)
        self.finalize_times: Deque[float] = collections.deque(maxlen=4096)
        self.on_batch_done = None  # optional callback(ids) after a batch is completed or failed
        self._h_batch = REGISTRY.histogram(f"batch_size{endpoint}", buckets=(1, 8, 32, 64, 128, 256, 512, 1024))
        self._c_images = REGISTRY.counter(f"images_total{endpoint}")

    def step(self, timeout_s: Optional[float] = None) -> int:
        """Receive at most one batch, launch it, finalize older batches. Returns #images launched."""
        t0 = time.perf_counter()
        if timeout_s is None:
            # never park in receive while a launched batch may be finishing: poll at 0.5 ms
            timeout_s = 0.0005 if self.pending else self.poll_s
        msgs = self.queue.receive(self.max_batch, timeout_s, self.max_delay_s)
        n = len(msgs)
        t1 = time.perf_counter()
        self.phase_s["receive"] += t1 - t0
        if n:
            ids = [m.task_id for m in msgs]
            slots = [m.ref for m in msgs]
            seqs = [m.seq for m in msgs]
            self.store.transition_many(ids, STATE_RUNNING, STATE_RUNNING)
            t2 = time.perf_counter()
            self.phase_s["unpack+running"] += t2 - t1
            try:
                res = self.engine.submit(self.ring.buf, slots)
                self.phase_s["submit"] += time.perf_counter() - t2
            except Exception as e:  # launch failure -> redeliver the whole batch
                self.cp.log.log_error(f"batch launch failed: {e}", self.endpoint)
                for s in seqs:
                    if self.queue.abandon(s, self.retry_delay_s) == "deadlettered":
                        pass
                self._fail_deadletters()
                return 0
            self.pending.append((ids, seqs, slots, res))
            self._h_batch.observe(n)
        # keep one launched batch queued behind the running one while the next is being formed; retire
        # a batch as soon as its completion event fires. Never block on the GPU while there is only one
        # batch in flight: an empty receive must not turn into a synchronize, or the next batch (arriving
        # a moment later) is launched only after the GPU has drained and the H2D copy stalls it. At most
        # two batches stay pending, so the engine's third buffer set is never reused before its batch
        # was finalized (InferenceEngine nbuf = 3).
        while len(self.pending) > 2 or (self.pending and self.pending[0][3].done.query()):
            self._finalize(self.pending.popleft())
        return n

    def _finalize(self, item) -> None:
        ids, seqs, slots, res = item
        t0 = time.perf_counter()
        res.done.synchronize()
        t1 = time.perf_counter()
        self.phase_s["gpu_wait"] += t1 - t0
        self.ring.free(slots)
        self.results.put_batch(ids, res.top_idx.numpy().copy(), res.top_prob.numpy().copy())
        self.store.transition_many(ids, STATE_COMPLETED, STATE_COMPLETED)
        self.queue.complete(seqs)
        self.batches += 1
        self.images += len(ids)
        self._c_images.inc(len(ids))
        self.phase_s["finalize"] += time.perf_counter() - t1
        self.finalize_times.append(t1)
        if self.on_batch_done is not None:
            self.on_batch_done(ids)

    def _fail_deadletters(self) -> None:
        dead = self.queue.take_deadletters()
        if dead:
            self.store.transition_many(dead, STATE_FAILED, "Task failed - maximum retries exceeded")
            if self.on_batch_done is not None:
                self.on_batch_done(dead)

    def flush(self) -> None:
        while self.pending:
            self._finalize(self.pending.popleft())

    def _loop(self) -> None:
        while not self._stop.is_set():
            self.step()
        self.flush()

    def start(self) -> "GpuBatchWorker":
        self._thread = threading.Thread(target=self._loop, daemon=True, name=f"ai4e-gpu-worker{self.endpoint}")
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(10)
