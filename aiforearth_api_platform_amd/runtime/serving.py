"""In-process GPU batch worker: dispatch queue -> dynamic batch -> engine -> task completion.

The single-GPU, single-process form of the serving path (the multi-GPU form is the native
:class:`NodeScheduler` behind :class:`runtime.worker_pool.WorkerPool`). It replaces the reference's
per-endpoint ``BackendQueueProcessor`` (``ProcessManager/BackendQueueProcessor/
BackendQueueProcessor.cs:27-81``) *plus* the model container's async thread
(``APIs/1.0/base-py/ai4e_service.py:180-213``): instead of one HTTP POST and one OS thread per
request, a worker pinned to one MI355X pulls up to ``max_batch`` peek-locked messages at once
(``receive(max_n, timeout, linger)`` — the dynamic batcher), marks them ``running`` in one store
call, runs them as one batch and attaches the result rows to the task records in one store call.

Failure handling: messages without a valid payload slot fail on their own (a task recovered after
a restart whose ring slot is gone must not poison the batch); a batch whose launch raises is
re-run item by item, so only items that fail alone are failed ("Task failed - try again"); the
loop itself never dies on an exception (the batch is failed and the loop goes on).
"""
from __future__ import annotations

import collections
import threading
import time
from typing import Deque, List, Optional, Sequence

import numpy as np

from ..store import STATE_FAILED, STATE_RUNNING
from ..utils.metrics import REGISTRY
from .servable import OutputField, encode_rows, format_result, row_bytes

INVALID_PAYLOAD = "Task failed - invalid payload"
TRY_AGAIN = "Task failed - try again"


def classifier_fields(topk: int) -> List[OutputField]:
    return [OutputField("classes", "int32", (topk,)), OutputField("probabilities", "float32", (topk,))]


class GpuBatchWorker:
    def __init__(self, control_plane, endpoint: str, engine, ring, max_batch: Optional[int] = None,
                 max_delay_s: Optional[float] = None, retry_delay_s: float = 1.0, poll_s: float = 0.05,
                 kind: str = "classifier", outputs: Optional[Sequence[OutputField]] = None, results=None):
        self.cp = control_plane
        self.endpoint = endpoint
        self.queue = control_plane.queue_for(endpoint)
        self.store = control_plane.store
        self.engine = engine
        self.ring = ring
        self.kind = kind
        self.outputs = list(outputs) if outputs is not None else classifier_fields(engine.topk)
        self.row_bytes = row_bytes(self.outputs)
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

    @property
    def describe(self) -> dict:
        return {"kind": self.kind, "outputs": [f.to_json() for f in self.outputs]}

    def result(self, task_id: str) -> Optional[dict]:
        return format_result(self.kind, self.describe["outputs"], self.store.result(task_id))

    def _notify(self, ids) -> None:
        if self.on_batch_done is not None and ids:
            self.on_batch_done(ids)

    def step(self, timeout_s: Optional[float] = None) -> int:
        """Receive at most one batch, launch it, finalize older batches. Returns #images launched."""
        t0 = time.perf_counter()
        if timeout_s is None:
            # never park in receive while a launched batch may be finishing: poll at 0.5 ms
            timeout_s = 0.0005 if self.pending else self.poll_s
        ids, refs, seqs = self.queue.receive_batch(self.max_batch, timeout_s, self.max_delay_s)
        t1 = time.perf_counter()
        self.phase_s["receive"] += t1 - t0
        n = len(ids)
        if n:
            nslots = self.ring.nslots
            bad = [i for i, r in enumerate(refs) if not 0 <= r < nslots]
            if bad:  # poison guard: no payload slot -> fail the item alone
                bad_ids = [ids[i] for i in bad]
                self.store.transition_many(bad_ids, STATE_FAILED, INVALID_PAYLOAD)
                self.queue.complete([seqs[i] for i in bad])
                keep = [i for i in range(n) if 0 <= refs[i] < nslots]
                ids, refs, seqs = [ids[i] for i in keep], [refs[i] for i in keep], [seqs[i] for i in keep]
                self._notify(bad_ids)
        if ids:
            self.store.transition_many(ids, STATE_RUNNING, STATE_RUNNING)
            t2 = time.perf_counter()
            self.phase_s["unpack+running"] += t2 - t1
            try:
                res = self.engine.submit(self.ring.buf, refs)
                self.phase_s["submit"] += time.perf_counter() - t2
                self.pending.append((ids, seqs, refs, res))
            except Exception as e:
                self.cp.log.log_error(f"batch launch failed, isolating items: {e}", self.endpoint)
                self.flush()
                self._isolate(ids, seqs, refs)
            self._h_batch.observe(len(ids))
        # keep one launched batch queued behind the running one while the next is being formed; retire
        # a batch as soon as its completion event fires. Never block on the GPU while there is only one
        # batch in flight: an empty receive must not turn into a synchronize, or the next batch (arriving
        # a moment later) is launched only after the GPU has drained and the H2D copy stalls it. At most
        # two batches stay pending, so the engine's third buffer set is never reused before its batch
        # was finalized (InferenceEngine nbuf = 3).
        while len(self.pending) > 2 or (self.pending and self.pending[0][3].done.query()):
            self._finalize(self.pending.popleft())
        return len(ids)

    def _isolate(self, ids: List[str], seqs: List[int], refs: List[int]) -> None:
        rows = np.zeros((len(ids), self.row_bytes), np.uint8)
        ok = np.ones(len(ids), np.uint8)
        for i, r in enumerate(refs):
            try:
                outs = self.engine.run_sync(self.ring.buf[r:r + 1])
                rows[i] = np.frombuffer(encode_rows([o.numpy() for o in outs], 1), np.uint8)
            except Exception:
                ok[i] = 0
        self.store.finish_batch(ids, rows.tobytes(), self.row_bytes, ok.tolist(), [], -1, "completed", TRY_AGAIN)
        self.queue.complete(seqs)
        self.ring.free(refs)
        self._notify(ids)

    def _finalize(self, item) -> None:
        ids, seqs, slots, res = item
        t0 = time.perf_counter()
        res.done.synchronize()
        t1 = time.perf_counter()
        self.phase_s["gpu_wait"] += t1 - t0
        self.ring.free(slots)
        h2d, comp = res.gpu_ms()
        rows = encode_rows([o.numpy() for o in res.outputs], len(ids))
        self.store.finish_batch(ids, rows, self.row_bytes, [], [0.0, res.t_launch, time.monotonic(), h2d, comp], -1,
                                "completed", TRY_AGAIN)
        self.queue.complete(seqs)
        self.batches += 1
        self.images += len(ids)
        self._c_images.inc(len(ids))
        self.phase_s["finalize"] += time.perf_counter() - t1
        self.finalize_times.append(t1)
        self._notify(ids)

    def flush(self) -> None:
        while self.pending:
            self._finalize(self.pending.popleft())

    def _fail_pending(self, err: Exception) -> None:
        items, self.pending = list(self.pending), collections.deque()
        for ids, seqs, slots, _ in items:
            self.store.transition_many(ids, STATE_FAILED, TRY_AGAIN)
            self.queue.complete(seqs)
            self.ring.free(slots)
            self._notify(ids)
        self.cp.log.log_error(f"gpu worker step failed: {err}", self.endpoint)

    def _loop(self) -> None:
        while not self._stop.is_set():
            try:
                self.step()
            except Exception as e:  # the worker thread must never die with tasks left 'running'
                self._fail_pending(e)
                time.sleep(0.01)
        try:
            self.flush()
        except Exception as e:
            self._fail_pending(e)

    def start(self) -> "GpuBatchWorker":
        self._thread = threading.Thread(target=self._loop, daemon=True, name=f"ai4e-gpu-worker{self.endpoint}")
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(10)
