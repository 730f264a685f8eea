"""A GPU model exposed as an API endpoint: payload decode -> payload-ring slot -> task -> batch worker.

This is the "drop-in model" container of the reference (``APIs/Charts/templates/async-gpu``,
``APIs/1.0/base-py/ai4e_service.py``) collapsed into the node process: request bodies are decoded
once on the CPU straight into a slot of the payload ring, the task record is created in the native
store and the slot index travels through the dispatch queue, so the GPU worker's H2D copy reads the
request bytes exactly where the front end put them. The backend is either the per-GPU
:class:`WorkerPool` (native scheduler, one process per GPU) or an in-process
:class:`GpuBatchWorker` (single GPU / CPU tests).

Durability (survey §5.4, the reference's ``{TaskId}_ORIG`` replay, ``CacheConnectorUpsert.cs:150-176``):
with a journal configured, request bodies up to ``journal_payload_max_bytes`` are journaled as the
task's ``_ORIG`` body, and :meth:`replay` re-ingests them after a restart; tasks whose payload was
not journaled are failed with a reason instead of being requeued without a payload.
"""
from __future__ import annotations

import base64
import json
import threading
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..store import STATE_CREATED, STATE_FAILED
from .decode import PayloadError, decode_image  # noqa: F401  (re-exported: the endpoint's payload API)
from .ingest import StreamedBatch
from .jpeg_gpu import JPEG_TYPES, prepare_into_slot
from .serving import GpuBatchWorker

PAYLOAD_LOST = "Task failed - payload lost on restart"
PUBLISH_FAILED = "Failed - unable to send to backend service."
_ORIG_PREFIX = "ai4e-b64:"


class ModelEndpoint:
    def __init__(self, control_plane, path: str, engine=None, ring=None, worker=None,
                 decode: Optional[Callable[[bytes, str], np.ndarray]] = None, base_url: str = "http://127.0.0.1",
                 journal_payload_max_bytes: Optional[int] = None, decode_processes: int = 0):
        self.cp = control_plane
        self.path = path
        self.endpoint = base_url.rstrip("/") + path
        self.worker = worker if worker is not None else GpuBatchWorker(control_plane, self.endpoint, engine, ring)
        self.ring = self.worker.ring
        self.is_pool = hasattr(self.worker, "submit_slots")
        self.decode = decode or (lambda body, ct: decode_image(body, ct, self.ring.item_shape))
        self.custom_decode = decode is not None  # (not an image endpoint: the ingest front-ends leave it alone)
        # decode worker processes writing into the shared ring (pool backends: the ring is shared memory)
        self.decode_pool = None
        if decode_processes > 0 and decode is None and hasattr(self.ring, "name"):
            from .decode_pool import DecodePool

            self.decode_pool = DecodePool(decode_processes, self.ring.name, self.ring.nslots, self.ring.item_shape)
        self.queue = control_plane.queue_for(self.endpoint)
        self._waiters: Dict[str, Callable[[str], None]] = {}
        self._wmu = threading.Lock()
        if not self.is_pool:
            self.worker.on_batch_done = self._on_done
        cap = getattr(control_plane.cfg, "journal_payload_max_bytes", 0) if journal_payload_max_bytes is None \
            else journal_payload_max_bytes
        self.journal_cap = int(cap) if control_plane.cfg.journal_path else 0
        control_plane.register_replayer(self.endpoint, self.replay)

    @property
    def paths(self) -> List[str]:
        """Endpoint paths whose tasks this endpoint owns: its own + later ensemble stages."""
        from ..store.pystore import absolute_path

        stages = getattr(getattr(self.worker, "spec", None), "stage_endpoints", ()) or ()
        return [self.path] + [absolute_path(e) for e in stages]

    @property
    def item_shape(self) -> Tuple[int, ...]:
        return tuple(self.ring.item_shape)

    # ------------------------------------------------------------- ingest
    def _queue(self, slot: int):
        """The dispatch queue that serves a payload in ``slot`` (a GPU-sharded pool: the owning shard's)."""
        return self.worker.queue_for_slot(slot) if self.is_pool else self.queue

    def _send_existing(self, tid: str, slot: int) -> bool:
        """Queue an existing task record (through the pool's scheduler, so the shard's load counters see it)."""
        if self.is_pool and hasattr(self.worker, "send_existing"):
            return self.worker.send_existing(tid, slot)
        return self._queue(slot).send(tid, slot, "")

    def _enqueue(self, slots: List[int], trace: str = "") -> List[str]:
        if self.is_pool:
            return self.worker.submit_slots(slots, trace)
        ids = self.cp.store.create_many(self.endpoint, len(slots), trace=trace)
        sent = self.queue.send_many(ids, slots)
        if sent < len(ids):
            self.cp.store.transition_many(ids[sent:], STATE_FAILED, PUBLISH_FAILED)
            self.ring.free(slots[sent:])
        return ids

    def _write(self, slots: Sequence[int], images_u8: np.ndarray) -> None:
        if self.is_pool:  # SharedPayloadRing: one copy per contiguous run of slots
            self.ring.write(slots, images_u8)
            return
        src = torch.from_numpy(np.require(images_u8, np.uint8, ["C", "W"]))
        for i, s in enumerate(slots):
            self.ring.buf[s].copy_(src[i])

    def submit(self, body: bytes, content_type: str = "application/octet-stream", task_id: str = "",
               on_done: Optional[Callable[[str], None]] = None, trace: str = "") -> str:
        """Async API: decode, create task (or adopt an upstream ``taskId``), enqueue. Returns task JSON.

        Raises :class:`PayloadError` (-> HTTP 400/415) before any task exists for undecodable bodies."""
        ct = (content_type or "").split(";")[0].strip().lower()
        key = getattr(self.ring, "jpeg_key", 0) if self.is_pool and not self.custom_decode else 0
        if key and ct in JPEG_TYPES:
            # JPEG: prepared straight into the slot (headers + unstuffed scan, ~0.2 ms) for the worker to decode on its
            # GPU (runtime/jpeg_gpu.py); frames outside the GPU path's envelope are decoded here as before
            slot = self.ring.alloc(1, timeout=30)[0]
            try:
                item = int(np.prod(self.item_shape))
                if not prepare_into_slot(body, self.ring.buf[slot].data_ptr(), item, self.item_shape, key):
                    self._write([slot], self.decode(body, content_type)[None])
            except BaseException:
                self.ring.free([slot])
                raise
        elif self.decode_pool is not None and ct not in ("", "application/octet-stream"):
            slot = self.ring.alloc(1, timeout=30)[0]
            try:
                self.decode_pool.decode_into(slot, body, content_type)
            except BaseException:
                self.ring.free([slot])
                raise
        else:
            arr = self.decode(body, content_type)
            slot = self.ring.alloc(1, timeout=30)[0]
            self._write([slot], arr[None])
        orig = self._orig(body, content_type)
        if task_id or orig is not None:
            # upstream TaskId (header taskId, api_task.py:12-20) or a journaled payload: explicit upsert
            serialized, _ = self.cp.store.upsert(task_id, STATE_CREATED, STATE_CREATED, self.endpoint, orig, True)
            tid = json.loads(serialized)["TaskId"]
            if trace:
                self.cp.store.set_trace(tid, trace)
            if on_done is not None:
                self._add_waiter(tid, on_done)
            if not self._send_existing(tid, slot):
                self.ring.free([slot])
                serialized, _ = self.cp.store.upsert(tid, PUBLISH_FAILED, STATE_FAILED, self.endpoint, None, True)
                self._fire(tid)
            return serialized
        if on_done is not None and self.is_pool:
            self.worker.enable_completion_feed()
        if on_done is not None:
            # register before enqueueing: the batch may complete before submit returns
            tid_box: List[str] = []
            ids = self._enqueue_with_waiter([slot], trace, on_done, tid_box)
        else:
            ids = self._enqueue([slot], trace)
        serialized = self.cp.store.get(ids[0])
        rec = json.loads(serialized)
        if rec["BackendStatus"] == STATE_FAILED:
            self._fire(ids[0])
        return serialized

    def _enqueue_with_waiter(self, slots, trace, on_done, box) -> List[str]:
        # the id is only known after creation; completions that race ahead are caught by checking the
        # record state right after registration
        ids = self._enqueue(slots, trace)
        self._add_waiter(ids[0], on_done)
        rec = self.cp.store.get_record(ids[0])
        if rec is not None and rec["BackendStatus"] in ("completed", "failed"):
            self._fire(ids[0])
        return ids

    def submit_many(self, images_u8: np.ndarray, trace: str = "") -> List[str]:
        """Bulk async submit of already-decoded images (batch clients / benchmarks)."""
        n = images_u8.shape[0]
        slots = self.ring.alloc(n, timeout=60)
        self._write(slots, images_u8)
        return self._enqueue(slots, trace)

    def submit_raw_batch(self, body: bytes, trace: str = "") -> List[str]:
        """Binary batch ingest: ``n * prod(item_shape)`` raw uint8 bytes -> n tasks (one copy per run)."""
        if self.custom_decode:
            raise PayloadError("binary batch ingest is not accepted by this endpoint (its requests are decoded)", 415)
        item = int(np.prod(self.item_shape))
        if len(body) == 0 or len(body) % item:
            raise PayloadError(f"batch payload must be a multiple of {item} bytes (uint8 {self.item_shape})")
        arr = np.frombuffer(body, dtype=np.uint8).reshape(-1, *self.item_shape)
        return self.submit_many(arr, trace)

    def begin_stream_batch(self, nbytes: int, trace: str = "") -> "StreamedBatch":
        """Binary batch ingest without buffering the body: ``nbytes`` (a multiple of the item size) are
        fed chunk by chunk straight into ring slots allocated up front, then enqueued (``finish``)."""
        if self.custom_decode:
            raise PayloadError("binary batch ingest is not accepted by this endpoint (its requests are decoded)", 415)
        item = int(np.prod(self.item_shape))
        if nbytes <= 0 or nbytes % item:
            raise PayloadError(f"batch payload must be a multiple of {item} bytes (uint8 {self.item_shape})")
        n = nbytes // item
        cap = int(getattr(self.ring, "max_alloc", self.ring.nslots))  # (one allocation: one shard's partition)
        if n > cap:
            raise PayloadError(f"batch of {n} items exceeds the payload ring partition ({cap} slots)", 413)
        return StreamedBatch(self, n, item, trace)

    def _orig(self, body: bytes, content_type: str) -> Optional[str]:
        if not self.journal_cap or len(body) > self.journal_cap:
            return None
        return _ORIG_PREFIX + (content_type or "") + ";" + base64.b64encode(body).decode()

    def replay(self, task_id: str, orig: Optional[str]) -> bool:
        """Restart recovery of one unfinished task: re-ingest its journaled payload (the ``_ORIG`` body of the
        gateway path, or the slot of the previous crash-surviving ring the native ingest path wrote it to), or fail
        it with a reason."""
        if not orig or not orig.startswith(_ORIG_PREFIX):
            durable = getattr(self.worker, "durable", None) if self.is_pool else None
            arr = durable.payload(task_id) if durable is not None else None
            if arr is None:
                self.cp.store.upsert(task_id, PAYLOAD_LOST, STATE_FAILED, self.endpoint, None, True)
                return False
        else:
            ct, b64 = orig[len(_ORIG_PREFIX):].split(";", 1)
            try:
                arr = self.decode(base64.b64decode(b64), ct)
            except PayloadError:
                self.cp.store.upsert(task_id, "Task failed - invalid payload", STATE_FAILED, self.endpoint, None,
                                     True)
                return False
        slot = self.ring.alloc(1, timeout=30)[0]
        self._write([slot], arr[None])
        self.cp.store.upsert(task_id, "created - requeued after restart", STATE_CREATED, self.endpoint, None, True)
        if not self._send_existing(task_id, slot):
            self.ring.free([slot])
            self.cp.store.upsert(task_id, PUBLISH_FAILED, STATE_FAILED, self.endpoint, None, True)
            return False
        return True

    # ------------------------------------------------------------- results / completion
    def result(self, task_id: str) -> Optional[dict]:
        return self.worker.result(task_id)

    def _add_waiter(self, tid: str, cb: Callable[[str], None]) -> None:
        if self.is_pool:
            self.worker.enable_completion_feed()
            self.worker.add_waiter(tid, cb)
        else:
            with self._wmu:
                self._waiters[tid] = cb

    def _fire(self, tid: str) -> None:
        if self.is_pool:
            cb = self.worker.pop_waiter(tid)
        else:
            with self._wmu:
                cb = self._waiters.pop(tid, None)
        if cb is not None:
            cb(tid)

    def _on_done(self, ids: Sequence[str]) -> None:
        if not self._waiters:
            return
        with self._wmu:
            cbs = [(t, self._waiters.pop(t)) for t in ids if t in self._waiters]
        for t, cb in cbs:
            cb(t)

    def start(self) -> "ModelEndpoint":
        self.worker.start()
        return self

    def finish_recovery(self) -> None:
        """Restart recovery (``ControlPlane.recover``) has re-ingested what it could: drop the previous generation of
        the crash-surviving ring."""
        durable = getattr(self.worker, "durable", None) if self.is_pool else None
        if durable is not None:
            durable.release_previous()

    def stop(self) -> None:
        if self.decode_pool is not None:
            self.decode_pool.close()
            self.decode_pool = None
        self.worker.stop()
