"""Durable payloads on the native ingest path: the payload ring survives a crash of the serving tree.

The reference makes every task durable whatever path it came in on: ``CacheConnectorUpsert.cs:125-176`` writes the
task and its ``{TaskId}_ORIG`` body to Redis in one MULTI, and the Service Bus message persists until it is
completed. Here the native front-ends (``csrc/ingest/ingestd.cpp``) ``recv()`` request bodies straight into ring
slots and never hand the bytes to Python, so journaling them as base64 ``_ORIG`` text (what the gateway path does,
:mod:`runtime.model_endpoint`) would cost a second copy of every payload. Instead, with a task journal configured:

* the endpoint's payload ring is a POSIX shared-memory segment with a deterministic name that nothing unlinks on a
  crash (it is unregistered from Python's resource tracker; a clean stop unlinks it);
* a parallel *tag* segment holds, per slot, the id of the task whose payload the slot carries. The node scheduler
  writes the tags and flushes the task records to the journal before any id is acknowledged
  (``NodeScheduler::set_slot_tags``, ``csrc/core/scheduler.h``);
* a sidecar file next to the journal names the current segments. A restarted node opens the previous generation,
  and :meth:`DurableRing.payload` returns an unfinished task's payload for :meth:`ModelEndpoint.replay`, which
  re-ingests it into the new ring. A task whose slot was reused since (its completion record was lost with the
  crash) fails with a reason, never with another task's payload.
"""
from __future__ import annotations

import hashlib
import json
import os
import threading
from multiprocessing import resource_tracker, shared_memory
from typing import Dict, Optional, Sequence, Tuple

import numpy as np

TAG_BYTES = 48  # NodeScheduler::kTagBytes
PREFIX = "ai4ej_"  # segments that must outlive a crash (runtime/gpu_worker.attach_ring leaves them untracked)


_reg_mu = threading.Lock()


def open_untracked(name: str, create: bool = False, size: int = 0) -> shared_memory.SharedMemory:
    """A shared-memory segment Python's resource tracker never hears of (it would unlink it when the tracked
    processes exit, crash included; Python 3.10 has no ``track=False``). Every process that maps a durable segment
    maps it this way (runtime/gpu_worker.attach_ring)."""
    with _reg_mu:
        reg = resource_tracker.register
        resource_tracker.register = lambda *a, **k: None
        try:
            return shared_memory.SharedMemory(name=name, create=create, size=size)
        finally:
            resource_tracker.register = reg


def _unlink(shm: shared_memory.SharedMemory) -> None:
    """Unlink without telling the resource tracker (it never registered the segment)."""
    import _posixshmem  # (what SharedMemory.unlink calls, minus the tracker message)

    try:
        _posixshmem.shm_unlink(shm._name)  # type: ignore[attr-defined]
    except FileNotFoundError:
        pass


def _create(name: str, size: int) -> shared_memory.SharedMemory:
    try:  # a stale segment of the same generation (an earlier crash during startup)
        old = open_untracked(name)
        old.close()
        _unlink(old)
    except FileNotFoundError:
        pass
    return open_untracked(name, create=True, size=max(1, size))


def _open(name: str) -> Optional[shared_memory.SharedMemory]:
    try:
        return open_untracked(name)
    except FileNotFoundError:
        return None


class DurableRing:
    """The crash-surviving payload ring of one pool endpoint (generation ``gen``) and the previous generation's."""

    def __init__(self, journal_path: str, endpoint: str):
        """``endpoint``: the endpoint's path (not its URL: the port may differ across restarts)."""
        key = os.path.abspath(journal_path) + "|" + endpoint
        self.h = hashlib.sha1(key.encode()).hexdigest()[:12]
        self.sidecar = f"{journal_path}.ring-{self.h}.json"
        self.prev: Optional[dict] = None
        gen = 0
        if os.path.exists(self.sidecar):
            try:
                with open(self.sidecar) as f:
                    self.prev = json.load(f)
                gen = int(self.prev.get("gen", 0)) + 1
            except (ValueError, OSError):
                self.prev = None
        self.gen = gen
        self.ring_name = f"{PREFIX}{self.h}_{gen}"
        self.tags_name = f"{PREFIX}{self.h}_{gen}_t"
        self.ring_shm: Optional[shared_memory.SharedMemory] = None
        self.tags_shm: Optional[shared_memory.SharedMemory] = None
        self._prev_ring: Optional[shared_memory.SharedMemory] = None
        self._prev_tags: Optional[shared_memory.SharedMemory] = None
        self._prev_index: Optional[Dict[str, int]] = None

    # ---------------------------------------------------------------- this generation
    def create(self, nslots: int, item_shape: Sequence[int]) -> Tuple[shared_memory.SharedMemory, str]:
        """Create this generation's ring + tag segments and record them in the sidecar. Returns the ring segment."""
        from .jpeg_gpu import RING_TAIL_BYTES

        item = int(np.prod(item_shape))
        self._nbytes = int(nslots) * item
        self.ring_shm = _create(self.ring_name, self._nbytes + RING_TAIL_BYTES)
        self.tags_shm = _create(self.tags_name, int(nslots) * TAG_BYTES)
        meta = {"gen": self.gen, "ring": self.ring_name, "tags": self.tags_name, "nslots": int(nslots),
                "item_shape": [int(v) for v in item_shape]}
        tmp = self.sidecar + ".tmp"
        with open(tmp, "w") as f:
            json.dump(meta, f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, self.sidecar)
        return self.ring_shm, self.tags_name

    def close(self) -> None:
        """Clean stop: nothing is left to recover from this generation."""
        if self.tags_shm is not None:
            self.tags_shm.close()
            _unlink(self.tags_shm)
        if self.ring_shm is not None:  # (SharedPayloadRing closed its mapping already)
            _unlink(self.ring_shm)
        self.tags_shm = self.ring_shm = None
        try:
            with open(self.sidecar) as f:
                if json.load(f).get("gen") == self.gen:
                    os.unlink(self.sidecar)
        except (OSError, ValueError):
            pass
        self.release_previous()

    # ---------------------------------------------------------------- the previous generation (recovery)
    def _load_previous(self) -> bool:
        if self._prev_index is not None:
            return bool(self._prev_index)
        self._prev_index = {}
        if not self.prev:
            return False
        ring, tags = _open(self.prev["ring"]), _open(self.prev["tags"])
        if ring is None or tags is None:
            for s in (ring, tags):
                if s is not None:
                    s.close()
            return False
        self._prev_ring, self._prev_tags = ring, tags
        n = int(self.prev["nslots"])
        raw = np.frombuffer(tags.buf, dtype=np.uint8, count=n * TAG_BYTES).reshape(n, TAG_BYTES)
        for slot in np.nonzero(raw[:, 0])[0]:
            tid = bytes(raw[slot]).split(b"\0", 1)[0].decode(errors="replace")
            self._prev_index[tid] = int(slot)
        del raw  # (no view may outlive the mapping)
        return True

    def payload(self, task_id: str) -> Optional[np.ndarray]:
        """The previous generation's payload of ``task_id`` (a copy), or None when no slot is tagged with it."""
        if not self._load_previous():
            return None
        slot = self._prev_index.get(task_id[:TAG_BYTES - 1])
        if slot is None:
            return None
        shape = tuple(int(v) for v in self.prev["item_shape"])
        item = int(np.prod(shape))
        nbytes = int(self.prev["nslots"]) * item
        ring = np.frombuffer(self._prev_ring.buf, dtype=np.uint8, count=nbytes)
        out = ring[slot * item:(slot + 1) * item].copy()
        # a JPEG frame prepared into the slot is marked with the previous ring's key: re-key it for this ring's workers
        from .jpeg_gpu import SLOT_MAGIC, TRAILER_BYTES, ring_key

        old_key = ring_key(self._prev_ring.buf, nbytes)
        if old_key and item > TRAILER_BYTES:
            tr = out[item - TRAILER_BYTES:item - TRAILER_BYTES + 16].view(np.uint64)
            if int(tr[0]) == SLOT_MAGIC and int(tr[1]) == old_key:
                tr[1] = ring_key(self.ring_shm.buf, self._nbytes) if self.ring_shm is not None else 0
        return out.reshape(shape)

    def release_previous(self) -> None:
        """Recovery is over: unlink the previous generation's segments."""
        for shm in (self._prev_ring, self._prev_tags):
            if shm is not None:
                try:
                    shm.close()
                except BufferError:  # (a numpy view still alive: unlink anyway)
                    pass
        self._prev_ring = self._prev_tags = None
        if self.prev:
            for name in (self.prev.get("ring"), self.prev.get("tags")):
                s = _open(name) if name else None
                if s is not None:
                    s.close()
                    _unlink(s)
        self.prev = None
        self._prev_index = {}
