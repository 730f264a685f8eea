"""Torch-free ingest pieces shared by the gateway process and the ingest front-end processes.

* :class:`StreamedBatch` — a binary batch request body streamed chunk by chunk into payload-ring slots;
* :class:`IngestShard` — one front-end process's share of an endpoint: its partition of the node's shared
  payload ring (native ``SlotRing``), and the connection over which it hands the node scheduler the filled
  slots together with the task ids it minted (SUBMIT_IDS, acknowledged once the tasks exist) and gets its
  slots back (FREE) when the tasks finish.
"""
from __future__ import annotations

import asyncio
import itertools
import threading
import uuid
from typing import Dict, List, Optional, Sequence

import numpy as np

from .decode import PayloadError


class StreamedBatch:
    """Ring slots of one streamed batch request; bytes land in slot order (one copy per chunk piece)."""

    def __init__(self, ep, n: int, item: int, trace: str):
        self.ep, self.n, self.item, self.trace = ep, n, item, trace
        self.slots: List[int] = []
        self.pos = 0
        buf = ep.ring.buf
        self._flat = (buf.numpy() if hasattr(buf, "numpy") else buf).reshape(-1)  # torch or numpy ring

    def try_alloc(self) -> bool:
        """Non-blocking slot allocation (the event loop's fast path)."""
        s = self.ep.ring.slots.alloc(self.n, 0.0) if hasattr(self.ep.ring, "slots") else None
        if s:
            self._set(s)
        return bool(s)

    def alloc(self, timeout: float = 60.0) -> None:
        self._set(self.ep.ring.alloc(self.n, timeout=timeout))

    def _set(self, slots: List[int]) -> None:
        self.slots = list(slots)
        # contiguous slot runs: (first logical byte, ring byte offset, bytes)
        self.runs, i = [], 0
        while i < self.n:
            j = i + 1
            while j < self.n and self.slots[j] == self.slots[j - 1] + 1:
                j += 1
            self.runs.append((i * self.item, self.slots[i] * self.item, (j - i) * self.item))
            i = j
        self._run = 0

    def feed(self, chunk: bytes) -> None:
        src = np.frombuffer(chunk, np.uint8)
        off, m = 0, src.shape[0]
        if self.pos + m > self.n * self.item:
            raise PayloadError("batch payload longer than its Content-Length")
        while off < m:
            lo, ring_off, nb = self.runs[self._run]
            k = min(m - off, lo + nb - self.pos)
            dst = ring_off + self.pos - lo
            self._flat[dst:dst + k] = src[off:off + k]
            off += k
            self.pos += k
            if self.pos == lo + nb:
                self._run += 1

    def take_slots(self) -> List[int]:
        """The filled slots, once every byte arrived (ownership passes to the caller)."""
        if self.pos != self.n * self.item:
            raise PayloadError(f"batch payload truncated ({self.pos} of {self.n * self.item} bytes)")
        slots, self.slots = self.slots, []
        return slots

    def finish(self) -> List[str]:
        return self.ep._enqueue(self.take_slots(), self.trace)

    def abort(self) -> None:
        if self.slots:
            self.ep.ring.free(self.slots)
            self.slots = []


class IngestShard:
    """Front-end side of one endpoint (see module docstring); ``ring`` / ``_enqueue`` match what
    :class:`StreamedBatch` expects of an endpoint."""

    def __init__(self, conn, endpoint: str, shm_name: str, nslots: int, item_shape: Sequence[int], base: int,
                 length: int, on_close=None, digits: Optional[str] = None):
        from multiprocessing import shared_memory

        from ..store import native
        from . import protocol as P

        self.endpoint = endpoint
        self.item_shape = tuple(int(x) for x in item_shape)
        self.nslots = int(nslots)
        # spawned by the ring's owner: same resource tracker (no unregister, see worker_pool.SharedPayloadRing)
        self._shm = shared_memory.SharedMemory(name=shm_name)
        self.buf = np.ndarray((self.nslots, *self.item_shape), dtype=np.uint8, buffer=self._shm.buf)
        from .jpeg_gpu import ring_key

        self.jpeg_key = ring_key(self._shm.buf, self.buf.nbytes)  # (runtime/jpeg_gpu.py prepared JPEG slots)
        self.slots = native.SlotRing(int(length), int(base))
        self.part_len = int(length)
        self.fc = P.FrameConn(conn)
        self._P = P
        self._tokens = itertools.count(1)
        self._acks: Dict[int, object] = {}
        self._amu = threading.Lock()
        self._shard = itertools.count()
        self._digits = digits or "01234567"  # the task-store lock domains of this scheduler shard
        self._on_close = on_close  # called once the scheduler connection is gone (the serving process exited)
        self._closing = False
        self.ring = self  # StreamedBatch's view of an endpoint
        self._reader = threading.Thread(target=self._read_loop, daemon=True, name="ai4e-ingest-reader")
        self._reader.start()

    # ---------------------------------------------------------------- ring
    def alloc(self, n: int, timeout: Optional[float] = 30.0) -> List[int]:
        s = self.slots.alloc(int(n), -1.0 if timeout is None else float(timeout))
        if not s:
            raise TimeoutError("payload ring partition full")
        return s

    def free(self, slots: Sequence[int]) -> None:
        self.slots.free(list(slots))

    def write(self, slot: int, arr: np.ndarray) -> None:
        self.buf[slot] = arr

    # ---------------------------------------------------------------- tasks
    def mint_ids(self, n: int) -> List[str]:
        """uuid4 task ids whose last hex digit picks one store shard for the whole call (csrc task_store.h)."""
        d = self._digits[next(self._shard) % len(self._digits)]
        return [str(uuid.uuid4())[:-1] + d for _ in range(n)]

    def submit_ids(self, slots: Sequence[int], ids: Sequence[str], trace: str = ""):
        """Hand filled slots to the scheduler; returns a waitable that resolves once the tasks exist."""
        token = next(self._tokens)
        fut = _Ack()
        with self._amu:
            self._acks[token] = fut
        self.fc.submit_ids(slots, ids, trace, token, ack=True)
        return fut

    def _enqueue(self, slots: List[int], trace: str = "") -> List[str]:  # StreamedBatch.finish (blocking)
        ids = self.mint_ids(len(slots))
        self.submit_ids(slots, ids, trace).wait(30.0)
        return ids

    def _read_loop(self) -> None:
        P = self._P
        while True:
            try:
                buf = self.fc.recv()
            except (EOFError, OSError, TypeError, ValueError):  # (the last two: closed under us by close())
                if self._on_close is not None and not self._closing:
                    self._on_close()
                return
            t = P.frame_type(buf)
            if t == P.F_FREE:
                self.slots.free(list(P.parse_slots(buf)))
            elif t == P.F_SUBMITTED:
                token, n = P.parse_submitted(buf)
                with self._amu:
                    fut = self._acks.pop(token, None)
                if fut is not None:
                    fut.set(n)
            elif t == P.F_STOP:
                return

    def close(self) -> None:
        self._closing = True
        self.fc.close()
        self.slots.close()
        del self.buf
        self._shm.close()


class _Ack:
    """Thread-set result usable from threads (``wait``) and from asyncio (``await ack.wait_async()``)."""

    def __init__(self):
        self._ev = threading.Event()
        self.value = 0
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._afut: Optional[asyncio.Future] = None
        self._mu = threading.Lock()

    def set(self, value: int) -> None:
        with self._mu:
            self.value = value
            self._ev.set()
            loop, afut = self._loop, self._afut
        if loop is not None and afut is not None:
            loop.call_soon_threadsafe(lambda: afut.done() or afut.set_result(value))

    def wait(self, timeout: float) -> int:
        if not self._ev.wait(timeout):
            raise TimeoutError("node scheduler did not acknowledge the submission")
        return self.value

    async def wait_async(self, timeout: float) -> int:
        loop = asyncio.get_running_loop()
        with self._mu:
            if self._ev.is_set():
                return self.value
            self._loop, self._afut = loop, loop.create_future()
        return await asyncio.wait_for(self._afut, timeout)
