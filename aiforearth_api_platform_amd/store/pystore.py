"""Pure-Python reference implementation of the native control-plane core.

Same API and semantics as ``csrc/core/ai4e_core.cpp`` (``TaskStore`` / ``DispatchQueue``); the
test-suite runs every store/queue test against both so the C++ core stays pinned to this
executable specification.  Semantics mirror the reference's Redis usage in
``ProcessManager/CacheManager/CacheConnectorUpsert.cs:92-176`` (insert/update, per-state sorted
sets, ``{TaskId}_ORIG`` bodies), ``CacheConnectorGet.cs:56-65`` (GET / missing),
``RequestReporter/CurrentProcessingUpsert.cs:102-104`` (INCRBY) and the Service Bus peek-lock
contract used by ``BackendQueueProcessor/BackendQueueProcessor.cs:54-75``.
"""
from __future__ import annotations

import bisect
import heapq
import json
import random
import threading
import time
import uuid
from collections import deque
from datetime import datetime, timezone
from typing import Dict, List, Optional, Tuple
from urllib.parse import urlparse


def dotnet_timestamp(epoch_s: float) -> str:
    """``DateTime.UtcNow.ToString()`` under en-US culture: ``M/d/yyyy h:mm:ss tt``."""
    d = datetime.fromtimestamp(int(epoch_s), tz=timezone.utc)
    h12 = d.hour % 12 or 12
    return f"{d.month}/{d.day}/{d.year:04d} {h12}:{d.minute:02d}:{d.second:02d} {'AM' if d.hour < 12 else 'PM'}"


def absolute_path(endpoint: str) -> str:
    """``System.Uri(Endpoint).AbsolutePath`` (APITask.cs:19-26)."""
    if "://" in endpoint:
        p = urlparse(endpoint).path
        return p or "/"
    if not endpoint:
        return "/"
    p = endpoint.split("?", 1)[0].split("#", 1)[0]
    return p if p.startswith("/") else "/" + p


def uuid4() -> str:
    return str(uuid.UUID(int=random.getrandbits(128), version=4))


class _SortedSet:
    def __init__(self):
        self.score: Dict[str, float] = {}
        self.order: List[Tuple[float, str]] = []

    def add(self, tid: str, s: float) -> None:
        if tid in self.score:
            self.order.remove((self.score[tid], tid))
        self.score[tid] = s
        bisect.insort(self.order, (s, tid))

    def rem(self, tid: str) -> bool:
        if tid not in self.score:
            return False
        self.order.remove((self.score.pop(tid), tid))
        return True

    def __len__(self):
        return len(self.score)


class _Record:
    __slots__ = ("task_id", "timestamp", "status", "backend_status", "endpoint", "endpoint_path",
                 "publish_to_grid", "t_created", "t_running", "t_finished", "result", "stage", "trace")

    def __init__(self):
        self.task_id = ""
        self.timestamp = self.status = self.backend_status = self.endpoint = self.endpoint_path = ""
        self.publish_to_grid = False
        self.t_created = self.t_running = self.t_finished = 0.0
        self.result = None
        self.stage = None
        self.trace = ""

    def as_dict(self) -> dict:
        return {"TaskId": self.task_id, "Timestamp": self.timestamp, "Status": self.status,
                "BackendStatus": self.backend_status, "Endpoint": self.endpoint, "Body": None,
                "PublishToGrid": self.publish_to_grid, "EndpointPath": self.endpoint_path}


class TaskStore:
    def __init__(self, journal_path: str = ""):
        self._mu = threading.Lock()
        self._records: Dict[str, _Record] = {}
        self._index: Dict[str, _SortedSet] = {}
        self._orig: Dict[str, str] = {}
        self._counters: Dict[str, int] = {}
        self._journal = open(journal_path, "a") if journal_path else None

    # -- internals
    def _idx(self, key: str) -> _SortedSet:
        s = self._index.get(key)
        if s is None:
            s = self._index[key] = _SortedSet()
        return s

    def _apply_index(self, r: _Record, wnow: float, mnow: float) -> None:
        p = r.endpoint_path
        self._idx(f"{p}_{r.backend_status}").add(r.task_id, float(int(wnow)))
        if r.backend_status == "running":
            self._idx(f"{p}_created").rem(r.task_id)
            r.t_running = mnow
        elif r.backend_status in ("completed", "failed"):
            self._idx(f"{p}_running").rem(r.task_id)
            self._idx(f"{p}_created").rem(r.task_id)
            r.t_finished = mnow
        elif r.backend_status == "created":
            for s in ("running", "completed", "failed"):
                self._idx(f"{p}_{s}").rem(r.task_id)
            r.t_finished = 0.0

    @staticmethod
    def _serialize(r: _Record) -> str:
        return json.dumps(r.as_dict(), separators=(",", ":"), ensure_ascii=False)

    def _journal_write(self, r: _Record, orig: Optional[str]) -> None:
        if self._journal is None:
            return
        d = r.as_dict()
        d["_score"] = int(time.time())
        if orig is not None:
            d["_orig"] = orig
        self._journal.write(json.dumps(d, separators=(",", ":"), ensure_ascii=False) + "\n")

    # -- API (mirrors the native core)
    def upsert(self, task_id: str, status: str, backend_status: str, endpoint: str,
               body: Optional[str] = None, publish_to_grid: bool = False):
        with self._mu:
            if not task_id or not task_id.strip():
                task_id = uuid4()
            wnow, mnow = time.time(), time.monotonic()
            r = self._records.get(task_id)
            if r is None:
                r = self._records[task_id] = _Record()
                r.t_created = mnow
            elif absolute_path(endpoint) != r.endpoint_path:
                self._idx(f"{r.endpoint_path}_{r.backend_status}").rem(task_id)  # pipeline hop
            r.task_id = task_id
            r.timestamp = dotnet_timestamp(wnow)
            r.status, r.backend_status, r.endpoint = status, backend_status, endpoint
            r.endpoint_path = absolute_path(endpoint)
            r.publish_to_grid = bool(publish_to_grid)
            self._apply_index(r, wnow, mnow)
            publish_body = None
            if publish_to_grid:
                if body:
                    self._orig[task_id] = body
                    publish_body = body
                else:
                    publish_body = self._orig.get(task_id, "")
            self._journal_write(r, body if (publish_to_grid and body) else None)
            return self._serialize(r), publish_body

    def create_many(self, endpoint: str, n: int, status: str = "created", trace: str = "") -> List[str]:
        with self._mu:
            wnow, mnow = time.time(), time.monotonic()
            ts, path = dotnet_timestamp(wnow), absolute_path(endpoint)
            created = self._idx(f"{path}_created")
            ids = []
            for _ in range(n):
                r = _Record()
                r.task_id = uuid4()
                r.timestamp, r.status, r.backend_status = ts, status, "created"
                r.endpoint, r.endpoint_path, r.publish_to_grid, r.t_created = endpoint, path, True, mnow
                r.trace = trace
                self._records[r.task_id] = r
                created.add(r.task_id, float(int(wnow)))
                self._journal_write(r, None)
                ids.append(r.task_id)
            return ids

    def transition_many(self, ids, backend_status: str, status: str) -> int:
        with self._mu:
            wnow, mnow = time.time(), time.monotonic()
            ts = dotnet_timestamp(wnow)
            n = 0
            for tid in ids:
                r = self._records.get(tid)
                if r is None:
                    continue
                r.timestamp, r.status, r.backend_status = ts, status, backend_status
                self._apply_index(r, wnow, mnow)
                self._journal_write(r, None)
                n += 1
            return n

    def retarget_many(self, ids, endpoint: str, status: str) -> int:
        """Pipeline hop (AddPipelineTask): same TaskIds -> created@next endpoint -> running there."""
        n = 0
        for tid in ids:
            if tid in self._records:
                self.upsert(tid, status, "created", endpoint, None, self._records[tid].publish_to_grid)
                n += 1
        self.transition_many(ids, "running", status)
        return n

    def finish_batch(self, ids, rows: bytes, row_bytes: int, ok=(), stage=(), worker: int = -1,
                     status_ok: str = "completed", status_fail: str = "Task failed - try again") -> None:
        ok = list(ok)
        with self._mu:
            wnow, mnow = time.time(), time.monotonic()
            ts = dotnet_timestamp(wnow)
            for i, tid in enumerate(ids):
                r = self._records.get(tid)
                if r is None:
                    continue
                good = not ok or bool(ok[i])
                r.timestamp, r.status = ts, status_ok if good else status_fail
                r.backend_status = "completed" if good else "failed"
                if good:
                    r.result = bytes(rows[i * row_bytes:(i + 1) * row_bytes])
                    r.stage = (list(stage) + [0.0] * 5)[:5] + [worker]
                self._apply_index(r, wnow, mnow)
                self._journal_write(r, None)

    def result(self, task_id: str) -> Optional[bytes]:
        with self._mu:
            r = self._records.get(task_id)
            return r.result if r is not None and r.backend_status == "completed" else None

    def set_trace(self, task_id: str, trace: str) -> bool:
        with self._mu:
            r = self._records.get(task_id)
            if r is None:
                return False
            r.trace = trace
            return True

    def trace(self, task_id: str) -> Optional[dict]:
        with self._mu:
            r = self._records.get(task_id)
            if r is None:
                return None
            d = {"TaskId": r.task_id, "BackendStatus": r.backend_status, "trace": r.trace, "t_created": r.t_created,
                 "t_running": r.t_running, "t_finished": r.t_finished}
            if r.stage is not None:
                d.update(worker=r.stage[5], t_worker_recv=r.stage[0], t_worker_launch=r.stage[1],
                         t_worker_done=r.stage[2], gpu_h2d_ms=r.stage[3], gpu_compute_ms=r.stage[4])
            return d

    def latencies_window(self, path: str, t0: float, t1: float) -> List[float]:
        with self._mu:
            return [r.t_finished - r.t_created for r in self._records.values()
                    if r.endpoint_path == path and r.backend_status in ("completed", "failed")
                    and t0 <= r.t_finished <= t1]

    def set_status_text(self, task_id: str, status: str) -> bool:
        with self._mu:
            r = self._records.get(task_id)
            if r is None:
                return False
            r.status = status
            r.timestamp = dotnet_timestamp(time.time())
            self._journal_write(r, None)
            return True

    def get(self, task_id: str) -> Optional[str]:
        with self._mu:
            r = self._records.get(task_id)
            return None if r is None else self._serialize(r)

    def get_record(self, task_id: str) -> Optional[dict]:
        with self._mu:
            r = self._records.get(task_id)
            return None if r is None else r.as_dict()

    def get_orig_body(self, task_id: str) -> Optional[str]:
        with self._mu:
            return self._orig.get(task_id)

    def latencies(self, ids, to_running: bool = False) -> List[float]:
        out = []
        with self._mu:
            for tid in ids:
                r = self._records.get(tid)
                if r is None:
                    continue
                end = r.t_running if to_running else r.t_finished
                if end > 0:
                    out.append(end - r.t_created)
        return out

    def zcard(self, key: str) -> int:
        with self._mu:
            s = self._index.get(key)
            return 0 if s is None else len(s)

    def zrange(self, key: str, limit: int = -1) -> List[str]:
        with self._mu:
            s = self._index.get(key)
            if s is None:
                return []
            ids = [t for _, t in s.order]
            return ids if limit is None or limit < 0 else ids[:limit]

    def keys_with_suffix(self, suffix: str) -> List[str]:
        with self._mu:
            return sorted(k for k in self._index if k.endswith(suffix))

    def incrby(self, key: str, delta: int) -> int:
        with self._mu:
            self._counters[key] = self._counters.get(key, 0) + int(delta)
            return self._counters[key]

    def get_counter(self, key: str) -> Optional[int]:
        with self._mu:
            return self._counters.get(key)

    def counters(self) -> Dict[str, int]:
        with self._mu:
            return dict(sorted(self._counters.items()))

    def evict_finished(self, max_age_s: float, max_finished: Optional[int] = None) -> int:
        with self._mu:
            cutoff = time.monotonic() - max_age_s
            dead = [tid for tid, r in self._records.items() if 0 < r.t_finished <= cutoff]
            if max_finished is not None:
                dset = set(dead)
                for key, idx in self._index.items():
                    if key.endswith(("_completed", "_failed")):
                        live = [t for t in idx.score if t not in dset]  # insertion (= finish) order
                        dead += live[: max(0, len(live) - max_finished)]
            for tid in dead:
                r = self._records.pop(tid)
                self._idx(f"{r.endpoint_path}_{r.backend_status}").rem(tid)
                self._orig.pop(tid, None)
            return len(dead)

    def size(self) -> int:
        with self._mu:
            return len(self._records)

    def flush(self) -> None:
        with self._mu:
            if self._journal:
                self._journal.flush()

    def replay(self, path: str) -> int:
        n = 0
        try:
            f = open(path)
        except OSError:
            return 0
        with f, self._mu:
            saved, self._journal = self._journal, None
            for line in f:
                line = line.strip()
                if not line:
                    continue
                try:
                    d = json.loads(line)
                except json.JSONDecodeError:
                    continue
                tid = d["TaskId"]
                r = self._records.get(tid)
                if r is None:
                    r = self._records[tid] = _Record()
                    r.t_created = time.monotonic()
                elif r.backend_status:
                    self._idx(f"{r.endpoint_path}_{r.backend_status}").rem(tid)
                r.task_id, r.timestamp, r.status = tid, d["Timestamp"], d["Status"]
                r.backend_status, r.endpoint = d["BackendStatus"], d["Endpoint"]
                r.endpoint_path = absolute_path(r.endpoint)
                r.publish_to_grid = bool(d["PublishToGrid"])
                self._idx(f"{r.endpoint_path}_{r.backend_status}").add(tid, float(d["_score"]))
                if d.get("_orig") is not None:
                    self._orig[tid] = d["_orig"]
                # finished records get a finish time, so TTL eviction applies to them too
                r.t_finished = time.monotonic() if r.backend_status in ("completed", "failed") else 0.0
                n += 1
            self._journal = saved
        return n


class Message:
    __slots__ = ("seq", "task_id", "ref", "body", "delivery_count", "enqueued_at", "visible_at", "lock_until")

    def __init__(self, seq, task_id, ref=-1, body=b""):
        self.seq, self.task_id, self.ref = seq, task_id, ref
        self.body = body if isinstance(body, bytes) else str(body).encode()
        self.delivery_count = 0
        self.enqueued_at = time.monotonic()
        self.visible_at = 0.0
        self.lock_until = 0.0

    def __lt__(self, other):
        return self.visible_at < other.visible_at


class DispatchQueue:
    def __init__(self, name: str, max_delivery_count: int = 1440, lock_duration_s: float = 300.0,
                 max_size: int = 0):
        self.name = name
        self._max_delivery = max_delivery_count
        self._lock_s = lock_duration_s
        self._max_size = max_size
        self._cv = threading.Condition()
        self._ready: deque = deque()
        self._scheduled: list = []
        self._inflight: Dict[int, Message] = {}
        self._dead: List[Message] = []
        self._seq = 0
        self._dead_total = 0
        self._closed = False

    def _full(self) -> bool:
        return bool(self._max_size) and len(self._ready) + len(self._scheduled) >= self._max_size

    def send(self, task_id: str, ref: int = -1, body="") -> bool:
        with self._cv:
            if self._closed or self._full():
                return False
            self._seq += 1
            self._ready.append(Message(self._seq, task_id, ref, body))
            self._cv.notify()
            return True

    def send_many(self, ids, refs=()) -> int:
        refs = list(refs)
        if refs and len(refs) != len(ids):
            raise ValueError("ids/refs length mismatch")
        with self._cv:
            n = 0
            for i, tid in enumerate(ids):
                if self._closed or self._full():
                    break
                self._seq += 1
                self._ready.append(Message(self._seq, tid, refs[i] if refs else -1))
                n += 1
            self._cv.notify_all()
            return n

    def _requeue(self, m: Message, delay_s: float) -> str:
        if self._max_delivery > 0 and m.delivery_count >= self._max_delivery:
            self._dead.append(m)
            self._dead_total += 1
            return "deadlettered"
        m.visible_at = time.monotonic() + delay_s
        if delay_s <= 0:
            self._ready.append(m)
        else:
            heapq.heappush(self._scheduled, m)
        self._cv.notify()
        return "requeued"

    def _promote(self, now: float) -> None:
        while self._scheduled and self._scheduled[0].visible_at <= now:
            self._ready.append(heapq.heappop(self._scheduled))
        if self._inflight and self._lock_s > 0:
            for s in [s for s, m in self._inflight.items() if m.lock_until <= now]:
                self._requeue(self._inflight.pop(s), 0.0)

    def receive(self, max_n: int = 1, timeout_s: float = 0.0, linger_s: float = 0.0) -> List[Message]:
        out: List[Message] = []
        with self._cv:
            deadline = time.monotonic() + timeout_s
            while True:
                self._promote(time.monotonic())
                if self._ready or self._closed:
                    break
                now = time.monotonic()
                if now >= deadline:
                    return out
                wake = deadline
                if self._scheduled:
                    wake = min(wake, self._scheduled[0].visible_at)
                if self._inflight:
                    wake = min(wake, now + 0.05)
                self._cv.wait(max(0.0, wake - now))
            if linger_s > 0 and len(self._ready) < max_n and not self._closed:
                ldl = time.monotonic() + linger_s
                while len(self._ready) < max_n and not self._closed:
                    now = time.monotonic()
                    if now >= ldl:
                        break
                    self._cv.wait(ldl - now)
                    self._promote(time.monotonic())
            now = time.monotonic()
            while self._ready and len(out) < max_n:
                m = self._ready.popleft()
                m.delivery_count += 1
                m.lock_until = now + self._lock_s
                self._inflight[m.seq] = m
                out.append(m)
        return out

    def receive_batch(self, max_n: int = 1, timeout_s: float = 0.0, linger_s: float = 0.0):
        ms = self.receive(max_n, timeout_s, linger_s)
        return [m.task_id for m in ms], [m.ref for m in ms], [m.seq for m in ms]

    def complete(self, seqs) -> int:
        with self._cv:
            return sum(1 for s in seqs if self._inflight.pop(s, None) is not None)

    def abandon(self, seq: int, delay_s: float = 0.0) -> str:
        with self._cv:
            m = self._inflight.pop(seq, None)
            if m is None:
                return "unknown"
            return self._requeue(m, delay_s)

    def take_deadletters(self) -> List[str]:
        with self._cv:
            out = [m.task_id for m in self._dead]
            self._dead.clear()
            return out

    def close(self) -> None:
        with self._cv:
            self._closed = True
            self._cv.notify_all()

    def stats(self) -> dict:
        with self._cv:
            return {"name": self.name, "ready": len(self._ready), "scheduled": len(self._scheduled),
                    "inflight": len(self._inflight), "deadlettered": self._dead_total, "sent": self._seq}

    def depth(self) -> int:
        with self._cv:
            return len(self._ready) + len(self._scheduled)

    def set_lock_duration(self, seconds: float) -> None:
        """<= 0 disables lock expiry (queues drained by the NodeScheduler: dispatch_queue.h)."""
        with self._cv:
            self._lock_s = seconds
            now = time.monotonic()
            for m in self._inflight.values():
                m.lock_until = now + seconds if seconds > 0 else 0.0

    @property
    def lock_duration(self) -> float:
        return self._lock_s
