"""The task control plane: CacheConnectorUpsert/Get + RequestReporter + transport publish, in-process.

Mirrors, as plain method calls instead of Azure Functions over HTTP:

* ``upsert``  — ``ProcessManager/CacheManager/CacheConnectorUpsert.cs:40-213`` (parse object/array,
  new GUID on empty TaskId, timestamp overwrite, per-state index moves, ``_ORIG`` body, publish,
  "Failed - unable to send to backend service." on publish failure, 400 on empty body);
* ``get``     — ``CacheConnectorGet.cs:27-73`` (200 JSON / 204 missing);
* ``current_processing_upsert`` / ``_get`` — ``RequestReporter/CurrentProcessing{Upsert,Get}.cs``
  (one key layout for both; Appendix B #8 fixed);
* ``publish`` — ``CacheConnectorUpsert.cs:220-303``: queue per endpoint (transport ``queue`` /
  ``inproc``) or webhook push (transport ``eventgrid``);
* queue-depth metric timers — ``TaskProcessLogger/TaskQueueLogger.cs`` + ``Libraries/QueueLogger.cs``.
"""
from __future__ import annotations

import json
import threading
import time
from typing import Any, Callable, Dict, Optional, Tuple

from ..config import Config, get_config
from ..store import (STATE_CREATED, STATE_FAILED, APITask, make_queue, make_store,
                     queue_name_for_endpoint)
from ..utils.logging import AI4ELogger, get_logger
from ..utils.metrics import REGISTRY, current_requests_key

PUBLISH_FAILED_STATUS = "Failed - unable to send to backend service."


class ControlPlane:
    def __init__(self, cfg: Optional[Config] = None, logger: Optional[AI4ELogger] = None,
                 store=None):
        self.cfg = cfg or get_config()
        self.log = logger or get_logger()
        self.store = store if store is not None else make_store(self.cfg.journal_path, self.cfg.store_backend)
        self._queues: Dict[str, Any] = {}
        self._qmu = threading.Lock()
        # Optional push transport (eventgrid): callable(task_id, endpoint, body) -> bool accepted.
        self.push_transport: Optional[Callable[[str, str, str], bool]] = None
        self._timers: list = []
        self._stop = threading.Event()
        # endpoint path -> fn(task_id, orig_body) that re-ingests a GPU task's payload after a restart
        self._replayers: Dict[str, Callable[[str, Optional[str]], bool]] = {}

    # ------------------------------------------------------------------ queues
    def queue_for(self, endpoint: str, shard: Optional[int] = None):
        """Queue per endpoint, named like the reference's Service Bus queue (CacheConnectorUpsert.cs:269-271).

        Queues are keyed by the endpoint *path* so ``http://host/v1/x`` and ``/v1/x`` share one queue.
        ``shard``: the queue of one control-plane shard of a GPU-sharded endpoint (``<name>-s<k>``,
        runtime/worker_pool.py ShardedWorkerPool).
        """
        key = queue_name_for_endpoint(APITask(Endpoint=endpoint).EndpointPath)
        if shard is not None:
            key = f"{key}-s{int(shard)}"
        with self._qmu:
            q = self._queues.get(key)
            if q is None:
                q = make_queue(key, self.cfg.max_delivery_count, self.cfg.queue_lock_duration_s,
                               self.cfg.queue_max_size, self.cfg.store_backend)
                self._queues[key] = q
            return q

    def queues(self) -> Dict[str, Any]:
        with self._qmu:
            return dict(self._queues)

    # ------------------------------------------------------------------ upsert / get
    def upsert(self, payload: Any) -> Tuple[int, str]:
        """CacheConnectorUpsert: returns (http_status, body)."""
        if payload is None or (isinstance(payload, (bytes, str)) and len(payload) == 0):
            self.log.log_warn("Parameters missing. Unable to create task.")
            return 400, ""
        try:
            task = APITask.from_json(payload)
        except (ValueError, json.JSONDecodeError) as e:
            self.log.log_error(f"Redis upsert failed. {e}")
            return 500, ""
        return 200, self.upsert_task(task)

    def upsert_task(self, task: APITask) -> str:
        backend_status = task.BackendStatus or STATE_CREATED
        serialized, publish_body = self.store.upsert(task.TaskId, task.Status, backend_status, task.Endpoint,
                                                     task.Body, bool(task.PublishToGrid))
        if task.PublishToGrid:
            rec = json.loads(serialized)
            t0 = time.perf_counter()
            ok = self.publish(rec["TaskId"], task.Endpoint, publish_body or "")
            if not ok:
                serialized, _ = self.store.upsert(rec["TaskId"], PUBLISH_FAILED_STATUS, STATE_FAILED, task.Endpoint,
                                                  None, True)
            self.log.log_debug(f"PublishEvent duration: {(time.perf_counter() - t0) * 1e3:.3f}", task.Endpoint,
                               rec["TaskId"])
        return serialized

    def get(self, task_id: str) -> Tuple[int, Optional[str]]:
        """CacheConnectorGet: 200 + stored JSON, 204 when missing."""
        if not task_id:
            return 400, None
        s = self.store.get(task_id)
        return (200, s) if s is not None else (204, None)

    def get_dict(self, task_id: str) -> Optional[dict]:
        return self.store.get_record(task_id)

    # ------------------------------------------------------------------ transport
    def publish(self, task_id: str, endpoint: str, body: str, ref: int = -1) -> bool:
        transport = self.cfg.transport
        if transport == "eventgrid" and self.push_transport is not None:
            return bool(self.push_transport(task_id, endpoint, body))
        return bool(self.queue_for(endpoint).send(task_id, ref, body))

    def create_async_task(self, endpoint: str, body: str, status: str = STATE_CREATED) -> str:
        """The async gateway policy (APIManagement/request_policy.xml:5-21): create + publish, return task JSON."""
        return self.upsert_task(APITask(TaskId="", Status=status, BackendStatus=STATE_CREATED, Endpoint=endpoint,
                                        Body=body, PublishToGrid=True))

    # ------------------------------------------------------------------ request reporter
    def current_processing_upsert(self, payload: Any) -> Tuple[int, Optional[int]]:
        if not payload:
            return 400, None
        d = json.loads(payload) if isinstance(payload, (bytes, str)) else payload
        if isinstance(d, list):
            d = d[0] if d else None
        if not isinstance(d, dict):
            return 400, None
        key = current_requests_key(str(d.get("ServiceCluster", "")), str(d.get("ApiPath", "")))
        val = self.store.incrby(key, int(d.get("IncrementBy", 0)) - int(d.get("DecrementBy", 0)))
        REGISTRY.gauge(key).set(val)
        return 200, val

    def current_processing_get(self, service_cluster: str, api_path: str) -> Tuple[int, Optional[int]]:
        v = self.store.get_counter(current_requests_key(service_cluster, api_path))
        return (200, v) if v is not None else (204, None)

    # ------------------------------------------------------------------ restart recovery
    def register_replayer(self, endpoint: str, fn: Callable[[str, Optional[str]], bool]) -> None:
        """A GPU model endpoint's payloads live in the payload ring, which does not survive a restart:
        its tasks are recovered by re-ingesting the journaled ``_ORIG`` body (``fn``)."""
        self._replayers[APITask(Endpoint=endpoint).EndpointPath] = fn

    def recover(self, journal_path: Optional[str] = None) -> Dict[str, int]:
        """Replay a task journal and re-enqueue unfinished work (survey §5.4).

        Tasks that were ``created`` or ``running`` when the process died are re-published with their
        original body (``{TaskId}_ORIG``), like a Service Bus redelivery. For GPU model endpoints the
        body is re-ingested into a fresh payload-ring slot by the endpoint's replayer; a task whose
        payload was not journaled is failed with a reason ("Task failed - payload lost on restart"),
        never requeued without a payload. Finished tasks stay queryable. Returns counts.
        """
        path = journal_path or self.cfg.journal_path
        n = self.store.replay(path) if path else 0
        requeued = failed = 0
        for suffix in ("_created", "_running"):
            for key in self.store.keys_with_suffix(suffix):
                for tid in self.store.zrange(key):
                    rec = self.store.get_record(tid)
                    if rec is None or not rec["PublishToGrid"]:
                        continue
                    body = self.store.get_orig_body(tid)
                    replay = self._replayers.get(rec["EndpointPath"])
                    if replay is not None:
                        if replay(tid, body):
                            requeued += 1
                        else:
                            failed += 1
                        continue
                    self.store.upsert(tid, "created - requeued after restart", STATE_CREATED, rec["Endpoint"],
                                      None, True)
                    if self.queue_for(rec["Endpoint"]).send(tid, -1, body or ""):
                        requeued += 1
        return {"replayed": n, "requeued": requeued, "failed": failed}

    # ------------------------------------------------------------------ queue-depth metrics
    def log_queue_lengths(self, suffix: str, adjust: int = 0) -> Dict[str, int]:
        """QueueLogger.LogSetCount: KEYS *suffix -> ZCARD (+adjust) -> metric."""
        out = {}
        for key in self.store.keys_with_suffix(suffix):
            n = self.store.zcard(key) + adjust
            out[key] = n
            REGISTRY.gauge(key).set(n)
        return out

    def start_metric_timers(self) -> None:
        """TaskQueueLogger (every 30 s, `_created` +1) and TaskProcessLogger (every 5 min)."""

        def loop(period, fn):
            while not self._stop.wait(period):
                try:
                    fn()
                except Exception as e:  # pragma: no cover - defensive
                    self.log.log_error(f"metric timer failed: {e}")

        def created():
            self.log_queue_lengths("_created", adjust=1)

        def processed():
            for s in ("_completed", "_running", "_failed"):
                self.log_queue_lengths(s)

        def evict():  # bounded store: finished tasks older than the TTL (and their results) are dropped
            n = self.store.evict_finished(self.cfg.finished_task_ttl_s, self.cfg.max_finished_tasks)
            if n:
                REGISTRY.counter("tasks_evicted_total").inc(n)

        for period, fn in ((self.cfg.queue_logger_period_s, created), (self.cfg.process_logger_period_s, processed),
                           (self.cfg.evict_period_s, evict)):
            t = threading.Thread(target=loop, args=(period, fn), daemon=True, name="ai4e-metric-timer")
            t.start()
            self._timers.append(t)

    def stats(self) -> dict:
        return {"tasks": self.store.size(), "queues": {k: q.stats() for k, q in self.queues().items()},
                "counters": self.store.counters()}

    def close(self) -> None:
        self._stop.set()
        for q in self.queues().values():
            q.close()
        self.store.flush()


_CP: Optional[ControlPlane] = None
_CP_MU = threading.Lock()


def get_control_plane() -> ControlPlane:
    global _CP
    with _CP_MU:
        if _CP is None:
            _CP = ControlPlane()
        return _CP


def set_control_plane(cp: Optional[ControlPlane]) -> None:
    global _CP
    with _CP_MU:
        _CP = cp
