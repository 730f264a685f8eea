"""Backend dispatchers: the reference's BackendQueueProcessor (pull) and BackendWebhook (push).

``QueueDispatcher`` — ``ProcessManager/BackendQueueProcessor/BackendQueueProcessor.cs:27-81``:
receive a peek-locked message, POST the body to the backend with header ``taskId``;

* 429 (and 503, which the reference service emits when busy — Appendix B #7) ->
  ``Status = "Awaiting service availability. Queued for N seconds."`` then abandon with
  ``QUEUE_RETRY_DELAY_MS`` delay (redelivery, at most ``max_delivery_count`` times, then the
  task is failed from the dead-letter list);
* other non-2xx -> complete + task failed ``"Unable to send request to backend."``;
* 2xx -> complete.

Unlike the reference's ``maxConcurrentCalls: 1`` (``host.json:5-8``), concurrency per endpoint is
configurable (``dispatch_concurrency``); the in-process backend call removes the HTTP hop.

``WebhookDispatcher`` — ``ProcessManager/BackendWebhook/BackendWebhook.cs:24-90`` plus the Event
Grid retry policy (3 attempts, 5 min TTL; ``deploy_event_grid_subscription.sh:37``): push delivery
with bounded retries; also answers the subscription-validation handshake.
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Tuple, Union

from ..store import STATE_CREATED, STATE_FAILED

# A backend receives (task_id, body_bytes, headers) and returns an HTTP-like status code
# (optionally with a response body).
BackendFn = Callable[[str, bytes, Dict[str, str]], Union[int, Tuple[int, bytes]]]

RETRYABLE = (429, 503)


def http_backend(url: str, timeout_s: float = 60.0) -> BackendFn:
    """A backend that POSTs to a remote service (the reference's HttpClient.PostAsync)."""
    import requests

    def call(task_id: str, body: bytes, headers: Dict[str, str]) -> Tuple[int, bytes]:
        h = {"taskId": task_id, "Content-Type": "application/json", **headers}
        r = requests.post(url, data=body, headers=h, timeout=timeout_s)
        return r.status_code, r.content

    return call


def _status_of(res) -> int:
    return int(res[0] if isinstance(res, tuple) else res)


@dataclass
class DispatchStats:
    delivered: int = 0
    retried: int = 0
    failed: int = 0
    deadlettered: int = 0


class QueueDispatcher:
    def __init__(self, control_plane, endpoint: str, backend: BackendFn, concurrency: Optional[int] = None,
                 retry_delay_s: Optional[float] = None, poll_s: float = 0.1, clock=time.monotonic):
        self.cp = control_plane
        self.endpoint = endpoint
        self.queue = control_plane.queue_for(endpoint)
        self.backend = backend
        self.concurrency = concurrency or control_plane.cfg.dispatch_concurrency
        self.retry_delay_s = (control_plane.cfg.queue_retry_delay_ms / 1000.0
                              if retry_delay_s is None else retry_delay_s)
        self.poll_s = poll_s
        self.clock = clock
        self.stats = DispatchStats()
        self._stop = threading.Event()
        self._threads: List[threading.Thread] = []
        self._mu = threading.Lock()

    def process_one(self, timeout_s: float = 0.0) -> bool:
        """Receive and deliver one message; returns False if nothing was received."""
        msgs = self.queue.receive(1, timeout_s, 0.0)
        if not msgs:
            self._reap_deadletters()
            return False
        m = msgs[0]
        queued_s = max(0.0, self.clock() - m.enqueued_at)
        try:
            res = self.backend(m.task_id, bytes(m.body), {})
            code = _status_of(res)
        except Exception as e:  # transport error == non-2xx
            self.cp.log.log_error(f"dispatch error: {e}", self.endpoint, m.task_id)
            code = 500
        if code in RETRYABLE:
            # Reference logs "Queued for {ms/60} seconds" (Appendix B #12); report real seconds.
            self.cp.store.set_status_text(m.task_id, f"Awaiting service availability. Queued for {queued_s:.0f} seconds.")
            outcome = self.queue.abandon(m.seq, self.retry_delay_s)
            with self._mu:
                self.stats.retried += 1
            if outcome == "deadlettered":
                self._fail(m.task_id, "Unable to send request to backend. Maximum delivery count reached.")
                with self._mu:
                    self.stats.deadlettered += 1
        elif not (200 <= code < 300):
            self.queue.complete([m.seq])
            self._fail(m.task_id, "Unable to send request to backend.")
            with self._mu:
                self.stats.failed += 1
        else:
            self.queue.complete([m.seq])
            with self._mu:
                self.stats.delivered += 1
        return True

    def _fail(self, task_id: str, status: str) -> None:
        self.cp.store.transition_many([task_id], STATE_FAILED, status)

    def _reap_deadletters(self) -> None:
        for tid in self.queue.take_deadletters():
            self._fail(tid, "Unable to send request to backend. Maximum delivery count reached.")
            with self._mu:
                self.stats.deadlettered += 1

    def _loop(self) -> None:
        while not self._stop.is_set():
            self.process_one(self.poll_s)

    def start(self) -> "QueueDispatcher":
        for i in range(self.concurrency):
            t = threading.Thread(target=self._loop, daemon=True, name=f"ai4e-dispatch-{self.queue.name}-{i}")
            t.start()
            self._threads.append(t)
        return self

    def stop(self, join_timeout: float = 2.0) -> None:
        self._stop.set()
        for t in self._threads:
            t.join(join_timeout)
        self._threads.clear()

    def drain(self, timeout_s: float = 5.0) -> None:
        """Process until the queue is empty (tests / synchronous use)."""
        deadline = time.monotonic() + timeout_s
        while time.monotonic() < deadline:
            if not self.process_one(0.0) and self.queue.depth() == 0:
                return


SUBSCRIPTION_VALIDATION_EVENT = "Microsoft.EventGrid.SubscriptionValidationEvent"


class WebhookDispatcher:
    """Push transport with Event-Grid-style retry (max attempts within a TTL, exponential backoff)."""

    def __init__(self, control_plane, backends: Dict[str, BackendFn], max_attempts: Optional[int] = None,
                 ttl_s: Optional[float] = None, base_backoff_s: float = 0.01, workers: int = 4):
        self.cp = control_plane
        self.backends = backends
        self.max_attempts = max_attempts or control_plane.cfg.eventgrid_max_delivery_attempts
        self.ttl_s = ttl_s if ttl_s is not None else control_plane.cfg.eventgrid_event_ttl_s
        self.base_backoff_s = base_backoff_s
        self.stats = DispatchStats()
        import concurrent.futures as cf

        self._pool = cf.ThreadPoolExecutor(max_workers=workers, thread_name_prefix="ai4e-webhook")

    def handle_event(self, event: dict) -> Tuple[int, Optional[dict]]:
        """BackendWebhook.Run for one EventGridEvent: validation handshake or delivery."""
        if str(event.get("EventType", event.get("eventType", ""))).lower() == SUBSCRIPTION_VALIDATION_EVENT.lower():
            data = event.get("Data", event.get("data", {})) or {}
            return 200, {"ValidationResponse": data.get("ValidationCode", data.get("validationCode"))}
        task_id = str(event.get("Id", event.get("id", "")))
        subject = str(event.get("Subject", event.get("subject", "")))
        data = event.get("Data", event.get("data", ""))
        body = data.encode() if isinstance(data, str) else __import__("json").dumps(data).encode()
        backend = self._backend_for(subject)
        if backend is None:
            return 404, None
        try:
            return _status_of(backend(task_id, body, {})), None
        except Exception:
            return 500, None

    def _backend_for(self, endpoint: str) -> Optional[BackendFn]:
        from ..store.pystore import absolute_path

        return self.backends.get(endpoint) or self.backends.get(absolute_path(endpoint))

    def deliver(self, task_id: str, endpoint: str, body: str) -> bool:
        """Transport hook for ControlPlane.push_transport: accept and deliver asynchronously."""
        self._pool.submit(self._deliver_with_retry, task_id, endpoint, body.encode() if isinstance(body, str) else body)
        return True

    def _deliver_with_retry(self, task_id: str, endpoint: str, body: bytes) -> int:
        backend = self._backend_for(endpoint)
        t0 = time.monotonic()
        code = 404
        for attempt in range(self.max_attempts):
            if backend is None:
                break
            try:
                code = _status_of(backend(task_id, body, {}))
            except Exception:
                code = 500
            if 200 <= code < 300:
                self.stats.delivered += 1
                return code
            self.stats.retried += 1
            if time.monotonic() - t0 > self.ttl_s:
                break
            time.sleep(self.base_backoff_s * (2 ** attempt))
        self.stats.failed += 1
        self.cp.store.transition_many([task_id], STATE_FAILED, "Failed - unable to send to backend service.")
        return code

    def shutdown(self) -> None:
        self._pool.shutdown(wait=True)
