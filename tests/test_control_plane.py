"""ControlPlane (CacheConnectorUpsert/Get + RequestReporter) and the dispatchers."""
import json
import time

import pytest

from aiforearth_api_platform_amd.config import Config
from aiforearth_api_platform_amd.gateway.control import PUBLISH_FAILED_STATUS, ControlPlane
from aiforearth_api_platform_amd.sched.dispatcher import QueueDispatcher, WebhookDispatcher


@pytest.fixture
def cp(backend):
    cfg = Config.load(env={}, store_backend=backend, queue_retry_delay_ms=0, max_delivery_count=3)
    c = ControlPlane(cfg)
    yield c
    c.close()


def test_upsert_object_array_and_empty(cp):
    assert cp.upsert(b"")[0] == 400
    code, body = cp.upsert([{"Status": "created", "BackendStatus": "created", "Endpoint": "http://x/v1/a",
                             "Body": "{}", "PublishToGrid": False}])
    assert code == 200
    t = json.loads(body)
    assert t["TaskId"] and t["EndpointPath"] == "/v1/a"
    assert cp.get(t["TaskId"]) == (200, body)
    assert cp.get("missing") == (204, None)
    assert cp.upsert("{not json")[0] == 500


def test_async_create_publishes_to_endpoint_queue(cp):
    js = json.loads(cp.create_async_task("http://10.0.0.5/v1/landcover/classify", '{"img": 1}'))
    q = cp.queue_for("http://10.0.0.5/v1/landcover/classify")
    assert q.name == "v1landcoverclassify"
    m = q.receive(1, 0.1)
    assert m[0].task_id == js["TaskId"] and bytes(m[0].body) == b'{"img": 1}'


def test_publish_failure_marks_task_failed(backend):
    cfg = Config.load(env={}, store_backend=backend, queue_max_size=1)
    cp = ControlPlane(cfg)
    cp.create_async_task("http://h/v1/full", "a")
    t = json.loads(cp.create_async_task("http://h/v1/full", "b"))
    assert t["Status"] == PUBLISH_FAILED_STATUS and t["BackendStatus"] == "failed"
    assert cp.store.zcard("/v1/full_failed") == 1 and cp.store.zcard("/v1/full_created") == 1


def test_request_reporter_counters(cp):
    up = {"ApiPath": "/v1/x/detect", "ServiceCluster": "gpu", "IncrementBy": 1, "DecrementBy": 0}
    assert cp.current_processing_upsert(json.dumps(up)) == (200, 1)
    assert cp.current_processing_upsert([dict(up, IncrementBy=0, DecrementBy=1)]) == (200, 0)
    assert cp.current_processing_get("gpu", "/v1/x/detect") == (200, 0)
    assert cp.current_processing_get("gpu", "/nope") == (204, None)
    assert cp.current_processing_upsert("")[0] == 400


def test_queue_lengths_metric(cp):
    ids = cp.store.create_many("http://h/v1/q", 4)
    cp.store.transition_many(ids[:1], "running", "r")
    assert cp.log_queue_lengths("_created", adjust=1) == {"/v1/q_created": 4}
    assert cp.log_queue_lengths("_running") == {"/v1/q_running": 1}


def _make(cp, codes):
    calls = []
    def backend(task_id, body, headers):
        calls.append((task_id, body))
        return codes.pop(0) if codes else 200
    return backend, calls


def test_dispatcher_2xx_complete(cp):
    be, calls = _make(cp, [200])
    d = QueueDispatcher(cp, "http://h/v1/ok", be, retry_delay_s=0.0)
    t = json.loads(cp.create_async_task("http://h/v1/ok", "B"))
    assert d.process_one(0.1)
    assert calls == [(t["TaskId"], b"B")] and d.stats.delivered == 1
    assert d.queue.stats()["inflight"] == 0


def test_dispatcher_429_retry_then_success(cp):
    be, calls = _make(cp, [429, 503, 200])
    d = QueueDispatcher(cp, "http://h/v1/busy", be, retry_delay_s=0.0)
    t = json.loads(cp.create_async_task("http://h/v1/busy", "B"))
    d.drain(2.0)
    assert len(calls) == 3 and d.stats.retried == 2 and d.stats.delivered == 1
    assert json.loads(cp.get(t["TaskId"])[1])["Status"].startswith("Awaiting service availability")


def test_dispatcher_retry_exhaustion_deadletters(cp):
    be, calls = _make(cp, [429] * 10)
    d = QueueDispatcher(cp, "http://h/v1/dead", be, retry_delay_s=0.0)
    t = json.loads(cp.create_async_task("http://h/v1/dead", "B"))
    d.drain(2.0)
    assert len(calls) == 3  # max_delivery_count
    rec = json.loads(cp.get(t["TaskId"])[1])
    assert rec["BackendStatus"] == "failed"


def test_dispatcher_non_retryable_fails_task(cp):
    be, _ = _make(cp, [400])
    d = QueueDispatcher(cp, "http://h/v1/bad", be)
    t = json.loads(cp.create_async_task("http://h/v1/bad", "B"))
    d.drain(1.0)
    rec = json.loads(cp.get(t["TaskId"])[1])
    assert rec["BackendStatus"] == "failed" and rec["Status"] == "Unable to send request to backend."


def test_dispatcher_threads(cp):
    be, calls = _make(cp, [])
    d = QueueDispatcher(cp, "http://h/v1/thr", be, concurrency=3, retry_delay_s=0.0, poll_s=0.01).start()
    for i in range(30):
        cp.create_async_task("http://h/v1/thr", str(i))
    deadline = time.time() + 5
    while len(calls) < 30 and time.time() < deadline:
        time.sleep(0.01)
    d.stop()
    assert sorted(int(b) for _, b in calls) == list(range(30))


def test_webhook_validation_and_retry(backend):
    cfg = Config.load(env={}, store_backend=backend, transport="eventgrid")
    cp = ControlPlane(cfg)
    codes = [500, 429, 200]
    got = []
    def be(tid, body, h):
        got.append(tid)
        return codes.pop(0)
    wh = WebhookDispatcher(cp, {"/v1/push": be}, base_backoff_s=0.001)
    cp.push_transport = wh.deliver
    assert wh.handle_event({"EventType": "Microsoft.EventGrid.SubscriptionValidationEvent",
                            "Data": {"ValidationCode": "abc"}}) == (200, {"ValidationResponse": "abc"})
    t = json.loads(cp.create_async_task("http://h/v1/push", "B"))
    wh.shutdown()
    assert got == [t["TaskId"]] * 3 and wh.stats.delivered == 1
    # exhaust attempts -> failed
    wh2 = WebhookDispatcher(cp, {"/v1/push": lambda *a: 503}, base_backoff_s=0.0)
    cp.push_transport = wh2.deliver
    t2 = json.loads(cp.create_async_task("http://h/v1/push", "C"))
    wh2.shutdown()
    assert json.loads(cp.get(t2["TaskId"])[1])["BackendStatus"] == "failed"
    code, _ = wh2.handle_event({"Id": "x", "Subject": "http://h/v1/push", "Data": {"a": 1}, "EventType": "task"})
    assert code == 503


def test_telemetry_sampler_holds_the_rate_and_keeps_tasks_whole():
    """App Insights-style adaptive sampling (maxTelemetryItemsPerSecond = 50, the reference's host.json): at 2000
    offered items/s the emitted rate settles near 50/s, a task's items are kept or dropped together, errors always
    pass, and emitted records carry the re-weighting factor."""
    import io

    from aiforearth_api_platform_amd.utils.logging import AI4ELogger, TelemetrySampler

    now = [0.0]
    s = TelemetrySampler(50.0, clock=lambda: now[0])
    kept_by_task = {}
    for i in range(20000):  # 10 s at 2000 items/s, 4 items per task
        now[0] = i / 2000.0
        t = f"task-{i // 4}"
        kept_by_task.setdefault(t, set()).add(s.keep(t))
    assert all(len(v) == 1 for v in kept_by_task.values())  # whole tasks
    late = sum(1 for t, v in kept_by_task.items() if int(t.split("-")[1]) >= 1000 and True in v) * 4
    assert 30 * 7.5 < late < 70 * 7.5, late  # last 7.5 s: ~50 items/s
    assert s.keep("", always=True) and 0.02 < s.ratio < 0.04
    import json

    out = io.StringIO()
    log = AI4ELogger(stream=out)
    log.sampler = TelemetrySampler(5.0, clock=lambda: now[0])
    for i in range(4000):
        now[0] = 100 + i / 1000.0
        log.log_info("x", task_id=f"t{i}")
    log.log_error("boom", task_id="t-err")
    exported = [json.loads(l) for l in out.getvalue().splitlines()]
    assert 10 < len(exported) < 40 and exported[-1]["message"] == "boom"
    assert any(r.get("sample_rate", 1) > 100 for r in exported)
    # the local ring (/v1/platform/logs) is not sampled: its last 1000 records are all there
    assert len(log.records) == 1000 and log.records[-1]["message"] == "boom"
    assert "sample_rate" not in log.records[-2]
    # an error burst does not use up the burst cap of the sampled lines
    s2 = TelemetrySampler(5.0, clock=lambda: 0.5)
    assert all(s2.keep("", always=True) for _ in range(100))
    assert s2.keep("t")
    assert TelemetrySampler(0).keep("any")
