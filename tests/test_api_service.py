"""APIService decorator API on a Flask app: sync/async semantics, admission control, drain, tasks."""
import json
import threading

import pytest
from flask import Flask

from aiforearth_api_platform_amd import config as cfgmod
from aiforearth_api_platform_amd.api import APIService, InProcTaskClient, TaskManager
from aiforearth_api_platform_amd.gateway.control import ControlPlane, set_control_plane
from aiforearth_api_platform_amd.utils.logging import AI4ELogger


@pytest.fixture
def svc(backend):
    cfg = cfgmod.Config.load(env={"API_PREFIX": "/v1/test"}, store_backend=backend)
    cfgmod.set_config(cfg)
    cp = ControlPlane(cfg)
    set_control_plane(cp)
    app = Flask("t")
    s = APIService(app, AI4ELogger(stream=None), TaskManager(InProcTaskClient(cp)), install_signal_handlers=False)
    yield s, app.test_client(), cp
    cfgmod.set_config(None)
    set_control_plane(None)


def test_health_and_sync(svc):
    s, c, cp = svc

    def pre(req):
        return {"scale": int(req.args.get("scale", 1))}

    @s.api_sync_func(api_path="/echo", methods=["POST"], request_processing_function=pre,
                     content_types=["application/json"], content_max_length=100)
    def echo(*args, **kwargs):
        assert kwargs["api_path"] == "/echo" and callable(kwargs["func"])
        return json.dumps({"v": kwargs["request"].get_json()["v"] * kwargs["scale"]}) if "request" in kwargs else \
            json.dumps({"scale": kwargs["scale"]})

    assert c.get("/v1/test/").data == b"Health check OK"
    r = c.post("/v1/test/echo?scale=3", json={"v": 2})
    assert r.status_code == 200 and json.loads(r.data) == {"scale": 3}
    assert c.post("/v1/test/echo", data="x", content_type="text/plain").status_code == 401
    assert c.post("/v1/test/echo", data="x" * 200, content_type="application/json").status_code == 413


def test_async_task_lifecycle(svc):
    s, c, cp = svc
    done = threading.Event()

    @s.api_async_func(api_path="/detect", methods=["POST"])
    def detect(*args, **kwargs):
        tid = kwargs["taskId"]
        body = kwargs["request"].get_json()
        s.api_task_manager.UpdateTaskStatus(tid, "running - model loaded")
        s.api_task_manager.CompleteTask(tid, "completed - " + str(body["n"] * 2))
        done.set()

    r = c.post("/v1/test/detect", json={"n": 21})
    assert r.status_code == 200 and r.data.startswith(b"TaskId: ")
    tid = r.data.decode().split(": ")[1]
    assert done.wait(5)
    s.wait_idle(5)
    st = c.get(f"/v1/test/task/{tid}").get_json()
    assert st["Status"] == "completed - 42" and st["TaskId"] == tid
    rec = json.loads(cp.get(tid)[1])
    assert rec["BackendStatus"] == "completed"
    # JSON form when asked
    r = c.post("/v1/test/detect", json={"n": 1}, headers={"Accept": "application/json"})
    assert "TaskId" in r.get_json()


def test_async_uses_upstream_task_id_header(svc):
    s, c, cp = svc
    t = json.loads(cp.create_async_task("http://gw/v1/test/up", "{}"))

    @s.api_async_func(api_path="/up", methods=["POST"])
    def up(*args, **kwargs):
        s.api_task_manager.CompleteTask(kwargs["taskId"], "completed")

    r = c.post("/v1/test/up", json={}, headers={"taskId": t["TaskId"]})
    assert r.data.decode() == "TaskId: " + t["TaskId"]
    s.wait_idle(5)
    assert json.loads(cp.get(t["TaskId"])[1])["BackendStatus"] == "completed"


def test_async_failure_marks_failed(svc):
    s, c, cp = svc

    @s.api_async_func(api_path="/boom", methods=["POST"])
    def boom(*args, **kwargs):
        raise RuntimeError("model exploded")

    tid = c.post("/v1/test/boom", json={}).data.decode().split(": ")[1]
    s.wait_idle(5)
    rec = json.loads(cp.get(tid)[1])
    assert rec["BackendStatus"] == "failed" and rec["Status"] == "Task failed - try again"


def test_max_concurrency_429_and_drain_503(svc):
    s, c, cp = svc
    gate = threading.Event()

    @s.api_async_func(api_path="/slow", methods=["POST"], maximum_concurrent_requests=1)
    def slow(*args, **kwargs):
        gate.wait(5)

    assert c.post("/v1/test/slow", json={}).status_code == 200
    assert c.post("/v1/test/slow", json={}).status_code == 429  # busy, retryable
    gate.set()
    s.wait_idle(5)
    assert c.post("/v1/test/slow", json={}).status_code == 200
    s.wait_idle(5)
    s.initialize_term(2, None)
    assert c.post("/v1/test/slow", json={}).status_code == 503
    assert c.get("/v1/test/").status_code == 503


def test_pipeline_task_next_endpoint(svc):
    s, c, cp = svc
    tm = s.api_task_manager
    t = json.loads(cp.create_async_task("http://10.0.0.9/v1/org/stage1", '{"a": 1}'))
    nxt = tm.AddPipelineTask(t["TaskId"], "org", "v1", "stage2", {"crops": 3})
    assert nxt["TaskId"] == t["TaskId"] and nxt["Endpoint"] == "http://10.0.0.9/v1/org/stage2"
    assert cp.store.zcard("/v1/org/stage2_created") == 1
    q = cp.queue_for("/v1/org/stage2")
    assert json.loads(bytes(q.receive(1, 0.1)[0].body)) == {"crops": 3}
    assert tm.AddPipelineTask("missing", "o", "v1", "a", None) == {"TaskId": "-1", "Status": "error"}
    assert tm.GetTaskStatus("missing") == {"TaskId": "missing", "Status": "not found"}


def test_request_counter_metric_push(svc, monkeypatch):
    s, c, cp = svc
    s.cfg = s.cfg.replace(disable_current_request_metric=False, service_cluster="gpu")
    seen = []

    @s.api_sync_func(api_path="/cnt", methods=["GET"])
    def cnt(*args, **kwargs):
        seen.append(cp.current_processing_get("gpu", "/v1/test/cnt")[1])
        return "ok"

    assert c.get("/v1/test/cnt").data == b"ok"
    assert seen == [1] and cp.current_processing_get("gpu", "/v1/test/cnt") == (200, 0)
