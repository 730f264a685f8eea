"""Restart recovery from the journal, and the legacy Containers/ task-manager surface."""
import json

from flask import Flask

from aiforearth_api_platform_amd.api import InProcTaskClient, TaskManager
from aiforearth_api_platform_amd.api.legacy import ApiTaskManager, LegacyDistributedApiTaskManager
from aiforearth_api_platform_amd.config import Config
from aiforearth_api_platform_amd.gateway.control import ControlPlane


def test_recover_requeues_unfinished(tmp_path, backend):
    j = str(tmp_path / "j.jsonl")
    cp = ControlPlane(Config.load(env={}, journal_path=j, store_backend=backend))
    a = json.loads(cp.create_async_task("http://h/v1/x", "BODY-A"))["TaskId"]
    b = json.loads(cp.create_async_task("http://h/v1/x", "BODY-B"))["TaskId"]
    c = json.loads(cp.create_async_task("http://h/v1/x", "BODY-C"))["TaskId"]
    cp.store.transition_many([b], "running", "running")
    cp.store.transition_many([c], "completed", "done")
    cp.store.flush()
    # "crash": a new control plane over the same journal
    cp2 = ControlPlane(Config.load(env={}, journal_path=str(tmp_path / "j2.jsonl"), store_backend=backend))
    out = cp2.recover(j)
    assert out["requeued"] == 2
    q = cp2.queue_for("http://h/v1/x")
    msgs = q.receive(10, 0.1)
    assert sorted(m.task_id for m in msgs) == sorted([a, b])
    assert {bytes(m.body) for m in msgs} == {b"BODY-A", b"BODY-B"}
    assert json.loads(cp2.get(c)[1])["BackendStatus"] == "completed"


def test_legacy_surface(backend):
    cp = ControlPlane(Config.load(env={}, store_backend=backend))
    tm = TaskManager(InProcTaskClient(cp))
    app = Flask("legacy")
    mgr = ApiTaskManager(app, "/v1/legacy", tm)
    t = json.loads(cp.create_async_task("http://10.0.0.1/v1/org/a1", "{}"))
    got = mgr.GetTaskStatus(t["TaskId"])
    assert got["Uuid"] == got["TaskId"] == t["TaskId"]
    mgr.CompleteTask(t["TaskId"], "completed - legacy")
    r = app.test_client().get(f"/v1/legacy/task/{t['TaskId']}")
    assert r.get_json()["Status"] == "completed - legacy"
    nxt = mgr.AddPipelineTask(t["TaskId"], "org", "v1", "a2", {"x": 1})
    assert nxt["Endpoint"] == "http://10.0.0.1/org/v1/a2"
    new = LegacyDistributedApiTaskManager(tm).AddTask("http://h/v1/z")
    assert new["Uuid"] and new["Status"] == "created"
