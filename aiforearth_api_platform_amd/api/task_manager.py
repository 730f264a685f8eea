"""TaskManager facade + task-store clients (in-process or remote).

Same method names and return shapes as the reference:

* ``TaskManager`` — ``APIs/1.0/base-py/task_management/api_task.py:8-38``
  (``AddTask`` uses the ``taskId`` header of an upstream-created task, else creates one;
  ``CompleteTask``/``FailTask``/``UpdateTaskStatus``/``AddPipelineTask``/``GetTaskStatus``).
* ``DistributedApiTaskManager`` — ``APIs/1.0/Common/task_management/distributed_api_task.py:12-116``
  (status helpers map to BackendStatus ``completed``/``running``/``failed``; pipeline endpoint
  ``{scheme}://{netloc}/{version}/{org}/{api_name}``; missing task -> ``{"TaskId": id,
  "Status": "not found"}``).

Intended behaviour is implemented where the reference is broken (survey Appendix B): ``AddTask``
without a header really creates a task (the reference POSTs an empty body and gets 400); error
paths do not reference undefined names; one update is one atomic store call instead of a
GET+POST read-modify-write pair.
"""
from __future__ import annotations

import json
from typing import Any, Dict, Optional
from urllib.parse import urlparse

from ..store import STATE_COMPLETED, STATE_CREATED, STATE_FAILED, STATE_RUNNING, APITask


def _not_found(task_id: str) -> Dict[str, Any]:
    return {"TaskId": task_id, "Status": "not found"}


ERROR_TASK = {"TaskId": "-1", "Status": "error"}


class InProcTaskClient:
    """Talks to the in-process ControlPlane (no network hop)."""

    def __init__(self, control_plane=None):
        if control_plane is None:
            from ..gateway.control import get_control_plane

            control_plane = get_control_plane()
        self.cp = control_plane

    def upsert(self, task: Dict[str, Any]) -> Optional[Dict[str, Any]]:
        code, body = self.cp.upsert(task)
        return json.loads(body) if code == 200 else None

    def get(self, task_id: str) -> Optional[Dict[str, Any]]:
        return self.cp.get_dict(task_id)


class HttpTaskClient:
    """Talks to a remote task store over HTTP (CACHE_CONNECTOR_UPSERT_URI / _GET_URI)."""

    def __init__(self, upsert_uri: str, get_uri: str, timeout_s: float = 60.0):
        import requests

        self._s = requests.Session()
        self.upsert_uri, self.get_uri, self.timeout_s = upsert_uri, get_uri, timeout_s

    def upsert(self, task: Dict[str, Any]) -> Optional[Dict[str, Any]]:
        r = self._s.post(self.upsert_uri, json=task, timeout=self.timeout_s)
        return r.json() if r.status_code == 200 else None

    def get(self, task_id: str) -> Optional[Dict[str, Any]]:
        r = self._s.get(self.get_uri, params={"taskId": task_id}, timeout=self.timeout_s)
        if r.status_code != 200 or not r.content:
            return None
        return r.json()


def default_client():
    from ..config import get_config

    cfg = get_config()
    if cfg.cache_connector_upsert_uri and cfg.cache_connector_get_uri:
        return HttpTaskClient(cfg.cache_connector_upsert_uri, cfg.cache_connector_get_uri)
    return InProcTaskClient()


class DistributedApiTaskManager:
    def __init__(self, client=None):
        self.client = client if client is not None else default_client()

    def AddTask(self, endpoint: str = "http://localhost/", body: Optional[str] = None) -> Dict[str, Any]:
        t = self.client.upsert({"TaskId": "", "Status": STATE_CREATED, "BackendStatus": STATE_CREATED,
                                "Endpoint": endpoint, "Body": body, "PublishToGrid": False})
        return t if t is not None else dict(ERROR_TASK)

    def _UpdateTaskStatus(self, taskId: str, status: str, backendStatus: str) -> Dict[str, Any]:
        old = self.client.get(taskId)
        endpoint = old["Endpoint"] if old and old.get("Endpoint") else "http://localhost"
        t = self.client.upsert({"TaskId": taskId, "Status": status, "BackendStatus": backendStatus,
                                "Endpoint": endpoint, "PublishToGrid": False})
        return t if t is not None else _not_found(taskId)

    def CompleteTask(self, taskId: str, status: str) -> Dict[str, Any]:
        return self._UpdateTaskStatus(taskId, status, STATE_COMPLETED)

    def UpdateTaskStatus(self, taskId: str, status: str) -> Dict[str, Any]:
        return self._UpdateTaskStatus(taskId, status, STATE_RUNNING)

    def FailTask(self, taskId: str, status: str) -> Dict[str, Any]:
        return self._UpdateTaskStatus(taskId, status, STATE_FAILED)

    @staticmethod
    def next_endpoint(old_endpoint: str, organization_moniker: str, version: str, api_name: str) -> str:
        p = urlparse(old_endpoint)
        return "{}://{}/{}".format(p.scheme, p.netloc, "{}/{}/{}".format(version, organization_moniker, api_name))

    def AddPipelineTask(self, taskId: str, organization_moniker: str, version: str, api_name: str,
                        body: Any) -> Dict[str, Any]:
        old = self.client.get(taskId)
        if old is None:
            return dict(ERROR_TASK)
        nxt = self.next_endpoint(old["Endpoint"], organization_moniker, version, api_name)
        if body is not None and not isinstance(body, str):
            body = json.dumps(body)
        t = self.client.upsert({"TaskId": taskId, "Status": STATE_CREATED, "BackendStatus": STATE_CREATED,
                                "Endpoint": nxt, "Body": body, "PublishToGrid": True})
        return t if t is not None else _not_found(taskId)

    def GetTaskStatus(self, taskId: str) -> Dict[str, Any]:
        t = self.client.get(str(taskId))
        return t if t is not None else _not_found(str(taskId))


class TaskManager:
    def __init__(self, client=None):
        self.distributed_api_task = DistributedApiTaskManager(client)

    def AddTask(self, request=None) -> Dict[str, Any]:
        headers = getattr(request, "headers", None) or {}
        tid = headers.get("taskId") if hasattr(headers, "get") else None
        if tid:
            return self.distributed_api_task.GetTaskStatus(tid)
        endpoint = getattr(request, "url", None) or "http://localhost/"
        return self.distributed_api_task.AddTask(str(endpoint))

    def CompleteTask(self, taskId, status):
        return self.distributed_api_task.CompleteTask(taskId, status)

    def FailTask(self, taskId, status):
        return self.distributed_api_task.FailTask(taskId, status)

    def UpdateTaskStatus(self, taskId, status):
        return self.distributed_api_task.UpdateTaskStatus(taskId, status)

    def AddPipelineTask(self, taskId, organization_moniker, version, api_name, body):
        return self.distributed_api_task.AddPipelineTask(taskId, organization_moniker, version, api_name, body)

    def GetTaskStatus(self, taskId):
        return self.distributed_api_task.GetTaskStatus(taskId)
