"""Legacy (``Containers/``) task-manager API, kept for drop-in compatibility.

The reference's first-generation overlay (``Containers/base-py/task_management/api_task.py:6-47``,
``Containers/Common/task_management/distributed_api_task.py:7-85``) exposed
``ApiTaskManager(flask_api, resource_prefix)`` with a ``/task/<int:id>`` resource and a client
that sent ``Uuid`` instead of ``TaskId`` and built pipeline URLs as ``/{org}/{version}/{api}``.
Those field/URL differences made the legacy client talk past the C# store (survey Appendix B #9);
here the legacy surface is an adapter over the current TaskManager: ``Uuid`` is accepted as an
alias of ``TaskId`` and the legacy pipeline URL order is honoured.
"""
from __future__ import annotations

import json
from typing import Any, Dict, Optional
from urllib.parse import urlparse

from .task_manager import TaskManager


class LegacyDistributedApiTaskManager:
    """``requests``-style legacy client surface; returns dicts with both ``Uuid`` and ``TaskId``."""

    def __init__(self, task_manager: Optional[TaskManager] = None):
        self.tm = task_manager or TaskManager()

    @staticmethod
    def _with_uuid(d: Dict[str, Any]) -> Dict[str, Any]:
        d = dict(d)
        d.setdefault("Uuid", d.get("TaskId"))
        return d

    def AddTask(self, endpoint: str = "http://localhost/", body: Optional[str] = None) -> Dict[str, Any]:
        return self._with_uuid(self.tm.distributed_api_task.AddTask(endpoint, body))

    def UpdateTaskStatus(self, uuid: str, status: str) -> Dict[str, Any]:
        return self._with_uuid(self.tm.UpdateTaskStatus(uuid, status))

    def CompleteTask(self, uuid: str, status: str) -> Dict[str, Any]:
        return self._with_uuid(self.tm.CompleteTask(uuid, status))

    def FailTask(self, uuid: str, status: str) -> Dict[str, Any]:
        return self._with_uuid(self.tm.FailTask(uuid, status))

    def GetTaskStatus(self, uuid: str) -> Dict[str, Any]:
        return self._with_uuid(self.tm.GetTaskStatus(uuid))

    def AddPipelineTask(self, uuid: str, organization_moniker: str, version: str, api_name: str,
                        body: Any) -> Dict[str, Any]:
        """Legacy URL order ``/{org}/{version}/{api}`` (Containers/Common/...:59)."""
        old = self.tm.distributed_api_task.client.get(uuid)
        if old is None:
            return {"Uuid": "-1", "TaskId": "-1", "Status": "error"}
        p = urlparse(old["Endpoint"])
        nxt = f"{p.scheme}://{p.netloc}/{organization_moniker}/{version}/{api_name}"
        if body is not None and not isinstance(body, str):
            body = json.dumps(body)
        t = self.tm.distributed_api_task.client.upsert({"TaskId": uuid, "Status": "created",
                                                        "BackendStatus": "created", "Endpoint": nxt, "Body": body,
                                                        "PublishToGrid": True})
        return self._with_uuid(t or {"TaskId": uuid, "Status": "not found"})


class ApiTaskManager:
    """``ApiTaskManager(flask_api, resource_prefix)``: registers ``GET {prefix}/task/<int:id>``."""

    def __init__(self, flask_api, resource_prefix: str = "", task_manager: Optional[TaskManager] = None):
        self.client = LegacyDistributedApiTaskManager(task_manager)
        app = getattr(flask_api, "app", flask_api)  # flask_restful.Api or a Flask app

        def get_task(id):
            return self.client.GetTaskStatus(str(id))

        app.add_url_rule(resource_prefix.rstrip("/") + "/task/<id>", endpoint="ai4e_legacy_task", view_func=get_task,
                         methods=["GET"])

    def AddTask(self, request=None):
        endpoint = getattr(request, "url", None) or "http://localhost/"
        return self.client.AddTask(str(endpoint))

    def UpdateTaskStatus(self, uuid, status):
        return self.client.UpdateTaskStatus(uuid, status)

    def CompleteTask(self, uuid, status):
        return self.client.CompleteTask(uuid, status)

    def FailTask(self, uuid, status):
        return self.client.FailTask(uuid, status)

    def GetTaskStatus(self, uuid):
        return self.client.GetTaskStatus(uuid)

    def AddPipelineTask(self, uuid, organization_moniker, version, api_name, body):
        return self.client.AddPipelineTask(uuid, organization_moniker, version, api_name, body)
