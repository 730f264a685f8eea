"""Task-status JSON schema (wire-compatible with the reference).

Field names and order follow ``ProcessManager/Classes/APITask.cs:12-27`` as serialized by
Newtonsoft (get-only ``EndpointPath`` included): ``TaskId, Timestamp, Status, BackendStatus,
Endpoint, Body, PublishToGrid, EndpointPath``.  ``BackendStatus`` takes the four values of
``CacheConnectorUpsert.cs:33-36``; ``Status`` is free text.
"""
from __future__ import annotations

import json
from dataclasses import dataclass
from typing import Any, Dict, Optional

from .pystore import absolute_path

STATE_CREATED = "created"
STATE_RUNNING = "running"
STATE_COMPLETED = "completed"
STATE_FAILED = "failed"
BACKEND_STATES = (STATE_CREATED, STATE_RUNNING, STATE_COMPLETED, STATE_FAILED)

FIELD_ORDER = ("TaskId", "Timestamp", "Status", "BackendStatus", "Endpoint", "Body", "PublishToGrid",
               "EndpointPath")


@dataclass
class APITask:
    TaskId: str = ""
    Timestamp: str = ""
    Status: str = ""
    BackendStatus: str = ""
    Endpoint: str = ""
    Body: Optional[str] = None
    PublishToGrid: bool = False

    @property
    def EndpointPath(self) -> str:
        return absolute_path(self.Endpoint)

    @classmethod
    def from_json(cls, payload: Any) -> "APITask":
        """Accepts an object or an array (first element used), like CacheConnectorUpsert.cs:63-70."""
        if isinstance(payload, (bytes, str)):
            payload = json.loads(payload)
        if isinstance(payload, list):
            if not payload:
                raise ValueError("empty task array")
            payload = payload[0]
        if not isinstance(payload, dict):
            raise ValueError("task must be a JSON object")
        body = payload.get("Body")
        if body is not None and not isinstance(body, str):
            body = json.dumps(body)
        pub = payload.get("PublishToGrid", False)
        if isinstance(pub, str):
            pub = pub.strip().lower() == "true"
        return cls(TaskId=str(payload.get("TaskId") or ""), Timestamp=str(payload.get("Timestamp") or ""),
                   Status=str(payload.get("Status") or ""), BackendStatus=str(payload.get("BackendStatus") or ""),
                   Endpoint=str(payload.get("Endpoint") or ""), Body=body, PublishToGrid=bool(pub))

    def to_dict(self) -> Dict[str, Any]:
        return {"TaskId": self.TaskId, "Timestamp": self.Timestamp, "Status": self.Status,
                "BackendStatus": self.BackendStatus, "Endpoint": self.Endpoint, "Body": self.Body,
                "PublishToGrid": self.PublishToGrid, "EndpointPath": self.EndpointPath}


def queue_name_for_endpoint(endpoint: str) -> str:
    """Queue per endpoint: the URL with '.', '/', ':' removed (CacheConnectorUpsert.cs:269-271)."""
    return endpoint.replace(".", "").replace("/", "").replace(":", "")
