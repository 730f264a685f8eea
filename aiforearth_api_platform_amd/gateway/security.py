"""Gateway security surface: subscription keys, TLS and the OpenAPI description of the route table.

The reference puts Azure API Management in front of the cluster: every published API is reached with a
subscription key (APIM's ``Ocp-Apim-Subscription-Key`` header or ``subscription-key`` query parameter; the
Function apps behind it take a function key, ``APIManagement/create_async_api_management_api.sh:33-42``), the
API documentation is generated from the API definitions (``APIManagement/README.md:2``), and the Istio
gateway terminates HTTPS on :443 with a mounted certificate (``Cluster/networking/secure_routing_base.yml:9-16``).
Here the one gateway process (and its ingest front-ends) does all three:

* :class:`KeyAuth` — global keys (``Config.subscription_keys``) valid on every API and task-management route,
  plus per-route keys (``keys:`` in the route table); a request without a valid key gets APIM's 401 JSON;
* :func:`server_ssl_context` — a TLS server context from a PEM certificate chain + key;
* :func:`openapi_document` — an OpenAPI 3.0 document listing every route (``GET /openapi.json``).
"""
from __future__ import annotations

import hmac
import ssl
from typing import Any, Dict, Iterable, List, Optional, Tuple

KEY_HEADER = "Ocp-Apim-Subscription-Key"
KEY_QUERY = "subscription-key"
MISSING_KEY = ("Access denied due to missing subscription key. Make sure to include subscription key when making "
               "requests to an API.")
INVALID_KEY = ("Access denied due to invalid subscription key. Make sure to provide a valid key for an active "
               "subscription.")


def parse_keys(spec: Any) -> List[str]:
    """Comma-separated string or a sequence -> list of non-empty keys."""
    if not spec:
        return []
    items = spec.split(",") if isinstance(spec, str) else list(spec)
    return [str(k).strip() for k in items if str(k).strip()]


class KeyAuth:
    """Subscription-key check. ``global_keys`` open every protected route; a route's own ``keys`` open that
    route only. With no global keys, routes without keys of their own are open."""

    def __init__(self, global_keys: Iterable[str] = ()):
        self.global_keys = parse_keys(list(global_keys))

    @property
    def enabled(self) -> bool:
        return bool(self.global_keys)

    @staticmethod
    def presented(headers, query) -> Optional[str]:
        k = headers.get(KEY_HEADER)
        if k is None and query is not None:
            k = query.get(KEY_QUERY)
        return k

    @staticmethod
    def _match(key: str, allowed: Iterable[str]) -> bool:
        ok = False
        for a in allowed:  # constant-time per candidate; no early exit on the first match
            ok |= hmac.compare_digest(key.encode(), a.encode())
        return ok

    def check(self, headers, query=None, route_keys: Optional[Iterable[str]] = None,
              locked: bool = False) -> Optional[Tuple[int, dict]]:
        """None when the request may pass, else (401, APIM-style body). ``locked``: the route is protected even
        when no key opens it (a request then always gets 401)."""
        allowed = list(self.global_keys) + parse_keys(route_keys or [])
        if not allowed and not locked:
            return None
        key = self.presented(headers, query)
        if not key:
            return 401, {"statusCode": 401, "message": MISSING_KEY}
        if not self._match(key, allowed):
            return 401, {"statusCode": 401, "message": INVALID_KEY}
        return None


def server_ssl_context(cert: str, key: str) -> Optional[ssl.SSLContext]:
    """TLS server context (TLS 1.2+) from PEM files; None when neither is configured."""
    if not cert and not key:
        return None
    if not (cert and key):
        raise ValueError("TLS needs both a certificate (AI4E_TLS_CERT) and a private key (AI4E_TLS_KEY)")
    ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    ctx.minimum_version = ssl.TLSVersion.TLSv1_2
    ctx.load_cert_chain(cert, key)
    return ctx


_TASK_SCHEMA = {
    "type": "object",
    "description": "Task status record (ProcessManager/Classes/APITask.cs field names and order)",
    "properties": {
        "TaskId": {"type": "string"},
        "Timestamp": {"type": "string"},
        "Status": {"type": "string"},
        "BackendStatus": {"type": "string", "enum": ["created", "running", "completed", "failed"]},
        "Endpoint": {"type": "string"},
        "Body": {"type": "string", "nullable": True},
        "PublishToGrid": {"type": "boolean"},
        "EndpointPath": {"type": "string"},
    },
}


def openapi_document(routes: List[Any], title: str = "AI for Earth API Platform (MI355X)", version: str = "1.0",
                     keys_required: bool = False, servers: Optional[List[str]] = None) -> Dict[str, Any]:
    """OpenAPI 3.0 document of the gateway: every route of the route table plus the task-management API.
    ``routes``: gateway ``Route`` objects (prefix, mode, content_types, max_content_length, keys, rewrite,
    max_concurrent)."""
    paths: Dict[str, Any] = {}
    secured = keys_required

    def op_security(route_keys) -> Optional[list]:
        return [{"subscriptionKey": []}, {"subscriptionKeyQuery": []}] if (keys_required or route_keys) else None

    for r in routes:
        ct = list(r.content_types or ["application/json", "application/octet-stream", "image/jpeg", "image/png"])
        body = {"required": True, "content": {c: {"schema": {"type": "string", "format": "binary"}} for c in ct}}
        if r.mode == "async":
            ok = {"description": "Task created: the task status record (Accept: text/plain -> 'TaskId: <id>'); "
                                 "binary batches (application/x-ai4e-batch) answer {\"TaskIds\": [...]}",
                  "content": {"application/json": {"schema": {"$ref": "#/components/schemas/APITask"}}}}
        else:
            ok = {"description": "Model output", "content": {"application/json": {"schema": {"type": "object"}}}}
        responses = {"200": ok,
                     "400": {"description": "Undecodable payload"},
                     "401": {"description": "Missing / invalid subscription key, or content type not accepted"},
                     "413": {"description": "Request content too large"},
                     "429": {"description": "Service is busy (maximum concurrent requests)"},
                     "503": {"description": "Service is terminating"}}
        if r.mode == "sync":
            responses["504"] = {"description": "Task did not finish within the sync timeout"}
        op: Dict[str, Any] = {"summary": f"{r.mode} API {r.prefix}", "operationId": "api_" + r.prefix.strip("/").replace("/", "_"),
                              "requestBody": body, "responses": responses,
                              "x-ai4e": {"mode": r.mode, "rewrite": r.rewrite, "max_concurrent": r.max_concurrent,
                                         "max_content_length": r.max_content_length}}
        sec = op_security(getattr(r, "keys", None))
        if sec:
            op["security"] = sec
            secured = True
        paths[r.prefix] = {"post": op}
        paths[r.prefix.rstrip("/") + "/{operation}"] = {
            "post": dict(op, operationId=op["operationId"] + "_sub",
                         parameters=[{"name": "operation", "in": "path", "required": True,
                                      "schema": {"type": "string"}}])}
    tsec = op_security(None)
    tid = [{"name": "taskId", "in": "path", "required": True, "schema": {"type": "string"}}]
    for suffix, summary, content in (
            ("", "Task status (task_management_policy.xml -> CacheConnectorGet)",
             {"application/json": {"schema": {"$ref": "#/components/schemas/APITask"}}}),
            ("/result", "Model output of a completed task", {"application/json": {"schema": {"type": "object"}}}),
            ("/trace", "Per-stage timeline and B3 trace ids of a task", {"application/json": {"schema": {"type": "object"}}})):
        op = {"summary": summary, "operationId": "task" + suffix.replace("/", "_"), "parameters": tid,
              "responses": {"200": {"description": "OK", "content": content}, "204": {"description": "Unknown task"},
                            "401": {"description": "Missing / invalid subscription key"}}}
        if tsec:
            op["security"] = tsec
        paths["/v1/taskmanagement/task/{taskId}" + suffix] = {"get": op}
    paths["/"] = {"get": {"summary": "Health check", "operationId": "health",
                          "responses": {"200": {"description": "Health check OK"},
                                        "503": {"description": "Service is terminating"}}}}
    doc: Dict[str, Any] = {
        "openapi": "3.0.3",
        "info": {"title": title, "version": version},
        "paths": paths,
        "components": {"schemas": {"APITask": _TASK_SCHEMA}},
    }
    if servers:
        doc["servers"] = [{"url": s} for s in servers]
    if secured:
        doc["components"]["securitySchemes"] = {
            "subscriptionKey": {"type": "apiKey", "in": "header", "name": KEY_HEADER},
            "subscriptionKeyQuery": {"type": "apiKey", "in": "query", "name": KEY_QUERY}}
    return doc
