"""HTTP front end: the API Management gateway + Istio routing + Functions HTTP triggers, in one process.

Routes (all served by one aiohttp application):

* ``POST <route prefix>[/...]`` — per the route table (replaces the Istio VirtualService prefix match
  + rewrite of ``APIs/Charts/templates/routing.yml:10-18`` and the APIM API definitions):
  ``async`` routes create a task and return ``200`` + the task JSON immediately
  (``APIManagement/request_policy.xml:5-28``; ``500 "Task insert failed."`` on failure); ``sync``
  routes proxy to the backend and return its response (``request_backend_policy.xml``).
* ``GET /v1/taskmanagement/task/{taskId}`` — task status, verbatim store JSON or ``204``
  (``task_management_policy.xml`` -> ``CacheConnectorGet``); ``.../result`` returns the model output,
  ``.../trace`` the per-stage timeline (accept -> batch -> worker -> GPU -> complete) + B3 ids.
* Binary batch ingest: an async model route accepts ``Content-Type: application/x-ai4e-batch`` with
  ``n`` raw uint8 payloads back to back and answers ``{"TaskIds": [...]}`` (one copy per request into
  the payload ring; the high-rate client path).
* ``POST /v1/cache/upsert``, ``GET /v1/cache/get?taskId=`` — CacheConnectorUpsert / Get.
* ``POST /v1/requests/upsert``, ``POST /v1/requests/get`` — RequestReporter (CURRENT_REQUESTS).
* ``POST /v1/backend/webhook`` — BackendWebhook incl. the Event Grid validation handshake.
* ``GET /metrics`` (Prometheus text), ``GET /v1/platform/stats`` (JSON), ``GET /`` health,
  ``GET /openapi.json`` (OpenAPI 3.0 description of the route table, gateway/security.py).

Security (gateway/security.py): APIM-style subscription keys (``Ocp-Apim-Subscription-Key`` header or
``subscription-key`` query) on every API, task-management and control route when keys are configured (global
``AI4E_SUBSCRIPTION_KEYS`` and/or per-route ``keys``; 401 otherwise; health and the OpenAPI document stay open),
and an HTTPS listener when ``AI4E_TLS_CERT`` / ``AI4E_TLS_KEY`` name a PEM certificate and key.

Admission control per route mirrors ``APIService.before_request`` (429 busy, 503 draining,
401 content type, 413 too large); undecodable payloads get 400 (415 for unknown media types) and
no task; a sync request that outlives ``sync_timeout_s`` gets 504. B3 headers
(``x-b3-traceid``/``spanid``) are read or created, stored with the task and echoed back.
"""
from __future__ import annotations

import asyncio
import json
import signal
import threading
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

from aiohttp import ClientSession, web

from ..utils.metrics import REGISTRY
from ..utils.tracing import StageClock, b3_from_headers, b3_pack, b3_unpack
from .control import ControlPlane
from .security import KeyAuth, openapi_document, parse_keys, server_ssl_context

TASK_INSERT_FAILED = "Task insert failed."


def valid_task_id(tid: str) -> bool:
    """An upstream task id (``taskId`` header) the store and the scheduler wire format accept: 1-128 printable
    ASCII characters (the wire carries ids as fixed-length byte strings, runtime/protocol.py)."""
    return 0 < len(tid) <= 128 and tid.isascii() and tid.isprintable()
BATCH_CONTENT_TYPE = "application/x-ai4e-batch"
MAX_BODY = 1 << 30  # request-body cap (aiohttp client_max_size; the native front-end applies the same one)


@dataclass
class Route:
    prefix: str
    mode: str = "async"                      # async | sync
    backend: Any = None                      # ModelEndpoint | callable(task_id, body, headers) | "http://..."
    rewrite: Optional[str] = None            # VirtualService rewrite of the matched prefix
    max_concurrent: Optional[int] = None
    content_types: Optional[List[str]] = None
    max_content_length: Optional[int] = None
    inline: bool = False                     # sync callable cheap enough to run on the event loop (no thread hop)
    keys: Optional[List[str]] = None         # subscription keys valid on this route (besides the global ones)
    inflight: int = field(default=0, repr=False)

    def target_path(self, path: str) -> str:
        if self.rewrite is None:
            return path
        return self.rewrite + path[len(self.prefix):]


class RouteTable:
    def __init__(self, routes: Optional[List[Route]] = None):
        self.routes: List[Route] = list(routes or [])
        self.version = 0  # bumped on every change (the gateway's precomputed key sets follow it)

    def add(self, route: Route) -> Route:
        self.routes.append(route)
        self.routes.sort(key=lambda r: -len(r.prefix))  # longest prefix wins
        self.version += 1
        return route

    def match(self, path: str) -> Optional[Route]:
        for r in self.routes:
            if path == r.prefix or path.startswith(r.prefix.rstrip("/") + "/"):
                return r
        return None

    @classmethod
    def from_yaml(cls, path: str, backends: Dict[str, Any]) -> "RouteTable":
        import yaml

        with open(path) as f:
            doc = yaml.safe_load(f) or {}
        t = cls()
        for r in doc.get("routes", []):
            be = r.get("backend")
            if isinstance(be, str) and be.startswith("inproc:"):
                be = backends[be.split(":", 1)[1]]
            t.add(Route(prefix=r["prefix"], mode=r.get("mode", "async"), backend=be, rewrite=r.get("rewrite"),
                        max_concurrent=r.get("max_concurrent"), content_types=r.get("content_types"),
                        max_content_length=r.get("max_content_length"), inline=bool(r.get("inline", False)),
                        keys=parse_keys(r.get("keys")) or None))
        return t


class Gateway:
    def __init__(self, control_plane: ControlPlane, routes: Optional[RouteTable] = None, webhook=None,
                 base_url: str = "http://127.0.0.1", auth: Optional[KeyAuth] = None):
        self.cp = control_plane
        self.auth = auth if auth is not None else KeyAuth(parse_keys(getattr(control_plane.cfg, "subscription_keys", "")))
        self.routes = routes or RouteTable()
        self.webhook = webhook
        self.base_url = base_url.rstrip("/")
        self.is_terminating = False
        self.on_drain: List[Callable[[], None]] = []
        self._stopped = threading.Event()
        self._session: Optional[ClientSession] = None
        self.app = web.Application(client_max_size=MAX_BODY, middlewares=[self._key_middleware])
        self.app.router.add_get("/", self.health)
        self.app.router.add_get("/openapi.json", self.openapi)
        self.app.router.add_get("/metrics", self.metrics)
        self.app.router.add_get("/v1/platform/stats", self.stats)
        self.app.router.add_get("/v1/taskmanagement/task/{taskId}", self.task_get)
        self.app.router.add_get("/v1/taskmanagement/task/{taskId}/result", self.task_result)
        self.app.router.add_get("/v1/taskmanagement/task/{taskId}/trace", self.task_trace)
        self.app.router.add_post("/v1/cache/upsert", self.cache_upsert)
        self.app.router.add_get("/v1/cache/get", self.cache_get)
        self.app.router.add_post("/v1/requests/upsert", self.requests_upsert)
        self.app.router.add_post("/v1/requests/get", self.requests_get)
        self.app.router.add_post("/v1/backend/webhook", self.backend_webhook)
        self.app.router.add_route("*", "/{tail:.*}", self.dispatch)
        self.app.on_cleanup.append(self._cleanup)
        self._c_req = REGISTRY.counter("gateway_requests_total")

    # ------------------------------------------------------------------ security
    OPEN_PATHS = ("/", "/openapi.json")
    TASK_PREFIX = "/v1/taskmanagement/"
    CONTROL_PATHS = ("/v1/cache/upsert", "/v1/cache/get", "/v1/requests/upsert", "/v1/requests/get",
                     "/v1/backend/webhook", "/metrics", "/v1/platform/stats")

    def _key_sets(self):
        """(control keys, control + every route's keys, protected?) — computed once per route-table version and
        control-key setting instead of on every request."""
        control = getattr(self.cp.cfg, "control_keys", "")
        tag = (self.routes.version, len(self.routes.routes), control, tuple(self.auth.global_keys))
        if getattr(self, "_keys_tag", None) != tag:
            control_keys = parse_keys(control)
            route_keys = [k for r in self.routes.routes for k in (r.keys or [])]
            self._keys = (control_keys, control_keys + route_keys,
                          bool(self.auth.global_keys or control_keys or route_keys))
            self._keys_tag = tag
        return self._keys

    @web.middleware
    async def _key_middleware(self, request, handler):
        """Subscription-key check ahead of every handler. API routes accept the global keys and their own. Once
        any key is configured anywhere, the task-management routes accept the global keys, the control keys and
        any route's keys (every subscriber polls its tasks), and the control routes only the global and control
        keys (no key at all opens them then: they are the reference's key-protected Function endpoints). Health
        and the OpenAPI document are open.

        Task scope is intentionally the APIM product's, not the route's: the reference publishes its TaskManagement
        API beside the model APIs for every subscriber (InfrastructureDeployment/deploy_api_management.sh:58-100, APIManagement/task_management_api_body.json),
        so a subscriber with any route's key may poll a task by id, and the id (uuid4, 122 random bits, never listed)
        is the capability. Route-scoped task reads would need the creating route's key set recorded on the task."""
        path = request.path
        if path not in self.OPEN_PATHS:
            control_keys, task_keys, protected = self._key_sets()
            if path in self.CONTROL_PATHS:
                rej = self.auth.check(request.headers, request.query, control_keys, locked=protected)
            elif path.startswith(self.TASK_PREFIX):
                rej = self.auth.check(request.headers, request.query, task_keys, locked=protected)
            else:
                route = self.routes.match(path)
                rej = self.auth.check(request.headers, request.query, route.keys if route is not None else None)
            if rej is not None:
                return web.json_response(rej[1], status=rej[0])
        return await handler(request)

    async def openapi(self, request):
        return web.json_response(openapi_document(self.routes.routes, keys_required=self.auth.enabled,
                                                  servers=[self.base_url]))

    # ------------------------------------------------------------------ platform routes
    async def health(self, request):
        if self.is_terminating:
            return web.Response(status=503, text="Service is terminating")
        return web.Response(text="Health check OK")

    async def metrics(self, request):
        for s in ("_created", "_running", "_completed", "_failed"):
            self.cp.log_queue_lengths(s, adjust=0)
        self.collect_backend_metrics()
        return web.Response(text=REGISTRY.prometheus_text(), content_type="text/plain")

    async def stats(self, request):
        self.collect_backend_metrics()
        return web.json_response({"control_plane": self.cp.stats(), "metrics": REGISTRY.snapshot(),
                                  "backends": self.backend_stats()})

    def _backends(self):
        seen = []
        for r in self.routes.routes:
            if r.backend is not None and hasattr(r.backend, "submit") and r.backend not in seen:
                seen.append(r.backend)
        return seen

    def backend_stats(self) -> dict:
        out = {}
        for be in self._backends():
            st = getattr(getattr(be, "worker", None), "stats", None)
            if callable(st):
                out[be.path] = st()
        return out

    def collect_backend_metrics(self) -> None:
        """Per-GPU gauges from the worker pools' heartbeats (survey §5.5): HBM used/total, GPU busy ms,
        images, batches, in-flight batches, GFX clock and board power; the batch-size histogram comes from the
        native scheduler."""
        for path, st in self.backend_stats().items():
            for w in st.get("workers", []):
                tag = f"{path}/gpu{w.get('rank')}"
                for k in ("hbm_used", "hbm_total", "gpu_busy_ms", "images", "batches", "outstanding",
                          "failed_items", "retried_items", "xgmi_tx_bytes", "xgmi_rx_bytes", "gfx_mhz", "power_w"):
                    if k in w:
                        REGISTRY.gauge(f"{k}{tag}").set(float(w[k]))
            for i, c in enumerate(st.get("batch_histogram", [])):
                REGISTRY.gauge(f"batch_size_le_{1 << i}{path}").set(float(c))
            for k, v in (st.get("xgmi") or {}).items():
                REGISTRY.gauge(f"xgmi_{k}{path}").set(float(v))

    async def task_get(self, request):
        code, body = self.cp.get(request.match_info["taskId"])
        if code != 200:
            return web.Response(status=code)
        return web.Response(text=body, content_type="application/json")

    def _backend_for_task(self, tid: str):
        rec = self.cp.get_dict(tid)
        if rec is None:
            return None, None
        for be in self._backends():
            paths = getattr(be, "paths", None) or [getattr(be, "path", None)]
            if rec["EndpointPath"] in paths or getattr(be, "endpoint", None) == rec["Endpoint"]:
                return rec, be
        return rec, None

    async def task_result(self, request):
        tid = request.match_info["taskId"]
        rec, be = self._backend_for_task(tid)
        if be is not None:
            out = await asyncio.get_running_loop().run_in_executor(None, be.result, tid)
            if out is not None:
                return web.json_response({"TaskId": tid, "Result": out})
        return web.Response(status=204)

    async def task_trace(self, request):
        tid = request.match_info["taskId"]
        tr = self.cp.store.trace(tid)
        if tr is None:
            return web.Response(status=204)
        out = dict(tr, **StageClock.from_trace(tr).to_dict())
        out.update(b3_unpack(tr.get("trace", "")))
        return web.json_response(out)

    async def cache_upsert(self, request):
        code, body = self.cp.upsert(await request.read())
        return web.Response(status=code, text=body or None, content_type="application/json" if body else None)

    async def cache_get(self, request):
        code, body = self.cp.get(request.query.get("taskId", ""))
        if code != 200:
            return web.Response(status=code)
        return web.Response(text=body, content_type="application/json")

    async def requests_upsert(self, request):
        code, val = self.cp.current_processing_upsert(await request.read())
        return web.Response(status=code)

    async def requests_get(self, request):
        d = json.loads(await request.read() or b"{}")
        code, val = self.cp.current_processing_get(str(d.get("ServiceCluster", "")), str(d.get("ApiPath", "")))
        return web.Response(status=code, text=None if val is None else str(val))

    async def backend_webhook(self, request):
        if self.webhook is None:
            return web.Response(status=404)
        events = json.loads(await request.read() or b"[]")
        if isinstance(events, dict):
            events = [events]
        for ev in events:  # BackendWebhook.cs: "We should only have 1 event"
            code, payload = await asyncio.get_running_loop().run_in_executor(None, self.webhook.handle_event, ev)
            return web.json_response(payload, status=code) if payload is not None else web.Response(status=code)
        return web.Response(status=200)

    # ------------------------------------------------------------------ API routes
    def _admit(self, route: Route, request) -> Optional[web.Response]:
        if self.is_terminating:
            return web.json_response({"message": "Service is terminating, please try again later."}, status=503)
        if route.max_concurrent is not None and route.inflight + 1 > route.max_concurrent:
            return web.json_response({"message": "Service is busy, please try again later."}, status=429)
        if route.content_types and request.content_type not in route.content_types:
            return web.json_response({"message": f"Content-type must be {route.content_types}"}, status=401)
        limit = min(route.max_content_length or MAX_BODY, MAX_BODY)
        if (request.content_length or 0) > limit:  # declared length: answered before any of the body is read
            return web.json_response({"message": f"Request content too large ({request.content_length}). Must be "
                                                 f"smaller than: {limit}"}, status=413)
        return None

    async def dispatch(self, request):
        route = self.routes.match(request.path)
        if route is None or request.method not in ("POST", "PUT", "GET"):
            return web.Response(status=404)
        self._c_req.inc()
        rej = self._admit(route, request)
        if rej is not None:
            return rej
        route.inflight += 1
        try:
            if (route.mode == "async" and request.content_type == BATCH_CONTENT_TYPE and request.content_length
                    and hasattr(route.backend, "begin_stream_batch")):
                return await self._async_stream_batch(route, request)
            body = await request.read()
            if route.mode == "async":
                return await self._async(route, request, body)
            return await self._sync(route, request, body)
        finally:
            route.inflight -= 1

    @staticmethod
    def _payload_error(e: Exception) -> Optional[web.Response]:
        from ..runtime.model_endpoint import PayloadError

        if isinstance(e, PayloadError):
            return web.json_response({"message": str(e)}, status=getattr(e, "status", 400))
        return None

    async def _async_stream_batch(self, route: Route, request):
        """Binary batch ingest: the body streams chunk by chunk into ring slots (no buffered copy)."""
        b3 = b3_from_headers(request.headers)
        sb = None
        try:
            sb = route.backend.begin_stream_batch(request.content_length, b3_pack(b3))
            if not sb.try_alloc():
                await asyncio.get_running_loop().run_in_executor(None, sb.alloc)
            async for chunk in request.content.iter_any():
                sb.feed(chunk)
            ids = sb.finish()
        except Exception as e:
            if sb is not None:
                sb.abort()
            rej = self._payload_error(e)
            if rej is not None:
                return rej
            self.cp.log.log_error(f"{TASK_INSERT_FAILED} {e}", request.path)
            return web.Response(status=500, text=TASK_INSERT_FAILED)
        return web.json_response({"TaskIds": ids}, headers=b3)

    async def _async(self, route: Route, request, body: bytes):
        loop = asyncio.get_running_loop()
        target = route.target_path(request.path)
        upstream_id = request.headers.get("taskId", "")
        if upstream_id and not valid_task_id(upstream_id):
            return web.json_response({"message": "taskId header must be 1-128 printable ASCII characters"}, status=400)
        b3 = b3_from_headers(request.headers)
        trace = b3_pack(b3)
        try:
            if hasattr(route.backend, "submit"):
                if request.content_type == BATCH_CONTENT_TYPE:
                    ids = await loop.run_in_executor(None, route.backend.submit_raw_batch, body, trace)
                    return web.json_response({"TaskIds": ids}, headers=b3)
                js = await loop.run_in_executor(
                    None, lambda: route.backend.submit(body, request.content_type, upstream_id, None, trace))
            else:
                js = await loop.run_in_executor(None, self.cp.create_async_task, self.base_url + target,
                                                body.decode("utf-8", "replace"))
                self.cp.store.set_trace(json.loads(js)["TaskId"], trace)
        except Exception as e:
            rej = self._payload_error(e)
            if rej is not None:
                return rej
            self.cp.log.log_error(f"{TASK_INSERT_FAILED} {e}", request.path)
            return web.Response(status=500, text=TASK_INSERT_FAILED)
        if "application/json" in request.headers.get("Accept", "application/json") or "*/*" in request.headers.get(
                "Accept", ""):
            return web.Response(text=js, content_type="application/json", headers=b3)
        return web.Response(text="TaskId: " + json.loads(js)["TaskId"], headers=b3)

    async def _sync(self, route: Route, request, body: bytes):
        loop = asyncio.get_running_loop()
        be = route.backend
        if hasattr(be, "submit"):
            fut = loop.create_future()

            def done(tid, _f=fut):
                loop.call_soon_threadsafe(lambda: _f.done() or _f.set_result(tid))

            trace = b3_pack(b3_from_headers(request.headers))
            try:
                js = await loop.run_in_executor(None, lambda: be.submit(body, request.content_type, "", done, trace))
            except Exception as e:
                rej = self._payload_error(e)
                if rej is not None:
                    return rej
                raise
            tid = json.loads(js)["TaskId"]
            try:
                await asyncio.wait_for(fut, timeout=self.cp.cfg.sync_timeout_s)
            except asyncio.TimeoutError:
                return web.json_response({"TaskId": tid, "message": "Task did not finish in time; poll "
                                          f"/v1/taskmanagement/task/{tid}"}, status=504)
            rec = self.cp.get_dict(tid)
            if rec is None or rec["BackendStatus"] != "completed":
                return web.json_response(rec or {"TaskId": tid, "Status": "failed"}, status=500)
            return web.json_response(be.result(tid))
        if isinstance(be, str):
            if self._session is None:
                self._session = ClientSession()
            url = be.rstrip("/") + route.target_path(request.path) if route.rewrite is not None else be
            async with self._session.post(url, data=body, headers={"Content-Type": request.content_type or
                                                                   "application/octet-stream"}) as r:
                return web.Response(status=r.status, body=await r.read(), content_type=r.content_type)
        if callable(be):
            hdrs = dict(request.headers)
            res = be("", body, hdrs) if route.inline else await loop.run_in_executor(None, be, "", body, hdrs)
            code, payload = (res if isinstance(res, tuple) else (200, res))
            if isinstance(payload, (dict, list)):
                return web.json_response(payload, status=code)
            return web.Response(status=code, body=payload if isinstance(payload, bytes) else str(payload).encode())
        return web.Response(status=502)

    async def _cleanup(self, app):
        if self._session is not None:
            await self._session.close()

    # ------------------------------------------------------------------ lifecycle
    def idle(self) -> bool:
        return all(r.inflight == 0 for r in self.routes.routes) and all(
            q.depth() == 0 and q.stats()["inflight"] == 0 for q in self.cp.queues().values())

    def install_signal_handlers(self, grace_s: float = 30.0) -> None:
        """SIGINT/SIGTERM: stop admitting (503), finish queued + in-flight work, then exit."""
        import time

        def wait_then_exit():
            deadline = time.time() + grace_s
            while time.time() < deadline and not self.idle():
                time.sleep(0.05)
            self._stopped.set()  # run() returns

        def drain(*_):
            if not self.is_terminating:
                self.is_terminating = True
                for hook in self.on_drain:  # e.g. stop the ingest front-ends so no new tasks arrive
                    try:
                        hook()
                    except Exception as e:  # draining must go on
                        self.cp.log.log_error(f"drain hook failed: {e}")
                threading.Thread(target=wait_then_exit, daemon=True).start()

        for sig in (signal.SIGINT, signal.SIGTERM):
            try:
                signal.signal(sig, drain)
            except ValueError:
                pass

    def add_public_socket(self, sock) -> bool:
        """Start serving one more listening socket (HTTPS when the gateway has a certificate) while ``run`` is
        running: the public port taken back from native front-ends that all exited (``serve.py``)."""
        serving = getattr(self, "_serving", None)
        if serving is None:
            return False
        loop, runner, ssl_context = serving
        fut = asyncio.run_coroutine_threadsafe(web.SockSite(runner, sock, ssl_context=ssl_context).start(), loop)
        fut.result(10)
        return True

    def run(self, host: str = "127.0.0.1", port: int = 8080, socks=None, ssl_context=None,
            internal_only: bool = False) -> None:
        """Serve on (host, port), or on the given listening sockets (public SO_REUSEPORT socket shared with
        the ingest front-ends + the internal socket they proxy to: serve.open_listeners), until the drain
        (install_signal_handlers) has finished. ``ssl_context`` (default: from the config's TLS cert/key) makes the
        public listener HTTPS; the front-ends' internal loopback listener (the second socket) stays plain HTTP.
        ``internal_only``: ``socks`` is just that internal listener (native front-ends own the public port)."""
        if ssl_context is None:
            ssl_context = server_ssl_context(self.cp.cfg.tls_cert, self.cp.cfg.tls_key)

        async def serve():
            # the drain already waited for in-flight work: do not hold the exit on idle keep-alive connections
            # (e.g. the front-ends' proxy sessions) for aiohttp's default 60 s
            runner = web.AppRunner(self.app, handle_signals=False, access_log=None, shutdown_timeout=2.0)
            await runner.setup()
            self._serving = (asyncio.get_running_loop(), runner, ssl_context)  # (add_public_socket)
            if socks:
                sites = [web.SockSite(runner, sk, ssl_context=ssl_context if i == 0 and not internal_only else None)
                         for i, sk in enumerate(socks)]
            else:
                sites = [web.TCPSite(runner, host, port, ssl_context=ssl_context)]
            for site in sites:
                await site.start()
            try:
                while not self._stopped.is_set():
                    await asyncio.sleep(0.1)
            finally:
                await runner.cleanup()

        try:
            asyncio.run(serve())
        except KeyboardInterrupt:
            pass
