"""Ingest front-end processes: the gateway's request ingest spread over several processes.

One Python process tops out at a few thousand requests/s of HTTP parsing + payload decoding (the GIL),
far below what the GPUs of a node consume. With ``frontend_processes: N`` the serving process
(:mod:`serve`) spawns N front-ends that listen on the public port beside it (``SO_REUSEPORT``: the
kernel spreads connections over all listeners). A front-end handles the async POSTs of the GPU
endpoints itself:

* the payload is decoded (or, for the binary batch type, streamed) straight into a slot of the
  front-end's own partition of the endpoint's shared payload ring;
* it mints the task id(s), hands slots + ids to the node scheduler over its connection (SUBMIT_IDS,
  acknowledged once the tasks exist) and answers the client — the same JSON the gateway answers;
* slots come back (FREE) when the tasks finish.

Everything else (task status / result / trace queries, sync routes, metrics, generic backends, and async
requests that carry an upstream ``taskId`` header, which the gateway adopts as the reference's
``TaskManager.AddTask`` does) is proxied to the serving process's internal listener, where the task store lives.

Admission matches the gateway's (``gateway/server.py``): subscription keys (401), the route's
``max_concurrent`` per process (429), draining after SIGTERM (503), content type (401) and length (413); the
listener is HTTPS when the platform has a TLS certificate. When the scheduler's acknowledgement does not come in
time the tasks may already exist, so the minted ids are returned with 202 (not a 503 that invites a duplicate
retry). The reference scales
its front door with APIM + Istio in front of one Flask container per model
(``APIs/1.0/base-py/ai4e_service.py``); here the ingest path itself scales across cores.
"""
from __future__ import annotations

import asyncio
import json
import time
from typing import Dict, List, Optional

BATCH_CONTENT_TYPE = "application/x-ai4e-batch"
_HOP = {"connection", "keep-alive", "proxy-authenticate", "proxy-authorization", "te", "trailers",
        "transfer-encoding", "upgrade", "host", "content-length"}


def frontend_main(index: int, host: str, port: int, internal_url: str, endpoints: Dict[str, dict],
                  routes: List[dict], conns: Dict[str, object], ack_timeout_s: float = 30.0,
                  security: Optional[dict] = None) -> None:
    """Process entry point. ``endpoints``: name -> {endpoint, shm, nslots, item_shape, base, len};
    ``routes``: [{prefix, rewrite, mode, endpoint (name or None), content_types, max_content_length,
    max_concurrent, keys}]; ``conns``: name -> the Connection to that endpoint's node scheduler;
    ``security``: {keys (global subscription keys), tls_cert, tls_key}."""
    import signal

    from aiohttp import ClientSession, web

    from ..gateway.security import KeyAuth, server_ssl_context

    from ..store.pystore import absolute_path, dotnet_timestamp
    from ..utils.tracing import b3_from_headers, b3_pack
    from .decode import PayloadError, decode_image
    import numpy as np

    from .jpeg_gpu import JPEG_TYPES, prepare_into_slot
    from .ingest import IngestShard

    import os

    # the serving process owns the store and the rings: when its connection closes, this process has nothing
    # left to serve (and must not outlive it as an orphan holding the port)
    shards = {name: IngestShard(conns[name], e["endpoint"], e["shm"], e["nslots"], e["item_shape"], e["base"],
                                e["len"], on_close=lambda: os._exit(0), digits=e.get("digits"))
              for name, e in endpoints.items()}
    # endpoint name -> its control-plane shards ("name", "name#1", ...: one per scheduler shard of a sharded pool)
    groups: Dict[str, List[IngestShard]] = {}
    for name in endpoints:
        groups.setdefault(name.split("#", 1)[0], []).append(shards[name])
    rr = [0]

    def pick(group: List[IngestShard]) -> IngestShard:  # least-loaded partition, ties round-robin
        rr[0] += 1
        k = len(group)
        return min((group[(rr[0] + i) % k] for i in range(k)), key=lambda sh: sh.slots.used() / max(1, sh.part_len))
    table = sorted(routes, key=lambda r: -len(r["prefix"]))
    state: Dict[str, object] = {"session": None, "draining": False}
    sec = security or {}
    auth = KeyAuth(sec.get("keys") or [])
    inflight: Dict[str, int] = {}

    def on_term(*_):  # drain: refuse new ingest (503), let in-flight requests finish, then exit
        state["draining"] = True
        import threading

        threading.Timer(5.0, lambda: os._exit(0)).start()

    signal.signal(signal.SIGTERM, on_term)

    def match(path: str) -> Optional[dict]:
        for r in table:
            if path == r["prefix"] or path.startswith(r["prefix"].rstrip("/") + "/"):
                return r
        return None

    def task_json(tid: str, endpoint: str) -> str:
        return json.dumps({"TaskId": tid, "Timestamp": dotnet_timestamp(time.time()), "Status": "created",
                           "BackendStatus": "created", "Endpoint": endpoint, "Body": None, "PublishToGrid": True,
                           "EndpointPath": absolute_path(endpoint)}, separators=(",", ":"))

    async def proxy(request):
        if state["session"] is None:
            state["session"] = ClientSession()
        headers = {k: v for k, v in request.headers.items() if k.lower() not in _HOP}
        body = await request.read()
        async with state["session"].request(request.method, internal_url + request.path_qs, data=body or None,
                                            headers=headers, allow_redirects=False) as r:
            data = await r.read()
            out = {k: v for k, v in r.headers.items() if k.lower() not in _HOP and k.lower() != "content-encoding"}
            return web.Response(status=r.status, body=data, headers=out)

    async def ingest(request, route: dict, shard: IngestShard):
        if state["draining"]:
            return web.json_response({"message": "Service is terminating, please try again later."}, status=503)
        mc = route.get("max_concurrent")
        if mc is not None and inflight.get(route["prefix"], 0) + 1 > mc:
            return web.json_response({"message": "Service is busy, please try again later."}, status=429)
        inflight[route["prefix"]] = inflight.get(route["prefix"], 0) + 1
        try:
            return await _ingest(request, route, shard)
        finally:
            inflight[route["prefix"]] -= 1

    async def _ingest(request, route: dict, shard: IngestShard):
        if route.get("content_types") and request.content_type not in route["content_types"]:
            return web.json_response({"message": f"Content-type must be {route['content_types']}"}, status=401)
        mcl = route.get("max_content_length")
        if mcl and (request.content_length or 0) > mcl:
            return web.json_response({"message": f"Request content too large ({request.content_length}). Must be "
                                                 f"smaller than: {mcl}"}, status=413)
        b3 = b3_from_headers(request.headers)
        trace = b3_pack(b3)
        loop = asyncio.get_running_loop()
        try:
            if request.content_type == BATCH_CONTENT_TYPE and request.content_length:
                sb = _begin(shard, request.content_length, trace)
                try:
                    if not sb.try_alloc():
                        await loop.run_in_executor(None, sb.alloc)
                    async for chunk in request.content.iter_any():
                        sb.feed(chunk)
                    slots = sb.take_slots()
                except BaseException:
                    sb.abort()
                    raise
                ids = shard.mint_ids(len(slots))
                try:
                    await shard.submit_ids(slots, ids, trace).wait_async(ack_timeout_s)
                except (TimeoutError, asyncio.TimeoutError):  # submitted, not yet acknowledged: do not invite a retry
                    return web.json_response({"TaskIds": ids, "message": "accepted, not yet acknowledged"},
                                             status=202, headers=b3)
                return web.json_response({"TaskIds": ids}, headers=b3)
            body = await request.read()
            if shard.jpeg_key and request.content_type in JPEG_TYPES:
                # prepared into the slot for the worker's GPU decode (runtime/jpeg_gpu.py); else decoded here
                slot = shard.slots.alloc(1, 0.0) or await loop.run_in_executor(None, shard.alloc, 1)
                try:
                    addr = shard.buf[slot[0]].ctypes.data
                    item = int(np.prod(shard.item_shape))
                    if not await loop.run_in_executor(None, prepare_into_slot, body, addr, item, shard.item_shape,
                                                      shard.jpeg_key):
                        arr = await loop.run_in_executor(None, decode_image, body, request.content_type,
                                                         shard.item_shape)
                        shard.write(slot[0], arr)
                except BaseException:
                    shard.free(slot)
                    raise
            else:
                arr = await loop.run_in_executor(None, decode_image, body, request.content_type, shard.item_shape)
                slot = shard.slots.alloc(1, 0.0) or await loop.run_in_executor(None, shard.alloc, 1)
                shard.write(slot[0], arr)
            tid = shard.mint_ids(1)[0]
            try:
                n = await shard.submit_ids(slot, [tid], trace).wait_async(ack_timeout_s)
            except (TimeoutError, asyncio.TimeoutError):
                return web.Response(text=task_json(tid, shard.endpoint), status=202, content_type="application/json",
                                    headers=b3)
            if n != 1:  # (minted ids are unique: only a scheduler that refused the payload gets here)
                return web.json_response({"message": "Task insert failed."}, status=500)
        except PayloadError as e:
            return web.json_response({"message": str(e)}, status=e.status)
        except (TimeoutError, asyncio.TimeoutError):  # no ring slot in time: nothing was created
            return web.json_response({"message": "Service is busy, please try again later."}, status=429)
        js = task_json(tid, shard.endpoint)
        accept = request.headers.get("Accept", "application/json")
        if "application/json" in accept or "*/*" in accept:
            return web.Response(text=js, content_type="application/json", headers=b3)
        return web.Response(text="TaskId: " + tid, headers=b3)

    async def handle(request):
        r = match(request.path)
        # route-less paths (task management, control routes) are proxied: the serving process's key policy decides
        if request.path not in ("/", "/openapi.json") and r is not None:
            rej = auth.check(request.headers, request.query, r.get("keys") if r is not None else None)
            if rej is not None:
                return web.json_response(rej[1], status=rej[0])
        if (r is not None and r["mode"] == "async" and r.get("endpoint") in groups and request.method in ("POST", "PUT")
                and not request.headers.get("taskId")):
            return await ingest(request, r, pick(groups[r["endpoint"]]))
        return await proxy(request)

    app = web.Application(client_max_size=1 << 30)
    app.router.add_route("*", "/{tail:.*}", handle)

    async def close_session(_app):
        if state["session"] is not None:
            await state["session"].close()

    app.on_cleanup.append(close_session)
    try:
        web.run_app(app, host=host, port=port, reuse_port=True, access_log=None, print=None, handle_signals=False,
                    ssl_context=server_ssl_context(sec.get("tls_cert", ""), sec.get("tls_key", "")))
    finally:
        for s in shards.values():
            s.close()


def open_listeners(host: str, port: int, shared: bool) -> list:
    """The serving process's listening sockets: the public one (SO_REUSEPORT when front-ends share it) and,
    with front-ends, an internal loopback one they proxy non-ingest requests to."""
    import socket

    pub = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    pub.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    if shared:
        pub.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    pub.bind((host, port))
    pub.listen(1024)
    socks = [pub]
    if shared:
        internal = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        internal.bind(("127.0.0.1", 0))
        internal.listen(1024)
        socks.append(internal)
    return socks


def spawn_frontends(n: int, pools: Dict[str, object], routes: List[dict], host: str, port: int,
                    internal_url: str, security: Optional[dict] = None) -> list:
    """Start ``n`` front-end processes on (host, port) for the pool-backed ``ModelEndpoint``s in ``pools``
    (name -> endpoint; each WorkerPool built with ``frontends >= n``), attached to every endpoint's node
    scheduler over their own connection. ``routes``: as :func:`frontend_main`."""
    import multiprocessing as mp

    if not n or not pools:
        return []
    ctx = mp.get_context("spawn")
    procs = []
    for i in range(n):
        eps, conns = {}, {}
        for name, ep in pools.items():
            for k, pool in enumerate(getattr(ep.worker, "control_shards", [ep.worker])):
                base, length, rank = pool.frontend_partitions[i]
                parent, child = ctx.Pipe(duplex=True)
                pool.attach_ingest(rank, parent)
                key = name if k == 0 else f"{name}#{k}"
                conns[key] = child
                eps[key] = {"endpoint": ep.endpoint, "shm": ep.ring.name, "nslots": ep.ring.nslots,
                            "item_shape": list(ep.item_shape), "base": base, "len": length,
                            "digits": pool.mint_digits() if hasattr(pool, "mint_digits") else None}
        p = ctx.Process(target=frontend_main, args=(i, host, port, internal_url, eps, routes, conns),
                        kwargs={"security": security}, daemon=True, name=f"ai4e-frontend-{i}")
        p.start()
        for c in conns.values():
            c.close()
        procs.append(p)
    return procs


def _item(shard) -> int:
    n = 1
    for v in shard.item_shape:
        n *= int(v)
    return n


def _begin(shard, nbytes: int, trace: str):
    from .decode import PayloadError
    from .ingest import StreamedBatch

    item = _item(shard)
    if nbytes <= 0 or nbytes % item:
        raise PayloadError(f"batch payload must be a multiple of {item} bytes (uint8 {shard.item_shape})")
    n = nbytes // item
    if n > shard.part_len:  # could never be allocated from this front-end's ring partition
        raise PayloadError(f"batch of {n} items exceeds the ingest partition ({shard.part_len} slots)", 413)
    return StreamedBatch(shard, n, item, trace)
