"""Platform launcher: one command replaces the reference's deployment pipeline.

``InfrastructureDeployment/deploy_infrastructure.sh:5-39`` provisions APIM, AKS + GPU node pools,
Istio, Redis, Service Bus / Event Grid and five Function apps, then every API is a Helm release +
VirtualService + APIM API. Here a single YAML file (``examples/platform.yaml``) declares the model
endpoints (factory, input shape, batch, GPUs, in-process engine or per-GPU worker pool) and the
route table, and::

    python -m aiforearth_api_platform_amd.serve --config examples/platform.yaml [--port 8080]

brings up the control plane, the GPU workers, the dispatchers and the HTTP gateway in one process
tree. Env/flags precedence follows :mod:`config` (CLI > env > YAML > defaults).
"""
from __future__ import annotations

import argparse
import importlib
import logging
import os
import sys
import threading
import time
from typing import Any, Dict

import torch
import yaml

from .config import Config, bucket_list, set_config
from .gateway.control import ControlPlane, set_control_plane
from .gateway.security import parse_keys
from .gateway.server import Gateway, Route, RouteTable
from .sched.dispatcher import QueueDispatcher, WebhookDispatcher, http_backend
from .utils.logging import AI4ELogger


def _load(path: str):
    mod, fn = path.split(":")
    return getattr(importlib.import_module(mod), fn)


def _devices(spec) -> list:
    if spec in (None, "all"):
        n = torch.cuda.device_count() if torch.cuda.is_available() else 0
        return [f"cuda:{i}" for i in range(n)] or ["cpu"]
    return list(spec)


from .runtime.frontend import open_listeners  # noqa: E402  (re-exported for the CLI)


def frontend_count(cfg: Config) -> int:
    """Ingest front-end processes to run. With a task journal, the payloads they ingest stay durable in the
    crash-surviving ring of each pool endpoint (runtime/durable_ring.py)."""
    return max(0, int(cfg.frontend_processes))


def start_frontends(cfg: Config, doc: Dict[str, Any], endpoints: Dict[str, Any], port: int, internal_port: int):
    """Spawn the ingest front-end processes for the platform's pool endpoints: native (runtime/native_frontend.py,
    the default) or Python (runtime/frontend.py; always with TLS)."""
    from .runtime.frontend import spawn_frontends

    # image endpoints only: requests of endpoints with their own decoder (extent records) go to the gateway
    pools = {name: ep for name, ep in endpoints.items() if getattr(ep, "is_pool", False)
             and not getattr(ep, "custom_decode", False)}
    routes = []
    for r in doc.get("routes") or []:
        be = r.get("backend")
        name = be.split(":", 1)[1] if isinstance(be, str) and be.startswith("inproc:") else None
        routes.append({"prefix": r["prefix"], "rewrite": r.get("rewrite"), "mode": r.get("mode", "async"),
                       "endpoint": name if name in pools else None, "content_types": r.get("content_types"),
                       "max_content_length": r.get("max_content_length"), "max_concurrent": r.get("max_concurrent"),
                       "keys": parse_keys(r.get("keys"))})
    security = {"keys": parse_keys(cfg.subscription_keys), "tls_cert": cfg.tls_cert, "tls_key": cfg.tls_key}
    if cfg.frontend_impl == "native":  # (TLS terminated in the native front-ends too)
        from .runtime.native_frontend import spawn_native_frontends

        return spawn_native_frontends(frontend_count(cfg), pools, routes, cfg.host, port,
                                      f"http://127.0.0.1:{internal_port}", security=security,
                                      max_queue_ms=cfg.max_queue_ms)
    return spawn_frontends(frontend_count(cfg), pools, routes, cfg.host, port, f"http://127.0.0.1:{internal_port}",
                           security=security)


def _public_port_watchdog(gw, frontends, host: str, port: int, period_s: float = 1.0) -> None:
    """Native front-ends own the public port (``handover_public_port``). If every one of them exits while the
    gateway is not draining, the serving process binds the port again and serves it itself (the gateway path: the
    same routes and admission rules, without the native ingest), so the service stays reachable."""
    while not gw.is_terminating:
        time.sleep(period_s)
        if gw.is_terminating or any(p.is_alive() for p in frontends):
            continue
        pub, internal = open_listeners(host, port, shared=True)
        internal.close()
        sock = pub
        if gw.add_public_socket(sock):
            print(f"ai4e-mi355x: every ingest front-end exited; the gateway serves {host}:{port} itself",
                  file=sys.stderr, flush=True)
        else:
            sock.close()
        return


def _request_decoder(e: Dict[str, Any]):
    """Endpoints whose requests are not images: ``request: extent`` = land-cover classifybyextent /
    tilebyextent (``extent_op: classify | tile``), JSON extents encoded into 64-byte records (runtime/extent.py)."""
    if e.get("request") != "extent":
        return None
    from .runtime.extent import OP_CLASSIFY, OP_TILE, MosaicSpec, request_decoder

    kw = e.get("kwargs") or {}
    return request_decoder(MosaicSpec.parse(kw.get("mosaics") or {}), OP_TILE if e.get("extent_op") == "tile"
                           else OP_CLASSIFY, tuple(kw.get("max_extent", (2048, 2048))), int(kw.get("tile", 512)),
                           int(kw.get("stride", 448)))


def control_plane_shards(cfg: Config, e: Dict[str, Any], spec, devs) -> int:
    """Scheduler shards of a pool endpoint: the YAML's ``control_plane_shards``, else the config's, where 0 means
    one per GPU (worker group); stage-graph pools (several leaders per group) keep one scheduler."""
    groups = max(1, len(devs) // max(1, spec.group_size))
    if spec.group_leaders > 1 or spec.stage_endpoints:
        return 1
    n = int(e.get("control_plane_shards", cfg.control_plane_shards))
    return max(1, min(groups, n if n > 0 else groups, 8))


def build_platform(doc: Dict[str, Any], cfg: Config):
    """Build (control_plane, gateway, endpoints, dispatchers) from a platform YAML document."""
    from .runtime.engine import InferenceEngine, PayloadRing
    from .runtime.model_endpoint import ModelEndpoint
    from .runtime.servable import as_servable
    from .runtime.serving import GpuBatchWorker
    from .runtime.worker_pool import ModelSpec, ShardedWorkerPool, WorkerPool

    cp = ControlPlane(cfg, AI4ELogger(level=logging.DEBUG if cfg.debug else logging.INFO))
    set_control_plane(cp)
    base_url = f"{'https' if cfg.tls_cert else 'http'}://{cfg.host}:{cfg.port}"
    endpoints: Dict[str, Any] = {}
    for name, e in (doc.get("endpoints") or {}).items():
        shape = tuple(e["item_shape"])
        mb = int(e.get("max_batch", cfg.max_batch))
        devs = _devices(e.get("devices", "all"))
        buckets = bucket_list(e.get("batch_buckets", cfg.batch_buckets), mb)
        graphs = bool(e.get("hip_graphs", cfg.use_hip_graphs))
        if e.get("mode", "pool") == "pool":
            spec = ModelSpec(e["factory"], shape, mb, int(e.get("topk", 5)), dict(e.get("kwargs") or {}), graphs,
                             tuple(buckets), tuple(base_url + p for p in e.get("stage_paths", [])),
                             int(e.get("group_size", 1)), int(e.get("group_leaders", 1)))
            kw = dict(max_delay_s=cfg.max_batch_delay_ms / 1e3, heartbeat_interval_s=cfg.heartbeat_interval_s,
                      heartbeat_timeout_s=cfg.heartbeat_timeout_s, ring_slots=int(e.get("ring_slots", 0)),
                      frontends=frontend_count(cfg),
                      frontend_slots=int(e.get("frontend_ring_slots", cfg.frontend_ring_slots)))
            nshards = control_plane_shards(cfg, e, spec, devs)
            if cfg.journal_path:  # payloads survive a crash in the ring itself (any ingest path)
                from .runtime.durable_ring import DurableRing

                kw["durable"] = DurableRing(cfg.journal_path, e["path"])
            # the control plane scales with the GPUs: one scheduler shard per GPU (worker group) by default
            pool = (ShardedWorkerPool(cp, base_url + e["path"], spec, devs, shards=nshards, **kw) if nshards > 1
                    else WorkerPool(cp, base_url + e["path"], spec, devs, **kw))
            decode = _request_decoder(e)
            ep = ModelEndpoint(cp, e["path"], worker=pool, base_url=base_url, decode=decode,
                               decode_processes=0 if decode else int(e.get("decode_processes", cfg.decode_processes)))
        else:
            dev = torch.device(devs[0])
            servable = as_servable(_load(e["factory"])(device=str(dev), **(e.get("kwargs") or {})),
                                   int(e.get("topk", 5)))
            eng = InferenceEngine(None, shape, mb, device=dev, use_graphs=graphs, buckets=buckets,
                                  output_fn=servable, timing=dev.type == "cuda")
            eng.warmup()
            ring = PayloadRing(int(e.get("ring_slots", 0)) or mb * 4, shape)
            worker = GpuBatchWorker(cp, base_url + e["path"], eng, ring, kind=servable.kind, outputs=servable.outputs)
            ep = ModelEndpoint(cp, e["path"], worker=worker, base_url=base_url)
        endpoints[name] = ep
    table = RouteTable()
    dispatchers = []
    backends: Dict[str, Any] = {}
    for r in doc.get("routes") or []:
        be = r.get("backend")
        if isinstance(be, str) and be.startswith("inproc:"):
            be = endpoints[be.split(":", 1)[1]]
        elif isinstance(be, str) and be.startswith("callable:"):
            be = _load(be.split(":", 1)[1])
        route = table.add(Route(prefix=r["prefix"], mode=r.get("mode", "async"), backend=be, rewrite=r.get("rewrite"),
                                max_concurrent=r.get("max_concurrent"), content_types=r.get("content_types"),
                                max_content_length=r.get("max_content_length"), inline=bool(r.get("inline", False)),
                                keys=parse_keys(r.get("keys")) or None))
        # async route to a generic backend: a queue dispatcher delivers each task (BackendQueueProcessor)
        if route.mode == "async" and not hasattr(be, "submit") and be is not None:
            target = base_url + (route.rewrite or route.prefix)
            fn = http_backend(be) if isinstance(be, str) else be
            backends[target] = fn
            if cfg.transport != "eventgrid":
                dispatchers.append(QueueDispatcher(cp, target, fn))
    webhook = WebhookDispatcher(cp, backends)
    if cfg.transport == "eventgrid":
        cp.push_transport = webhook.deliver
    gw = Gateway(cp, table, webhook=webhook, base_url=base_url)
    return cp, gw, endpoints, dispatchers


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="AI4E MI355X serving platform")
    ap.add_argument("--config", required=True, help="platform YAML (endpoints + routes + settings)")
    ap.add_argument("--host")
    ap.add_argument("--port", type=int)
    ap.add_argument("--transport", choices=["inproc", "queue", "eventgrid"])
    args = ap.parse_args(argv)
    with open(args.config) as f:
        doc = yaml.safe_load(f) or {}
    settings = dict(doc.get("settings") or {})
    cfg = Config.load(env=os.environ, yaml_values=settings, host=args.host, port=args.port,
                      transport=args.transport)
    set_config(cfg)
    cp, gw, endpoints, dispatchers = build_platform(doc, cfg)
    for ep in endpoints.values():  # (workers first: a recovery larger than the ring drains while it re-ingests)
        ep.start()
    if cfg.journal_path and os.path.exists(cfg.journal_path):
        print(f"recovered from journal: {cp.recover(cfg.journal_path)}", file=sys.stderr, flush=True)
    for ep in endpoints.values():
        if hasattr(ep, "finish_recovery"):
            ep.finish_recovery()
    for d in dispatchers:
        d.start()
    cp.start_metric_timers()
    scalers = []
    if cfg.autoscale:
        from .runtime.autoscale import QueueDepthAutoscaler

        for ep in endpoints.values():
            if getattr(ep, "is_pool", False):
                scalers.append(QueueDepthAutoscaler(ep.worker, min_workers=cfg.autoscale_min_workers,
                                                    target_per_worker=cfg.autoscale_target_per_worker,
                                                    period_s=cfg.autoscale_period_s).start())
    gw.install_signal_handlers()
    nfe = frontend_count(cfg)
    socks = open_listeners(cfg.host, cfg.port, shared=nfe > 0)
    frontends = start_frontends(cfg, doc, endpoints, cfg.port, socks[1].getsockname()[1]) if nfe else []
    # native front-ends own the public port once they listen (admission on every public connection)
    from .runtime.native_frontend import handover_public_port

    n_socks = len(socks)
    socks = handover_public_port(socks, frontends)
    if len(socks) < n_socks:  # the front-ends own the public port: take it back if every one of them exits
        threading.Thread(target=_public_port_watchdog, args=(gw, frontends, cfg.host, cfg.port), daemon=True).start()
    # SIGTERM drain: the front-ends stop first (their own graceful shutdown), so no new tasks arrive meanwhile
    gw.on_drain.append(lambda: [p.terminate() for p in frontends])
    print(f"ai4e-mi355x gateway on {'https' if cfg.tls_cert else 'http'}://{cfg.host}:{cfg.port} endpoints={list(endpoints)} "
          f"ingest_frontends={len(frontends)}", file=sys.stderr, flush=True)
    try:
        gw.run(cfg.host, cfg.port, socks=socks, internal_only=len(socks) < n_socks)
    finally:
        for p in frontends:
            p.terminate()
        for sc in scalers:
            sc.stop()
        for d in dispatchers:
            d.stop()
        for ep in endpoints.values():
            ep.stop()
        cp.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
