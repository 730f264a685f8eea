"""Node serving benchmark harness (library): drives an endpoint through the production path.

Used by ``bench.py`` (the headline ResNet-50 API) and ``bench/api_bench.py`` (detector, land-cover,
ensemble): a node scheduler (native task store + dispatch queue + NodeScheduler) and ONE GPU worker
process per GPU. N = 1: the calling process is the scheduler and spawns the worker for cuda:0.

N > 1 (torchrun, one rank per GPU), three control-plane layouts:

* ``serve`` (default; AI4E_BENCH_CP=serve): the shipped server's topology (serve.py -> ShardedWorkerPool): rank 0 hosts
  the whole control plane — one task store, and one control-plane SHARD per GPU (node scheduler threads, dispatch
  queue, ring partition, ids minted in the shard's own store lock domains) — and spawns the worker for its GPU; rank r
  attaches to shard r over TCP as that shard's GPU worker and ingests its clients' payloads into its own partition of
  the one shared ring. Nothing per task crosses shards, and no task passes through another GPU's scheduler;
* ``sharded`` (AI4E_BENCH_CP=sharded): every rank is the node scheduler of its own GPU — its own task
  store shard, dispatch queue, payload ring and spawned worker process, its own clients — the reference's replica
  DP (HPA replicas behind Istio's ROUND_ROBIN, ``APIs/Charts/templates/async-gpu/autoscaler.yaml``) with the
  control plane scaling with the GPUs instead of serializing through one process (the reference's single
  dispatch point, ``ProcessManager/BackendQueueProcessor/host.json:3-11``). The window is the UNION of the
  ranks' steady-state windows (earliest start to latest end on the host's monotonic clock), so the whole-node
  rate is a lower bound;
* ``central`` (AI4E_BENCH_CP=central): rank 0 is the one scheduler (+ spawns the worker for its GPU); ranks
  1..N-1 connect to it over TCP as the GPU workers of their devices and ingest shards of a shared ring.

Clients write their payloads into the ring inside the timed region and enqueue them (weak scaling: --batch items
per step per GPU). torch.distributed (RCCL) brackets the timed region and reduces the timings.
"""
from __future__ import annotations

import json
import os
import threading
import time
from typing import Optional, Sequence

import numpy as np
import torch

class Client:
    """Synthetic clients of one ingest shard: per submission, write --batch images into this shard's
    ring partition (one copy per contiguous slot run) and enqueue them."""

    def __init__(self, ring_buf: torch.Tensor, alloc, submit, batch: int, seed: int):
        self.buf, self.alloc, self.submit, self.batch = ring_buf, alloc, submit, batch
        g = torch.Generator().manual_seed(1234 + seed)
        self.src = torch.randint(0, 256, (2 * batch, *ring_buf.shape[1:]), dtype=torch.uint8, generator=g)
        self.k = 0

    def step(self) -> None:
        slots = self.alloc(self.batch)
        src = self.src[(self.k % 2) * self.batch:(self.k % 2 + 1) * self.batch]
        self.k += 1
        i, n = 0, len(slots)
        while i < n:
            j = i + 1
            while j < n and slots[j] == slots[j - 1] + 1:
                j += 1
            self.buf[slots[i]:slots[i] + (j - i)].copy_(src[i:j])
            i = j
        self.submit(slots)

    def run(self, steps: int) -> None:
        for _ in range(steps):
            self.step()


def http_phase(cp, pool, seconds: float, batch: int, item_shape, path: str, frontends: int = 0,
               tls: bool = False, max_queue_ms: float = 0.0, jpeg: Optional[bytes] = None,
               phases: Sequence[str] = ("batch_route", "single_image_route"), jpeg_conc: int = 32) -> dict:
    """REST ingest on this node: aiohttp gateway (this process) + binary batch route (streamed into the
    payload ring), then single-image requests. ``frontends``: ingest front-end processes sharing the port
    (native C++ ``ai4e_ingestd`` by default, AI4E_FRONTEND_IMPL=python for runtime/frontend.py; the pool needs
    as many partitions). Load: the C++ generator (runtime/http_load.py ``run_native_clients``) in separate
    processes; the record carries the client and server CPU seconds, so a reader can see which side was
    the ceiling. ``tls``: the front-ends terminate TLS (OpenSSL in ``ai4e_ingestd``, the test certificate under
    tests/fixtures) and every client connection is an HTTPS session. ``max_queue_ms`` > 0: the front-ends' latency-
    budgeted admission (429 + Retry-After past the budget; the load generator backs off and retries). ``jpeg``: a
    JPEG frame for the ``jpeg_route`` phase (single ``image/jpeg`` requests: prepared into ring slots by the native
    front-ends when the pool's workers decode on the GPU, else proxied and decoded by the serving process)."""
    import asyncio

    from aiohttp import web

    from ..gateway.server import BATCH_CONTENT_TYPE, Gateway, Route, RouteTable
    from ..utils.metrics import percentile
    from .http_load import run_clients, run_native_clients
    from .model_endpoint import ModelEndpoint

    ep = ModelEndpoint(cp, path, worker=pool)
    table = RouteTable()
    table.add(Route("/v1/bench/async", "async", ep))
    gw = Gateway(cp, table)
    ready = threading.Event()
    box = {}

    from .frontend import open_listeners, spawn_frontends

    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    socks = open_listeners("127.0.0.1", port, shared=frontends > 0)
    impl = os.environ.get("AI4E_FRONTEND_IMPL", "native")
    # native front-ends take the public port over (serve.py's handover_public_port): the gateway serves only its
    # internal listener, the one the front-ends proxy to
    served = socks[1:] if frontends and impl == "native" else socks

    def serve():
        loop = asyncio.new_event_loop()
        asyncio.set_event_loop(loop)
        runner = web.AppRunner(gw.app, access_log=None)
        loop.run_until_complete(runner.setup())
        for sk in served:
            loop.run_until_complete(web.SockSite(runner, sk).start())
        box["loop"], box["runner"] = loop, runner
        ready.set()
        loop.run_forever()
        loop.run_until_complete(runner.cleanup())

    th = threading.Thread(target=serve, daemon=True)
    th.start()
    ready.wait(30)
    spawn = spawn_frontends
    if impl == "native":
        from .native_frontend import spawn_native_frontends as spawn
    sec = None
    if tls:
        if not frontends or impl != "native":
            raise ValueError("the HTTPS phase needs native front-ends (they terminate TLS)")
        fx = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests",
                          "fixtures")
        sec = {"tls_cert": os.path.join(fx, "tls_test_cert.pem"), "tls_key": os.path.join(fx, "tls_test_key.pem")}
    kw = {"max_queue_ms": max_queue_ms} if impl == "native" and max_queue_ms > 0 else {}
    fe = spawn(frontends, {"bench": ep}, [{"prefix": "/v1/bench/async", "mode": "async", "endpoint": "bench"}],
               "127.0.0.1", port, f"http://127.0.0.1:{socks[1].getsockname()[1]}", security=sec, **kw) \
        if frontends else []
    if fe:
        if impl == "native":  # (they listen already: the serving process leaves the public port to them)
            from .native_frontend import handover_public_port

            handover_public_port(socks, fe)
        else:
            time.sleep(5.0)  # they start and bind the shared port
    url = f"{'https' if tls else 'http'}://127.0.0.1:{port}/v1/bench/async"
    rng = np.random.default_rng(7)
    img = rng.integers(0, 256, tuple(item_shape), dtype=np.uint8)
    batch_body = np.broadcast_to(img, (batch, *img.shape)).tobytes()

    def wait_done(ids, timeout=60):
        deadline = time.time() + timeout
        while time.time() < deadline:
            lat = cp.store.latencies(ids)
            if len(lat) >= len(ids):
                return sorted(lat)
            time.sleep(0.01)
        return sorted(cp.store.latencies(ids))

    # load generators in their own processes (the server keeps this interpreter to itself)
    import psutil

    server_procs = [psutil.Process(os.getpid())] + [psutil.Process(p.pid) for p in fe]

    def server_cpu(split: bool = False):
        per = []
        for p in server_procs:
            try:
                c = p.cpu_times()
                per.append(c.user + c.system)
            except psutil.Error:
                per.append(0.0)
        return (per[0], sum(per[1:])) if split else sum(per)

    native = os.environ.get("AI4E_HTTP_CLIENT", "native") == "native"
    out = {}
    runs = [("batch_route", batch_body, BATCH_CONTENT_TYPE, True, 4, 4),
            ("single_image_route", img.tobytes(), "application/octet-stream", False, 4, 32)]
    if jpeg is not None:  # (a slower model: ~one budget's worth of requests in flight, 4 x jpeg_conc connections)
        runs.append(("jpeg_route", jpeg, "image/jpeg", False, 4, jpeg_conc))
    for name, body, ctype, is_batch, procs, conc in runs:
        if name not in phases:
            continue
        c0, s0 = server_cpu(), server_cpu(True)
        if native:
            res = run_native_clients(url, seconds / 2, conc, body, ctype, procs=procs)
            ids, t0, errors = res["ids"], res["t0"], res["errors"]
        else:
            ids, t0, _, errors = run_clients(url, seconds / 2, conc, body, ctype, is_batch, procs=procs)
            res = {}
        lat = wait_done(ids)
        dt = time.time() - t0
        out[name] = {"images": len(ids), "images_per_s": round(len(ids) / dt, 1), "connections": procs * conc,
                     "client_processes": procs, "client": "c++ ai4e_http_load" if native else "python aiohttp",
                     "ingest_frontends": len(fe), "frontend_impl": impl if fe else None, "errors": errors,
                     "scheme": "https" if tls else "http", "max_queue_ms": max_queue_ms if fe else None,
                     "busy_429": res.get("busy") if res else None,
                     "p50_task_latency_ms": round(percentile(lat, 50) * 1e3, 3),
                     "p99_task_latency_ms": round(percentile(lat, 99) * 1e3, 3),
                     "server_cpu_s": round(server_cpu() - c0, 3), "window_s": round(dt, 3)}
        s1 = server_cpu(True)  # where the server's CPU went: the serving process (scheduler, gateway) / front-ends
        out[name]["server_cpu_split_s"] = {"serving_process": round(s1[0] - s0[0], 3),
                                           "frontends": round(s1[1] - s0[1], 3)}
        if res:
            out[name]["client_cpu_s"] = round(res["client_cpu_s"], 3)
            rl = sorted(res.get("request_latency_ms") or [])
            if rl:  # what a client sees: first attempt -> 2xx, including 429 back-offs and retries
                out[name]["p50_request_latency_ms"] = round(percentile(rl, 50), 3)
                out[name]["p99_request_latency_ms"] = round(percentile(rl, 99), 3)
            out[name]["request_gbytes_per_s"] = round(res["bytes_sent"] / max(1e-9, res["t1"] - res["t0"]) / 1e9, 3)
        if is_batch:
            out[name]["request_images"] = batch
    for p in fe:
        p.terminate()
    for p in fe:
        p.join(10)
    box["loop"].call_soon_threadsafe(box["loop"].stop)
    th.join(10)
    return out


def run_node_bench(args, spec, path: str, metric: str, unit: str = "images/s", config: Optional[dict] = None,
                   flops_per_item: Optional[float] = None, baseline: Optional[float] = None,
                   dtype: str = "bf16") -> Optional[dict]:
    """Warm up, time exactly ``args.steps`` steps, return rank 0's JSON record (None elsewhere).

    ``args`` needs: steps, warmup, batch, inflight, device, http, http_seconds, json_out."""
    from .. import _build
    from ..config import Config
    from ..gateway.control import ControlPlane
    from ..parallel.dist import all_reduce_max, destroy, env_ranks, init_from_env, sync
    from ..utils.metrics import percentile
    from . import protocol as P
    from .hostperf import tune_gc
    from .worker_pool import WorkerPool

    endpoint = "http://127.0.0.1" + path
    hang_s = float(os.environ.get("AI4E_HANG_DUMP_S", "0"))  # diagnostic: every thread's stack after this long
    if hang_s > 0:
        import faulthandler
        import sys

        faulthandler.dump_traceback_later(hang_s, repeat=False, file=sys.stderr)
    _, world, _ = env_ranks()
    if world > 1 and args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} != WORLD_SIZE {world}")
    # worker-group forms (spec.group_size > 1: spatial segmentation, the N:M stage graph) run from ONE process:
    # the pool spawns the group's processes, one per GPU, joined over RCCL
    group = spec.group_size
    if group > 1 and world > 1:
        raise SystemExit("worker-group benches run in one process (the pool spawns one process per group GPU)")
    # rank 0 builds the in-tree HIP/C++ libraries, then everyone joins (RCCL on GPU, gloo on CPU)
    denv = init_from_env(args.device, build=_build.build_all)
    rank, device = denv.rank, denv.device
    cp_mode = os.environ.get("AI4E_BENCH_CP", "serve") if world > 1 and group == 1 else "central"
    if cp_mode not in ("serve", "sharded", "central"):
        raise SystemExit(f"AI4E_BENCH_CP={cp_mode}: serve, sharded or central")
    sharded = cp_mode == "sharded"
    served = cp_mode == "serve"
    B = args.batch
    part = B * (args.inflight + 1)  # ring slots per ingest shard
    hb = 0.5
    # completions this rank's scheduler counts: the whole node's (central) or its own shard's (sharded)
    counted_world = 1 if sharded else world
    total_images = (args.warmup + args.steps) * B * counted_world

    if rank == 0 or sharded:
        cfg = Config.load(env={}, max_batch=B, max_batch_delay_ms=0.0)
        cp = ControlPlane(cfg)
        remote = [] if sharded else [(part * r, part, r) for r in range(1, world)]
        if group > 1:
            devices = [f"cuda:{i}" for i in range(group)] if args.device == "cuda" else ["cpu"] * group
        else:
            devices = [f"{args.device}:{denv.local_rank}" if args.device == "cuda" else "cpu"]
        pkw = dict(ring_slots=part, max_delay_s=0.0005, heartbeat_interval_s=hb, heartbeat_timeout_s=120.0,
                   pipeline_depth=int(os.environ.get("AI4E_PIPELINE_DEPTH", "3")), poll_s=0.005,
                   frontends=getattr(args, "http_frontends", 0) if args.http else 0,
                   frontend_slots=3 * B)  # (REST phase only: keep the pinned ring small)
        if served:
            from .worker_pool import ShardedWorkerPool

            # shard r serves GPU r; shards 1..N-1 are served by the torchrun ranks that attach below
            pool = ShardedWorkerPool(cp, endpoint, spec, [f"{args.device}:{r}" if args.device == "cuda" else "cpu"
                                                          for r in range(world)],
                                     shards=world, remote=range(1, world), remote_slots=part, **pkw)
            remote = [pool.remote_partition(r) for r in range(1, world)]
        else:
            pool = WorkerPool(cp, endpoint, spec, devices, remote_partitions=remote, **pkw)
        info = None
        listener = None
        if world > 1 and not sharded:
            import secrets
            from multiprocessing.connection import Listener

            key = secrets.token_bytes(16)
            # backlog = every remote rank: with the default of 1, ranks that connect at once overflow the accept queue,
            # their SYNs are dropped and retried after 1, 2, 4, ... s (a 40-90 s stall, 2 in 6 world-8 runs)
            listener = Listener(("127.0.0.1", 0), authkey=key, backlog=max(1, world))
            info = {"shm": pool.ring.name, "nslots": pool.ring.nslots, "addr": listener.address, "key": key.hex(),
                    "parts": {int(rk): int(b) for b, _, rk in remote}}  # rank -> its ingest partition base
        objs = [info]
        if world > 1 and not sharded:
            import torch.distributed as dist

            dist.broadcast_object_list(objs, src=0)

            def accept():
                for _ in range(world - 1):
                    c = listener.accept()
                    r = int(c.recv_bytes().decode())
                    (pool.control_shards[r] if served else pool).attach_remote(r, c, device=f"cuda:{r}")

            acc = threading.Thread(target=accept, daemon=True)
            acc.start()
        pool.start(wait_ready_s=900)
        if world > 1 and not sharded:
            acc.join(900)
            pool.wait_ready(900)
        # (serve: rank 0's clients feed shard 0 only, like every other rank feeds its own shard)
        own = pool.control_shards[0] if served else pool
        client = Client(pool.ring.buf, lambda n: own.ring.alloc(n, timeout=600), own.submit_slots, B, rank)
    else:
        import torch.distributed as dist
        from multiprocessing.connection import Client as MPClient

        from ..store import native
        from .gpu_worker import attach_ring, worker_main

        objs = [None]
        dist.broadcast_object_list(objs, src=0)
        info = objs[0]
        conn = MPClient(tuple(info["addr"]), authkey=bytes.fromhex(info["key"]))
        conn.send_bytes(str(rank).encode())
        fc = P.FrameConn(conn)
        local_ring = native.SlotRing(part, int(info.get("parts", {}).get(rank, part * rank)))
        shm, ring_buf = attach_ring(info["shm"], info["nslots"], spec.item_shape, untrack=True)

        def alloc(n):
            s = local_ring.alloc(n, 600.0)
            if not s:
                raise TimeoutError("ingest partition full")
            return s

        client = Client(ring_buf, alloc, fc.submit, B, rank)
        ready = threading.Event()
        wth = threading.Thread(target=worker_main, args=(fc, rank, str(device), spec, info["shm"], info["nslots"], hb),
                               kwargs={"untrack": True, "local_ring": local_ring, "ready_event": ready}, daemon=True)
        wth.start()
        # the worker thread captures HIP graphs in global capture mode: this thread must not touch the device
        # (synchronize, RCCL barrier) until the capture is over
        if not ready.wait(1800):
            raise SystemExit(f"rank {rank}: GPU worker did not come up")

    def wait_images(target: int) -> None:
        while pool.images < target:
            time.sleep(0.0002)

    # ---------------------------------------------------------------- steady-state window
    # The clients submit warmup + steps + tail steps back to back and never stop between warmup and the
    # timed steps, so the serving pipeline never drains and refills inside the window. The window is
    # defined by completion counts on the scheduler (rank 0): t0 when warmup*B*world images have
    # completed, t1 when (warmup+steps)*B*world have; exactly steps*B*world images complete inside it.
    # The tail keeps the pipeline full up to t1 (its images are served, not counted). The barrier +
    # device drain bracket the whole run on every rank.
    tail = max(1, args.inflight + 1)
    warm_n = args.warmup * B * counted_world
    tel = None
    if rank == 0 and args.device == "cuda":
        from ..utils.gpu_telemetry import GpuTelemetry

        # (started before the barrier: its init must not hold rank 0 back while the other ranks' clients already run)
        tel = GpuTelemetry(denv.local_rank)  # clocks / power / hotspot sampled every 200 ms (fail-soft)
        tel.start()
    tune_gc()
    sync(denv)
    t_start = time.perf_counter()
    cth = threading.Thread(target=client.run, args=(args.warmup + args.steps + tail,), daemon=True)
    cth.start()
    dt, ramp_s, drain_s = 0.0, 0.0, 0.0
    tm0 = tm1 = time.monotonic()
    if rank == 0 or sharded:
        if warm_n:  # (no warmup: the window starts at the first submission, fill included)
            wait_images(warm_n)
            t0, tm0 = time.perf_counter(), time.monotonic()
        else:
            t0 = t_start
        wait_images(total_images)
        t1, tm1 = time.perf_counter(), time.monotonic()
        dt, ramp_s = t1 - t0, t0 - t_start
        wait_images(total_images + tail * B * counted_world)
        drain_s = time.perf_counter() - t1
    cth.join()
    sync(denv)
    telemetry = tel.stop() if tel is not None else {}
    p50 = p99 = 0.0
    stats = {}
    lat = []
    if rank == 0 or sharded:
        from ..store.pystore import absolute_path

        lat = sorted(x for pth in [path] + [absolute_path(e) for e in spec.stage_endpoints]
                     for x in cp.store.latencies_window(pth, tm0, tm1))  # ensembles finish at the last stage
        p50, p99 = percentile(lat, 50) * 1e3, percentile(lat, 99) * 1e3
        stats = pool.stats()
    if sharded:
        # the union of the ranks' windows (monotonic clock, one host): every counted image completed inside it
        from ..parallel.dist import gather_objects

        per = gather_objects({"tm0": tm0, "tm1": tm1, "lat": lat, "ramp": ramp_s, "drain": drain_s,
                              "stats": stats}, denv)
        dt = max(r["tm1"] for r in per) - min(r["tm0"] for r in per)
        ramp_s, drain_s = max(r["ramp"] for r in per), max(r["drain"] for r in per)
        lat = sorted(x for r in per for x in r["lat"])
        p50, p99 = percentile(lat, 50) * 1e3, percentile(lat, 99) * 1e3
        if rank == 0:
            stats = dict(per[0]["stats"])
            stats["workers"] = [dict(w, rank=i) for i, r in enumerate(per) for w in r["stats"].get("workers", [])]
            hists = [r["stats"].get("batch_histogram") or [] for r in per]
            stats["batch_histogram"] = [sum(h[i] for h in hists if i < len(h)) for i in range(max(map(len, hists)))]
    dt, p50, p99 = all_reduce_max([dt, p50, p99], denv)  # slowest rank defines the step time
    images = args.steps * B * world
    value = images / dt
    out = None
    if rank == 0:
        http = None
        if args.http and args.device == "cuda":
            try:
                http = http_phase(cp, pool, args.http_seconds, B, spec.item_shape, path)
                nfe = getattr(args, "http_frontends", 0)
                if nfe:
                    http["with_frontends"] = http_phase(cp, pool, args.http_seconds, B, spec.item_shape, path, nfe,
                                                        max_queue_ms=getattr(args, "max_queue_ms", 0.0))
            except Exception as e:  # the headline number stands on its own
                http = {"error": repr(e)}
            nfe = getattr(args, "http_frontends", 0)
            if getattr(args, "http_tls", 0) and nfe and isinstance(http, dict) and "error" not in http:
                try:
                    http["with_frontends_tls"] = http_phase(cp, pool, args.http_seconds, B, spec.item_shape, path,
                                                            nfe, tls=True, max_queue_ms=getattr(args, "max_queue_ms", 0.0))
                except Exception as e:
                    http["with_frontends_tls"] = {"error": repr(e)}
        workers = [{k: w.get(k) for k in ("rank", "images", "batches", "pinned", "hbm_used", "gpu_busy_ms", "gfx_mhz",
                                          "power_w")}
                   for w in stats.get("workers", [])]
        out = {
            "metric": metric, "value": round(value, 2), "unit": unit, "n_gpus": world * group, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None if baseline is None else round(value / baseline, 4),
            "dtype": dtype, "data": "synthetic uint8 payloads (written into the payload ring per submission), "
                                     "random-init weights",
            "p50_task_latency_ms": round(p50, 3), "p99_task_latency_ms": round(p99, 3),
            "window": {"kind": "steady-state, by completion count on the scheduler",
                       "first_counted_image": args.warmup * B * world, "counted_images": images,
                       "warmup_ramp_ms": round(ramp_s * 1e3, 3), "tail_drain_ms": round(drain_s * 1e3, 3),
                       "tail_steps_uncounted": tail},
            "config": dict(config or {}, global_batch=B * world, per_gpu_batch=B,
                           parallelism=(config or {}).get("parallelism", f"dp{world}"),
                           serving_path=("the serve topology: one control plane process, a scheduler shard per GPU "
                                         "(ShardedWorkerPool) + 1 GPU worker per GPU" if served else
                                         "one node scheduler (native) + GPU worker process per GPU, sharded by GPU"
                                         if sharded else "node scheduler (native) + 1 GPU worker process per GPU"),
                           control_plane=cp_mode,
                           ingest_shards=world, ring_slots_per_shard=part, hip_graphs=spec.use_graphs),
            "workers": workers, "batch_histogram": stats.get("batch_histogram"), "http": http,
        }
        if flops_per_item:
            out["tflops_effective"] = round(value * flops_per_item / 1e12, 2)
        if telemetry:
            out["gpu_telemetry"] = telemetry  # rank 0's GPU during the timed region
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    sync(denv)
    if rank == 0 or sharded:
        pool.stop()
        cp.close()
    else:
        wth.join(60)
        del ring_buf
        shm.close()
    destroy(denv)
    return out
