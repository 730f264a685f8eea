"""Node-scale load test of the control plane, CPU only (no model): how many tasks/s can ONE node
scheduler create, dispatch, complete and attach results for, with N worker processes?

Each fake worker speaks the real wire protocol (runtime/protocol.py) and answers every BATCH with a
DONE of top-5 rows immediately, so the measured ceiling is the host path the 8-GPU bench exercises:
native create + enqueue (ingest), dispatcher receive + running transition + BATCH frame, reader
DONE parse + result attach + completed transition + queue complete + slot release. Target: 8 GPUs x
~70k images/s = 560k tasks/s.

    python tools/cp_loadtest.py [--workers 8 --batch 250 --seconds 5 --ingest-threads 4]
    python tools/cp_loadtest.py --serve --workers 8 --frontends 4   (the shipped serve topology, over HTTP)
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def fake_worker(conn, rank: int, row_bytes: int, batch_ms: float = 0.0):
    import numpy as np

    from aiforearth_api_platform_amd.runtime import protocol as P

    fc = P.FrameConn(conn)
    fc.ready(rank, False, {"kind": "classifier", "outputs": [["classes", "int32", [5]], ["probabilities", "float32",
                                                                                         [5]]]})
    zeros = bytes(row_bytes * 1024)
    while True:
        try:
            buf = fc.recv()
        except (EOFError, OSError):
            return
        t = P.frame_type(buf)
        if t == P.F_BATCH:
            bid, slots = P.parse_batch(buf)
            n = slots.shape[0]
            if batch_ms > 0:  # a GPU that takes batch_ms per batch (REST admission experiments)
                time.sleep(batch_ms / 1e3)
            now = time.monotonic()
            fc.done(bid, np.zeros(n, np.uint8), zeros[: n * row_bytes], row_bytes, (now, now, now, 0.0, 0.0))
        elif t == P.F_STOP:
            return


def fake_rank(conn, rank: int, row_bytes: int, batch: int, base: int, part: int, stop_at: float):
    """A torchrun rank of the multi-GPU bench without the GPU: its ingest partition [base, base + part) submitted
    over its own scheduler connection (SUBMIT frames of `batch` slots), BATCHes answered with DONE at once, FREE
    frames returned to the partition — the per-task traffic rank 0's scheduler sees from 7 remote GPUs."""
    import numpy as np

    from aiforearth_api_platform_amd.runtime import protocol as P
    from aiforearth_api_platform_amd.store import native

    fc = P.FrameConn(conn)
    ring = native.SlotRing(part, base)
    fc.ready(rank, False, {"kind": "classifier", "outputs": [["classes", "int32", [5]], ["probabilities", "float32",
                                                                                         [5]]]})
    zeros = bytes(row_bytes * 1024)

    def submitter():
        while time.time() < stop_at:
            s = ring.alloc(batch, 0.5)
            if s:
                fc.submit(s)

    th = threading.Thread(target=submitter, daemon=True)
    th.start()
    while True:
        try:
            buf = fc.recv()
        except (EOFError, OSError):
            return
        t = P.frame_type(buf)
        if t == P.F_BATCH:
            bid, slots = P.parse_batch(buf)
            n = slots.shape[0]
            now = time.monotonic()
            fc.done(bid, np.zeros(n, np.uint8), zeros[: n * row_bytes], row_bytes, (now, now, now, 0.0, 0.0))
        elif t == P.F_FREE:
            ring.free(P.parse_slots(buf).tolist())
        elif t == P.F_STOP:
            return


def run_serve(a) -> dict:
    """The SHIPPED server's topology (serve.py): one serving process whose pool endpoint is a ShardedWorkerPool —
    one node scheduler + dispatch queue + ring partition per GPU, ``--workers`` of them, each with one fake worker
    process (DONE at once) — behind ``--frontends`` native ingest front-ends (ai4e_ingestd) on the public port, driven
    over HTTP by the C++ load generator with binary batches of ``--batch`` tiny (4x4x3) items. Counts completed tasks
    per second in the middle of the load window."""
    import asyncio
    import socket

    from aiohttp import web

    from aiforearth_api_platform_amd.config import Config
    from aiforearth_api_platform_amd.gateway.control import ControlPlane
    from aiforearth_api_platform_amd.gateway.server import BATCH_CONTENT_TYPE, Gateway, Route, RouteTable
    from aiforearth_api_platform_amd.runtime.frontend import open_listeners
    from aiforearth_api_platform_amd.runtime.http_load import run_native_clients
    from aiforearth_api_platform_amd.runtime.model_endpoint import ModelEndpoint
    from aiforearth_api_platform_amd.runtime.native_frontend import spawn_native_frontends
    from aiforearth_api_platform_amd.runtime.worker_pool import ModelSpec, ShardedWorkerPool

    cp = ControlPlane(Config.load(env={}))
    path = "/v1/ai4e/lt/classify"
    shape = tuple(int(v) for v in a.item_shape.split("x"))
    B = a.batch
    spec = ModelSpec("aiforearth_api_platform_amd.models.toy:tiny_classifier", shape, B, 5, {}, False)
    pool = ShardedWorkerPool(cp, "http://127.0.0.1" + path, spec, ["cpu"] * a.workers, frontends=a.frontends,
                             frontend_slots=B * 16, ring_slots=B * 4, max_delay_s=0.0005, poll_s=0.005,
                             heartbeat_timeout_s=60.0, shards=a.shards)
    ctx = mp.get_context("spawn")
    procs = []
    shards = pool.control_shards
    for i in range(a.workers):  # fake workers dealt round-robin over the control-plane shards
        shard = shards[i % len(shards)]
        parent, child = ctx.Pipe()
        p = ctx.Process(target=fake_worker, args=(child, i, 40, a.batch_ms), daemon=True)
        p.start()
        child.close()
        shard.attach_remote(i, parent, device="fake")
        procs.append(p)
    while sum(1 for w in pool.workers if w.stats.get("ready")) < a.workers:
        pool.refresh()
        time.sleep(0.01)
    ep = ModelEndpoint(cp, path, worker=pool)
    table = RouteTable()
    table.add(Route("/v1/lt/async", "async", ep))
    gw = Gateway(cp, table)
    with socket.socket() as s0:
        s0.bind(("127.0.0.1", 0))
        port = s0.getsockname()[1]
    socks = open_listeners("127.0.0.1", port, shared=True)
    box = {}

    def serve():
        loop = asyncio.new_event_loop()
        asyncio.set_event_loop(loop)
        runner = web.AppRunner(gw.app, access_log=None)
        loop.run_until_complete(runner.setup())
        loop.run_until_complete(web.SockSite(runner, socks[1]).start())
        box["loop"] = loop
        loop.run_forever()

    threading.Thread(target=serve, daemon=True).start()
    socks[0].close()  # only the front-ends answer on the public port
    fe = spawn_native_frontends(a.frontends, {"lt": ep}, [{"prefix": "/v1/lt/async", "mode": "async", "endpoint": "lt"}],
                                "127.0.0.1", port, f"http://127.0.0.1:{socks[1].getsockname()[1]}",
                                max_queue_ms=a.max_queue_ms)
    time.sleep(1.0)
    body = bytes(B * int(np.prod(shape)))
    samples = {}

    def sampler():
        time.sleep(1.0 + a.seconds * 0.25)  # (load generators start 1 s after the call)
        samples["n0"], samples["t0"] = pool.images, time.perf_counter()
        time.sleep(a.seconds * 0.5)
        samples["n1"], samples["t1"] = pool.images, time.perf_counter()

    th = threading.Thread(target=sampler)
    th.start()
    res = run_native_clients(f"http://127.0.0.1:{port}/v1/lt/async", a.seconds, a.conc, body, BATCH_CONTENT_TYPE,
                             procs=a.client_procs)
    th.join()
    rate = (samples["n1"] - samples["n0"]) / (samples["t1"] - samples["t0"])
    ids = res["ids"]
    lat = sorted(cp.store.latencies(ids[-20000:]))
    from aiforearth_api_platform_amd.utils.metrics import percentile

    out = {"metric": "control-plane tasks/s through the shipped serve topology (native front-ends -> sharded schedulers "
                     "-> fake workers), no model",
           "value": round(rate), "unit": "tasks/s", "control_plane_shards": len(pool.control_shards),
           "fake_workers": a.workers, "ingest_frontends": a.frontends, "batch": B, "http_requests": res["requests"],
           "http_errors": res["errors"], "busy_429": res.get("busy"), "accepted_tasks": len(ids),
           "client_cpu_s": round(res["client_cpu_s"], 2), "seconds": a.seconds, "cpu_count": os.cpu_count(),
           "p50_task_latency_ms": round(percentile(lat, 50) * 1e3, 3) if lat else None,
           "item_shape": list(shape), "batch_ms": a.batch_ms, "max_queue_ms": a.max_queue_ms}
    for p in fe:
        p.terminate()
    for p in fe:
        p.join(10)
    box["loop"].call_soon_threadsafe(box["loop"].stop)
    pool.stop()
    for p in procs:
        p.join(5)
        if p.is_alive():
            p.terminate()
    cp.close()
    return out


def _shard(args, barrier, out_q):
    """One control-plane shard (the sharded multi-GPU bench: one node scheduler per GPU) in its own process."""
    import argparse as _a

    a = _a.Namespace(**args)
    barrier.wait()
    out_q.put(run(a))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--batch", type=int, default=250)
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--ingest-threads", type=int, default=4)
    ap.add_argument("--remote", action="store_true",
                    help="every worker is a separate rank process that also submits its own tasks (torchrun topology)")
    ap.add_argument("--shards", type=int, default=0,
                    help="K independent scheduler processes (one per GPU, the sharded bench layout), "
                         "--workers fake workers each; the value is their sum")
    ap.add_argument("--serve", action="store_true",
                    help="the shipped server's topology: ShardedWorkerPool (one scheduler per worker) + native front-ends")
    ap.add_argument("--frontends", type=int, default=4)
    ap.add_argument("--conc", type=int, default=16, help="(--serve) HTTP connections per load process")
    ap.add_argument("--client-procs", type=int, default=2)
    ap.add_argument("--item-shape", default="4x4x3", help="(--serve) uint8 item shape HxWxC")
    ap.add_argument("--batch-ms", type=float, default=0.0, help="(--serve) fake GPU time per batch")
    ap.add_argument("--max-queue-ms", type=float, default=0.0, help="(--serve) front-end latency budget")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    if a.serve:
        out = run_serve(a)
    elif a.shards:
        ctx = mp.get_context("spawn")
        bar, q = ctx.Barrier(a.shards), ctx.Queue()
        kw = dict(vars(a), shards=0, json_out="")
        ps = [ctx.Process(target=_shard, args=(kw, bar, q)) for _ in range(a.shards)]
        [p.start() for p in ps]
        res = [q.get(timeout=600) for _ in ps]
        [p.join(60) for p in ps]
        out = {"metric": res[0]["metric"], "value": sum(r["value"] for r in res), "unit": "tasks/s",
               "shards": a.shards, "per_shard": [r["value"] for r in res], "workers_per_shard": a.workers,
               "batch": a.batch, "ingest": res[0]["ingest"], "seconds": a.seconds,
               "p50_task_latency_ms": max(r["p50_task_latency_ms"] or 0 for r in res), "cpu_count": os.cpu_count()}
    else:
        out = run(a)
    line = json.dumps(out)
    print(line)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")


def run(a) -> dict:
    from aiforearth_api_platform_amd.config import Config
    from aiforearth_api_platform_amd.gateway.control import ControlPlane
    from aiforearth_api_platform_amd.store import native
    from aiforearth_api_platform_amd.utils.metrics import percentile

    cp = ControlPlane(Config.load(env={}))
    path = "/v1/ai4e/resnet50/classify"
    q = cp.queue_for("http://127.0.0.1" + path)
    B = a.batch
    per_thread = B * 4
    nslots = per_thread * a.ingest_threads
    sched = native.NodeScheduler(cp.store, q, "http://127.0.0.1" + path, nslots, max_batch=B, linger_s=0.0005,
                                 depth=2, hb_timeout_s=60.0, poll_s=0.005)
    ctx = mp.get_context("spawn")
    procs = []
    rings = []
    if a.remote:
        part = B * int(os.environ.get("CP_PART_BATCHES", "16"))
        sched = native.NodeScheduler(cp.store, q, "http://127.0.0.1" + path, part * a.workers, max_batch=B,
                                     linger_s=0.0005, depth=2, hb_timeout_s=60.0, poll_s=0.005)
        stop_at = time.time() + 1.0 + a.seconds + 30.0
        for r in range(a.workers):
            sched.add_remote_partition(r * part, part, r)
            parent, child = ctx.Pipe()
            p = ctx.Process(target=fake_rank, args=(child, r, 40, B, r * part, part, stop_at), daemon=True)
            p.start()
            child.close()
            sched.attach(r, os.dup(parent.fileno()), True)
            parent.close()
            procs.append(p)
    else:
        rings = [native.SlotRing(per_thread, i * per_thread) for i in range(a.ingest_threads)]
        for r in rings:
            sched.add_local_ring(r)
        for r in range(a.workers):
            parent, child = ctx.Pipe()
            p = ctx.Process(target=fake_worker, args=(child, r, 40), daemon=True)
            p.start()
            child.close()
            sched.attach(r, os.dup(parent.fileno()), True)
            parent.close()
            procs.append(p)
    while sum(1 for w in sched.worker_stats() if w["ready"]) < a.workers:
        time.sleep(0.01)
    stop = threading.Event()

    def ingest(ring):
        while not stop.is_set():
            s = ring.alloc(B, 1.0)
            if s:
                sched.submit(s, "")

    evict_stop = threading.Event()

    def evictor():  # the serving process's TTL timer, at a short TTL so the store stays bounded
        while not evict_stop.wait(0.5):
            cp.store.evict_finished(2.0)

    ths = [threading.Thread(target=ingest, args=(r,), daemon=True) for r in rings]
    ev = threading.Thread(target=evictor, daemon=True)
    ev.start()
    for t in ths:
        t.start()
    time.sleep(1.0)  # warm
    n0, t0, m0 = sched.images_done(), time.perf_counter(), time.monotonic()
    time.sleep(a.seconds)
    n1, t1, m1 = sched.images_done(), time.perf_counter(), time.monotonic()
    stop.set()
    for t in ths:
        t.join(5)
    lat = sorted(cp.store.latencies_window(path, m0, m1))
    evict_stop.set()
    rate = (n1 - n0) / (t1 - t0)
    out = {"metric": "control-plane tasks/s (create + dispatch + complete + result attach), no model",
           "value": round(rate), "unit": "tasks/s", "workers": a.workers, "batch": B,
           "ingest": "remote ranks (SUBMIT frames)" if a.remote else f"{a.ingest_threads} local Python threads",
           "seconds": a.seconds, "p50_task_latency_ms": round(percentile(lat, 50) * 1e3, 3) if lat else None,
           "store_size_end": cp.store.size(), "cpu_count": os.cpu_count(),
           "batch_histogram": sched.batch_histogram()}
    sched.stop()
    for p in procs:
        p.join(5)
        if p.is_alive():
            p.terminate()
    cp.close()
    return out


if __name__ == "__main__":
    main()
