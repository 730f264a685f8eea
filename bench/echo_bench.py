"""BASELINE config #1: sync "echo" API on CPU (plumbing, no GPU) — this platform vs reference style.

* ``platform``: the aiohttp gateway route -> in-process echo backend (admission control, metrics).
* ``reference``: a Flask app with the ``APIService.api_sync_func`` decorator (the reference's
  container runtime, ``APIs/1.0/base-py/ai4e_service.py``), served by werkzeug's threaded server.

Each server runs in its own process (its own GIL, like a deployed service); the asyncio HTTP client
drives it at fixed concurrency from this process and reports req/s and p50/p99 latency.

The client is the measuring instrument, so its own host stalls must stay out of the numbers: it opens all
``--concurrency`` connections with an untimed warm-up wave first, and runs with its garbage collector frozen
(as the servers do, runtime/hostperf.py). Round 3's p99 of 160 ms (5000 requests) was one generation-2 GC pause of
the client (25-35 ms here, longer on the GPU box) stalling all 64 in-flight requests at once — 64 of 5000 requests
is more than the top 1 % — plus the connection-opening first wave; at 8000 requests (round 2) the same stall fell
just outside p99 (16 ms).

    python bench/echo_bench.py [--requests 20000 --concurrency 64]
"""
import argparse
import asyncio
import json
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def start_platform(port, ready=None):
    from aiohttp import web

    from aiforearth_api_platform_amd.config import Config
    from aiforearth_api_platform_amd.gateway.control import ControlPlane
    from aiforearth_api_platform_amd.gateway.server import Gateway, Route, RouteTable
    from aiforearth_api_platform_amd.models.toy import echo

    from aiforearth_api_platform_amd.runtime.hostperf import tune_gc

    t = RouteTable()
    t.add(Route("/v1/echo", "sync", echo, inline=True))
    gw = Gateway(ControlPlane(Config.load(env={})), t)
    tune_gc()
    web.run_app(gw.app, host="127.0.0.1", port=port, access_log=None, print=None)


def start_reference(port):
    os.environ["API_PREFIX"] = "/v1"
    from flask import Flask, request

    from aiforearth_api_platform_amd.api import APIService, InProcTaskClient, TaskManager
    from aiforearth_api_platform_amd.utils.logging import AI4ELogger

    app = Flask("echo")
    svc = APIService(app, AI4ELogger(stream=None), TaskManager(InProcTaskClient()), install_signal_handlers=False)

    @svc.api_sync_func(api_path="/echo", methods=["POST"])
    def echo(*args, **kwargs):
        return request.get_data()

    app.run("127.0.0.1", port, threaded=True)


async def drive(url, n, conc, warm: int = 0):
    import gc

    import aiohttp

    lat = []
    payload = json.dumps({"hello": "world"}).encode()
    async with aiohttp.ClientSession(connector=aiohttp.TCPConnector(limit=conc)) as s:
        for _ in range(200):
            try:
                async with s.post(url, data=payload) as r:
                    await r.read()
                    break
            except aiohttp.ClientError:
                await asyncio.sleep(0.05)
        sem = asyncio.Semaphore(conc)

        async def one(timed=True):
            async with sem:
                t = time.perf_counter()
                async with s.post(url, data=payload, headers={"Content-Type": "application/json"}) as r:
                    assert r.status == 200, r.status
                    await r.read()
                if timed:
                    lat.append(time.perf_counter() - t)

        # untimed warm-up: every connection of the pool opened, both sides' first-use paths taken
        await asyncio.gather(*[one(False) for _ in range(warm or 4 * conc)])
        gc.collect()
        gc.freeze()  # the client's own generation-2 pauses would stall every in-flight request at once
        gc.disable()
        try:
            t0 = time.perf_counter()
            await asyncio.gather(*[one() for _ in range(n)])
            dt = time.perf_counter() - t0
        finally:
            gc.enable()
            gc.unfreeze()
    lat.sort()
    return n / dt, lat[len(lat) // 2] * 1e3, lat[int(len(lat) * 0.99)] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=20000)
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    import multiprocessing as mp

    pp, rp = _port(), _port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=start_platform, args=(pp,), daemon=True),
             ctx.Process(target=start_reference, args=(rp,), daemon=True)]
    for p in procs:
        p.start()
    res = {}
    for name, url in (("platform", f"http://127.0.0.1:{pp}/v1/echo"), ("reference_style", f"http://127.0.0.1:{rp}/v1/echo")):
        rps, p50, p99 = asyncio.run(drive(url, a.requests, a.concurrency))
        res[name] = {"req_per_s": round(rps, 1), "p50_ms": round(p50, 3), "p99_ms": round(p99, 3)}
    out = {"metric": "echo API req/s (CPU, sync)", "value": res["platform"]["req_per_s"], "unit": "req/s",
           "vs_reference_style": round(res["platform"]["req_per_s"] / res["reference_style"]["req_per_s"], 3),
           "results": res, "config": {"requests": a.requests, "concurrency": a.concurrency}}
    for p in procs:
        p.terminate()
    print(json.dumps(out), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(json.dumps(out) + "\n")


if __name__ == "__main__":
    main()
