"""Self-measured comparator: the reference's request path, run on the same MI355X.

Reproduces the reference architecture for the ResNet-50 async API:

* gateway creates the task with an HTTP call to the task store (``request_policy.xml`` ->
  ``CacheConnectorUpsert``), then the dispatcher POSTs the body to the model container with a
  ``taskId`` header (``BackendQueueProcessor.cs:48-52``);
* the container is a threaded Flask app with the ``APIService.api_async_func`` decorator
  (``ai4e_service.py``): ``AddTask`` GETs the task, the work runs on a new thread per request,
  ``UpdateTaskStatus`` / ``CompleteTask`` are HTTP GET+POST round trips to the task store
  (``distributed_api_task.py:29-56``);
* the model runs **batch 1** per request (no batching in the reference);
* the client polls ``GET /task/{id}`` until completed.

Same fused ResNet-50 and GPU as bench.py, so the difference is the serving architecture.

    python bench/comparator_refstyle.py [--requests 512 --concurrency 32]
"""
import argparse
import asyncio
import json
import os
import socket
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=512)
    ap.add_argument("--concurrency", type=int, default=32)
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    from aiohttp import web
    from flask import Flask, request

    from aiforearth_api_platform_amd import _build
    from aiforearth_api_platform_amd import config as cfgmod
    from aiforearth_api_platform_amd.api import APIService, HttpTaskClient, TaskManager
    from aiforearth_api_platform_amd.gateway.control import ControlPlane
    from aiforearth_api_platform_amd.gateway.server import Gateway
    from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50
    from aiforearth_api_platform_amd.utils.logging import AI4ELogger

    _build.build_all()
    sp, mp_ = _port(), _port()
    os.environ["API_PREFIX"] = "/v1/resnet50"
    cfgmod.set_config(cfgmod.Config.load())
    # --- task store service (Redis + CacheConnector functions stand-in)
    gw = Gateway(ControlPlane(cfgmod.Config.load(env={})))

    def run_store():
        loop = asyncio.new_event_loop()
        asyncio.set_event_loop(loop)
        runner = web.AppRunner(gw.app)
        loop.run_until_complete(runner.setup())
        loop.run_until_complete(web.TCPSite(runner, "127.0.0.1", sp).start())
        loop.run_forever()

    threading.Thread(target=run_store, daemon=True).start()
    store = f"http://127.0.0.1:{sp}"
    # --- model container: Flask + APIService, batch-1 inference on a thread per request
    dev = torch.device("cuda:0")
    model = FusedResNet(resnet50(seed=0), device=dev)
    model(torch.zeros(1, 224, 224, 3, dtype=torch.uint8, device=dev))
    torch.cuda.synchronize()
    app = Flask("refstyle")
    tm = TaskManager(HttpTaskClient(store + "/v1/cache/upsert", store + "/v1/cache/get"))
    svc = APIService(app, AI4ELogger(stream=None), tm, max_workers=1024, install_signal_handlers=False)
    lock = threading.Lock()

    def pre(req):
        return {"img": np.frombuffer(req.get_data(), dtype=np.uint8).reshape(224, 224, 3)}

    @svc.api_async_func(api_path="/classify", methods=["POST"], request_processing_function=pre)
    def classify(*args, **kwargs):
        tid = kwargs["taskId"]
        svc.api_task_manager.UpdateTaskStatus(tid, "running")
        x = torch.from_numpy(kwargs["img"].copy())[None].to(dev)
        with lock:  # one CUDA stream, batch 1 (the reference runs one request per model call)
            logits = model(x)
            top = int(logits.argmax(1).item())
        svc.api_task_manager.CompleteTask(tid, f"completed - class {top}")

    threading.Thread(target=lambda: app.run("127.0.0.1", mp_, threaded=True), daemon=True).start()
    time.sleep(1.0)

    import requests as rq
    sess = rq.Session()
    img = np.random.default_rng(0).integers(0, 256, (224, 224, 3), dtype=np.uint8).tobytes()
    model_url = f"http://127.0.0.1:{mp_}/v1/resnet50/classify"

    def one(_):
        t0 = time.perf_counter()
        s = rq.Session()
        task = s.post(store + "/v1/cache/upsert", json={"TaskId": "", "Status": "created", "BackendStatus": "created",
                                                        "Endpoint": model_url, "PublishToGrid": False}).json()
        s.post(model_url, data=img, headers={"taskId": task["TaskId"]})
        while True:
            st = s.get(store + "/v1/cache/get", params={"taskId": task["TaskId"]}).json()
            if st["BackendStatus"] in ("completed", "failed"):
                break
            time.sleep(0.001)
        return time.perf_counter() - t0

    import concurrent.futures as cf
    with cf.ThreadPoolExecutor(a.concurrency) as ex:
        list(ex.map(one, range(16)))
        t0 = time.perf_counter()
        lat = sorted(ex.map(one, range(a.requests)))
        dt = time.perf_counter() - t0
    out = {"metric": "reference-style ResNet-50 async API images/s (1 GPU, batch 1, HTTP task store)",
           "value": round(a.requests / dt, 2), "unit": "images/s", "p50_task_latency_ms": round(lat[len(lat) // 2] * 1e3, 2),
           "p99_task_latency_ms": round(lat[int(len(lat) * 0.99)] * 1e3, 2),
           "config": {"requests": a.requests, "concurrency": a.concurrency, "model": "resnet50", "dtype": "bf16"}}
    print(json.dumps(out), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(json.dumps(out) + "\n")
    os._exit(0)


if __name__ == "__main__":
    main()
