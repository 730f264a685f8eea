"""HTTP -> GPU end to end for every model family (BASELINE configs 2-5 as APIs).

The platform is built from ``examples/platform_gpu_small.yaml`` (per-GPU worker pools on cuda:0,
hand-written kernels in the worker processes); requests go through the aiohttp gateway, tasks are
polled on ``GET /v1/taskmanagement/task/{id}`` until completed and ``/result`` is checked.
"""
import asyncio
import base64
import io
import os

import numpy as np
import pytest
import yaml
from aiohttp.test_utils import TestClient, TestServer

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def platform():
    from aiforearth_api_platform_amd.config import Config
    from aiforearth_api_platform_amd.serve import build_platform

    with open(os.path.join(ROOT, "examples", "platform_gpu_small.yaml")) as f:
        doc = yaml.safe_load(f)
    cfg = Config.load(env={}, yaml_values=doc.get("settings") or {})
    cp, gw, endpoints, _ = build_platform(doc, cfg)
    for ep in endpoints.values():
        ep.start()
    yield cp, gw, endpoints
    for ep in endpoints.values():
        ep.stop()
    cp.close()


async def _post_and_wait(c, route, body, timeout=240.0):
    r = await c.post(route, data=body, headers={"Content-Type": "application/octet-stream"})
    assert r.status == 200, await r.text()
    tid = (await r.json())["TaskId"]
    loop = asyncio.get_running_loop()
    deadline = loop.time() + timeout
    while loop.time() < deadline:
        rec = await (await c.get(f"/v1/taskmanagement/task/{tid}")).json()
        if rec["BackendStatus"] in ("completed", "failed"):
            break
        await asyncio.sleep(0.05)
    assert rec["BackendStatus"] == "completed", rec
    res = await (await c.get(f"/v1/taskmanagement/task/{tid}/result")).json()
    return tid, rec, res["Result"]


def _run(gw, fn):
    async def go():
        c = TestClient(TestServer(gw.app))
        await c.start_server()
        try:
            return await fn(c)
        finally:
            await c.close()

    return asyncio.new_event_loop().run_until_complete(go())


def test_classify_detect_landcover_ensemble_over_http(platform):
    import torch

    cp, gw, _ = platform
    rng = np.random.default_rng(3)
    img224 = rng.integers(0, 256, (224, 224, 3), dtype=np.uint8)
    img256 = rng.integers(0, 256, (256, 256, 3), dtype=np.uint8)
    mosaic = rng.integers(0, 256, (1024, 1024, 4), dtype=np.uint8)

    async def fn(c):
        out = {}
        out["cls"] = await _post_and_wait(c, "/v1/camera-trap/classify-async", img224.tobytes())
        out["det"] = await _post_and_wait(c, "/v1/camera-trap/detection-async", img256.tobytes())
        out["lc"] = await _post_and_wait(c, "/v1/landcover/classify", mosaic.tobytes())
        out["ens"] = await _post_and_wait(c, "/v1/camera-trap/detect-classify", img256.tobytes())
        r = await c.post("/v1/camera-trap/detection-sync", data=img256.tobytes(),
                         headers={"Content-Type": "application/octet-stream"})
        assert r.status == 200
        out["det_sync"] = await r.json()
        tr = await (await c.get(f"/v1/taskmanagement/task/{out['cls'][0]}/trace")).json()
        out["trace"] = tr
        return out

    out = _run(gw, fn)
    # classification: same answer as the fused model run eagerly in this process
    from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50
    ref = FusedResNet(resnet50(seed=0), device="cuda:0").topk_u8(torch.from_numpy(img224[None]).cuda(), 5)[0]
    assert out["cls"][2]["classes"][0] == int(ref[0, 0])
    # detection (async route rewritten to /v1/animal_detection like the reference chart)
    tid, rec, det = out["det"]
    assert rec["EndpointPath"] == "/v1/animal_detection"
    assert isinstance(det["detections"], list) and len(det["detections"]) > 0
    d0 = det["detections"][0]
    assert len(d0["bbox"]) == 4 and 0 <= d0["label"] < 4
    assert out["det_sync"]["detections"] == det["detections"]  # same image, same model: identical
    # land-cover: a full-resolution class map (PNG) + histogram over the 7 classes
    _, _, lc = out["lc"]
    from PIL import Image
    cls = np.asarray(Image.open(io.BytesIO(base64.b64decode(lc["class_map"]))))
    assert cls.shape == (1024, 1024) and cls.max() < 7 and sum(lc["histogram"]) == 1024 * 1024
    # ensemble: one TaskId across both stages, ending at the classifier stage endpoint
    tid, rec, ens = out["ens"]
    assert rec["EndpointPath"] == "/v1/camera-trap/ensemble/classify"
    assert cp.store.zcard("/v1/camera-trap/ensemble/detect_created") == 0
    assert 0 < len(ens["animals"]) <= 4 and all(0 <= a["species"] < 20 for a in ens["animals"])
    # per-task stage trace from the worker process
    tr = out["trace"]
    assert tr["t_worker_done"] >= tr["t_worker_launch"] > 0 and "durations_ms" in tr


def test_ingest_frontends_gpu():
    """Ingest front-end processes (runtime/frontend.py) in front of a GPU pool endpoint: POSTs over fresh
    connections are spread over the serving process and 2 front-ends (SO_REUSEPORT); every task completes
    on the GPU with the same top-5 as the serving process's own ingest path."""
    import socket
    import threading
    import time

    import requests
    from aiohttp import web

    from aiforearth_api_platform_amd.config import Config
    from aiforearth_api_platform_amd.runtime.frontend import open_listeners
    from aiforearth_api_platform_amd.serve import build_platform, start_frontends

    with open(os.path.join(ROOT, "examples", "platform_gpu_small.yaml")) as f:
        full = yaml.safe_load(f)
    doc = {"settings": dict(full.get("settings") or {}, frontend_processes=2),
           "endpoints": {"resnet50": full["endpoints"]["resnet50"]},
           "routes": [r for r in full["routes"] if r.get("backend") == "inproc:resnet50"]}
    cfg = Config.load(env={}, yaml_values=doc["settings"])
    cp, gw, endpoints, _ = build_platform(doc, cfg)
    for ep in endpoints.values():
        ep.start()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    socks = open_listeners("127.0.0.1", port, shared=True)
    box = {}

    def serve():
        loop = asyncio.new_event_loop()
        runner = web.AppRunner(gw.app, access_log=None)
        loop.run_until_complete(runner.setup())
        for sk in socks:
            loop.run_until_complete(web.SockSite(runner, sk).start())
        box["loop"] = loop
        loop.run_forever()
        loop.run_until_complete(runner.cleanup())

    th = threading.Thread(target=serve, daemon=True)
    th.start()
    cfg.host = "127.0.0.1"
    fe = start_frontends(cfg, doc, endpoints, port, socks[1].getsockname()[1])
    try:
        assert len(fe) == 2
        time.sleep(8.0)  # front-end interpreters start and bind
        route = next(r["prefix"] for r in doc["routes"] if r.get("mode", "async") == "async")
        img = np.random.default_rng(3).integers(0, 256, (224, 224, 3), dtype=np.uint8)
        ids = []
        for _ in range(24):
            r = requests.post(f"http://127.0.0.1:{port}{route}", data=img.tobytes(),
                              headers={"Content-Type": "application/octet-stream", "Connection": "close"}, timeout=60)
            assert r.status_code == 200, r.text
            ids.append(r.json()["TaskId"])
        deadline = time.time() + 120
        results = {}
        while time.time() < deadline and len(results) < len(ids):
            for t in ids:
                if t in results:
                    continue
                rec = requests.get(f"http://127.0.0.1:{port}/v1/taskmanagement/task/{t}", timeout=30).json()
                if rec["BackendStatus"] == "completed":
                    results[t] = requests.get(f"http://127.0.0.1:{port}/v1/taskmanagement/task/{t}/result",
                                              timeout=30).json()["Result"]
            time.sleep(0.05)
        assert len(results) == len(ids)
        classes = {tuple(r["classes"]) for r in results.values()}
        assert len(classes) == 1  # the same image -> the same top-5 whichever process ingested it
    finally:
        for p in fe:
            p.terminate()
        for p in fe:
            p.join(10)
        if "loop" in box:
            box["loop"].call_soon_threadsafe(box["loop"].stop)
        th.join(10)
        for ep in endpoints.values():
            ep.stop()
        cp.close()
