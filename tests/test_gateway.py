"""HTTP gateway end-to-end on CPU: async/sync model routes, task GET, cache/requests/webhook routes, metrics."""
import asyncio
import io
import json

import numpy as np
import pytest
import torch
from aiohttp.test_utils import TestClient, TestServer

from aiforearth_api_platform_amd.config import Config
from aiforearth_api_platform_amd.gateway.control import ControlPlane
from aiforearth_api_platform_amd.gateway.server import Gateway, Route, RouteTable
from aiforearth_api_platform_amd.runtime.engine import InferenceEngine, PayloadRing
from aiforearth_api_platform_amd.runtime.model_endpoint import ModelEndpoint, decode_image
from aiforearth_api_platform_amd.sched.dispatcher import QueueDispatcher, WebhookDispatcher


def tiny_model(x_u8):
    # logits = per-channel means (3 classes) + constant classes -> deterministic top-k
    m = x_u8.float().mean(dim=(1, 2))
    return torch.cat([m, torch.zeros(m.shape[0], 3)], dim=1)


@pytest.fixture
def stack():
    cfg = Config.load(env={}, queue_retry_delay_ms=0)
    cp = ControlPlane(cfg)
    eng = InferenceEngine(tiny_model, (8, 8, 3), 16, device=torch.device("cpu"), topk=2)
    ring = PayloadRing(64, (8, 8, 3))
    ep = ModelEndpoint(cp, "/v1/ai4e/tiny/classify", eng, ring).start()
    calls = []

    def echo(task_id, body, headers):
        calls.append(body)
        return 200, {"echo": json.loads(body or b"null")}

    table = RouteTable()
    table.add(Route("/v1/tiny/async", "async", ep))
    table.add(Route("/v1/tiny/sync", "sync", ep, max_concurrent=4))
    table.add(Route("/v1/echo", "sync", echo, content_types=["application/json"], max_content_length=64))
    table.add(Route("/v1/generic/async", "async", None, rewrite="/v1/backend/generic"))
    disp = QueueDispatcher(cp, "http://127.0.0.1/v1/backend/generic", lambda t, b, h: (calls.append(b), 200)[1],
                           retry_delay_s=0.0, poll_s=0.01).start()
    wh = WebhookDispatcher(cp, {"/v1/backend/generic": lambda t, b, h: 200})
    gw = Gateway(cp, table, webhook=wh)
    yield gw, cp, ep, calls
    ep.stop()
    disp.stop()
    wh.shutdown()
    cp.close()


def run(coro):
    return asyncio.new_event_loop().run_until_complete(coro)


async def _client(gw):
    c = TestClient(TestServer(gw.app))
    await c.start_server()
    return c


def test_async_model_route_and_task_get(stack):
    gw, cp, ep, _ = stack

    async def go():
        c = await _client(gw)
        img = np.full((8, 8, 3), 7, np.uint8)
        img[..., 1] = 200
        r = await c.post("/v1/tiny/async", data=img.tobytes(), headers={"Content-Type": "application/octet-stream"})
        assert r.status == 200
        t = await r.json()
        assert t["BackendStatus"] == "created" and t["EndpointPath"] == "/v1/ai4e/tiny/classify"
        for _ in range(200):
            r = await c.get(f"/v1/taskmanagement/task/{t['TaskId']}")
            st = await r.json()
            if st["BackendStatus"] == "completed":
                break
            await asyncio.sleep(0.01)
        assert st["BackendStatus"] == "completed"
        r = await c.get(f"/v1/taskmanagement/task/{t['TaskId']}/result")
        res = (await r.json())["Result"]
        assert res["classes"][0] == 1
        r = await c.get("/v1/taskmanagement/task/does-not-exist")
        assert r.status == 204
        await c.close()

    run(go())


def test_sync_model_route_png(stack):
    gw, cp, ep, _ = stack
    from PIL import Image

    async def go():
        c = await _client(gw)
        im = np.zeros((16, 16, 3), np.uint8)
        im[..., 2] = 255
        buf = io.BytesIO()
        Image.fromarray(im).save(buf, format="PNG")
        r = await c.post("/v1/tiny/sync", data=buf.getvalue(), headers={"Content-Type": "image/png"})
        assert r.status == 200
        out = await r.json()
        assert out["classes"][0] == 2
        await c.close()

    run(go())


def test_admission_and_echo(stack):
    gw, cp, ep, calls = stack

    async def go():
        c = await _client(gw)
        r = await c.post("/v1/echo", json={"a": 1})
        assert r.status == 200 and (await r.json()) == {"echo": {"a": 1}}
        r = await c.post("/v1/echo", data="x", headers={"Content-Type": "text/plain"})
        assert r.status == 401
        r = await c.post("/v1/echo", data=json.dumps({"a": "x" * 100}), headers={"Content-Type": "application/json"})
        assert r.status == 413
        gw.is_terminating = True
        r = await c.post("/v1/echo", json={"a": 1})
        assert r.status == 503
        assert (await c.get("/")).status == 503
        gw.is_terminating = False
        assert (await c.get("/nope")).status == 404
        await c.close()

    run(go())


def test_generic_async_route_rewrite_dispatch(stack):
    gw, cp, ep, calls = stack

    async def go():
        c = await _client(gw)
        r = await c.post("/v1/generic/async/sub", json={"job": 5})
        t = await r.json()
        assert t["Endpoint"] == "http://127.0.0.1/v1/backend/generic/sub"
        await c.close()
        return t

    t = run(go())
    # rewritten endpoint /v1/backend/generic/sub has its own queue; dispatcher serves /v1/backend/generic
    assert cp.queue_for(t["Endpoint"]).depth() == 1


def test_cache_requests_webhook_metrics_routes(stack):
    gw, cp, ep, calls = stack

    async def go():
        c = await _client(gw)
        r = await c.post("/v1/cache/upsert", data=b"")
        assert r.status == 400
        r = await c.post("/v1/cache/upsert", json={"TaskId": "", "Status": "created", "BackendStatus": "created",
                                                  "Endpoint": "http://x/v1/a", "PublishToGrid": False})
        t = await r.json()
        r = await c.get("/v1/cache/get", params={"taskId": t["TaskId"]})
        assert (await r.json())["TaskId"] == t["TaskId"]
        assert (await c.post("/v1/requests/upsert", json={"ApiPath": "/v1/a", "ServiceCluster": "c",
                                                          "IncrementBy": 2, "DecrementBy": 0})).status == 200
        r = await c.post("/v1/requests/get", json={"ApiPath": "/v1/a", "ServiceCluster": "c"})
        assert (await r.text()) == "2"
        r = await c.post("/v1/backend/webhook", json=[{"EventType": "Microsoft.EventGrid.SubscriptionValidationEvent",
                                                       "Data": {"ValidationCode": "zz"}}])
        assert (await r.json()) == {"ValidationResponse": "zz"}
        r = await c.post("/v1/backend/webhook", json=[{"Id": "t1", "Subject": "http://h/v1/backend/generic",
                                                       "Data": {"x": 1}, "EventType": "task"}])
        assert r.status == 200
        txt = await (await c.get("/metrics")).text()
        assert "CURRENT_REQUESTS_c_v1_a" in txt and "/v1/a_created" in txt
        st = await (await c.get("/v1/platform/stats")).json()
        assert st["control_plane"]["tasks"] >= 1
        await c.close()

    run(go())


def test_decode_image_formats():
    a = np.arange(4 * 4 * 3, dtype=np.uint8).reshape(4, 4, 3)
    assert np.array_equal(decode_image(a.tobytes(), "application/octet-stream", (4, 4, 3)), a)
    buf = io.BytesIO()
    np.save(buf, a)
    assert np.array_equal(decode_image(buf.getvalue(), "application/x-npy", (4, 4, 3)), a)
    import base64
    js = json.dumps({"image_b64": base64.b64encode(a.tobytes()).decode(), "shape": [4, 4, 3]}).encode()
    assert np.array_equal(decode_image(js, "application/json", (4, 4, 3)), a)
    assert decode_image(a.tobytes(), "application/octet-stream", (4, 4, 3)).shape == (4, 4, 3)
    big = decode_image(np.zeros((8, 8, 3), np.uint8).tobytes(), "application/json" if False else "application/octet-stream", (8, 8, 3))
    assert big.shape == (8, 8, 3)
    with pytest.raises(ValueError):
        decode_image(b"123", "application/octet-stream", (4, 4, 3))
