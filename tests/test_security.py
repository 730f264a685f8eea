"""Gateway security surface (gateway/security.py): APIM-style subscription keys (global and per route), the
OpenAPI description of the route table, and the HTTPS listener — in process, and through the platform CLI with
an ingest front-end process sharing the TLS port (the same requests must get the same answers whichever
process accepts the connection)."""
import asyncio
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest
import requests
import yaml
from aiohttp.test_utils import TestClient, TestServer

from aiforearth_api_platform_amd.config import Config
from aiforearth_api_platform_amd.gateway.control import ControlPlane
from aiforearth_api_platform_amd.gateway.security import KEY_HEADER, INVALID_KEY, MISSING_KEY, KeyAuth
from aiforearth_api_platform_amd.gateway.server import Gateway, Route, RouteTable

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CERT = os.path.join(ROOT, "tests", "fixtures", "tls_test_cert.pem")
KEY = os.path.join(ROOT, "tests", "fixtures", "tls_test_key.pem")


def run(coro):
    return asyncio.new_event_loop().run_until_complete(coro)


def _echo(task_id, body, headers):
    return 200, {"echo": json.loads(body or b"null")}


def _gateway(global_keys, control_keys=""):
    cp = ControlPlane(Config.load(env={}, subscription_keys=global_keys, control_keys=control_keys))
    t = RouteTable()
    t.add(Route("/v1/echo", "sync", _echo, content_types=["application/json"], keys=["route-key"]))
    t.add(Route("/v1/open", "sync", _echo))
    t.add(Route("/v1/generic/async", "async", None, rewrite="/v1/backend/generic"))
    return cp, Gateway(cp, t)


def test_key_auth_unit():
    a = KeyAuth(["g1", "g2"])
    assert a.check({}, {})[0] == 401 and a.check({}, {})[1]["message"] == MISSING_KEY
    assert a.check({KEY_HEADER: "nope"}, {})[1]["message"] == INVALID_KEY
    assert a.check({KEY_HEADER: "g2"}, {}) is None
    assert a.check({}, {"subscription-key": "g1"}) is None
    assert a.check({KEY_HEADER: "r"}, {}, route_keys=["r"]) is None
    assert KeyAuth([]).check({}, {}) is None
    assert KeyAuth([]).check({}, {}, route_keys=["r"])[0] == 401


def test_gateway_keys_global_and_per_route():
    cp, gw = _gateway("gk")

    async def go():
        c = TestClient(TestServer(gw.app))
        await c.start_server()
        try:
            assert (await c.get("/")).status == 200                       # health stays open
            assert (await c.get("/openapi.json")).status == 200           # so does the API description
            r = await c.get("/v1/taskmanagement/task/abc")
            assert r.status == 401 and (await r.json())["message"] == MISSING_KEY
            r = await c.get("/v1/taskmanagement/task/abc", headers={KEY_HEADER: "bad"})
            assert r.status == 401 and (await r.json())["message"] == INVALID_KEY
            assert (await c.get("/v1/taskmanagement/task/abc", headers={KEY_HEADER: "gk"})).status == 204
            assert (await c.get("/v1/taskmanagement/task/abc?subscription-key=gk")).status == 204
            body = json.dumps({"a": 1})
            hdr = {"Content-Type": "application/json"}
            assert (await c.post("/v1/echo", data=body, headers=hdr)).status == 401
            for k in ("gk", "route-key"):  # the global key and the route's own key both open the route
                r = await c.post("/v1/echo", data=body, headers=dict(hdr, **{KEY_HEADER: k}))
                assert r.status == 200 and (await r.json()) == {"echo": {"a": 1}}
            # a route key opens only its route
            assert (await c.post("/v1/open", data=body, headers={KEY_HEADER: "route-key"})).status == 401
            assert (await c.get("/metrics")).status == 401
            assert (await c.get("/metrics", headers={KEY_HEADER: "gk"})).status == 200
            # async generic route: key first, then the usual task creation
            r = await c.post("/v1/generic/async", data=body, headers={KEY_HEADER: "gk"})
            assert r.status == 200 and (await r.json())["BackendStatus"] == "created"
            # upstream taskId header must be printable ASCII (the scheduler wire carries fixed-length byte ids)
            r = await c.post("/v1/generic/async", data=body, headers={KEY_HEADER: "gk", "taskId": "x" * 200})
            assert r.status == 400
        finally:
            await c.close()

    run(go())
    cp.close()


def test_route_keys_without_global_keys():
    """Per-route keys only: unkeyed routes stay open, but the task-management routes want a key (any route's) and
    the control routes (the reference's key-protected Function endpoints) open to no route key."""
    cp, gw = _gateway("")

    async def go():
        c = TestClient(TestServer(gw.app))
        await c.start_server()
        try:
            body, hdr = json.dumps({"b": 2}), {"Content-Type": "application/json"}
            assert (await c.post("/v1/open", data=body, headers=hdr)).status == 200
            assert (await c.get("/v1/taskmanagement/task/abc")).status == 401
            assert (await c.get("/v1/taskmanagement/task/abc", headers={KEY_HEADER: "route-key"})).status == 204
            assert (await c.post("/v1/echo", data=body, headers=hdr)).status == 401
            assert (await c.post("/v1/echo", data=body, headers=dict(hdr, **{KEY_HEADER: "route-key"}))).status == 200
            upsert = json.dumps({"TaskId": "", "Status": "created", "BackendStatus": "created",
                                 "Endpoint": "http://h/v1/x", "Body": "", "PublishToGrid": False})
            for h in ({}, {KEY_HEADER: "route-key"}):
                assert (await c.post("/v1/cache/upsert", data=upsert, headers=h)).status == 401
                assert (await c.get("/v1/cache/get", params={"taskId": "abc"}, headers=h)).status == 401
                assert (await c.post("/v1/backend/webhook", data="[]", headers=h)).status == 401
                assert (await c.post("/v1/requests/upsert", data="{}", headers=h)).status == 401
        finally:
            await c.close()

    run(go())
    cp.close()


def test_control_keys_open_control_routes():
    cp, gw = _gateway("", control_keys="ck")

    async def go():
        c = TestClient(TestServer(gw.app))
        await c.start_server()
        try:
            upsert = json.dumps({"TaskId": "", "Status": "created", "BackendStatus": "created",
                                 "Endpoint": "http://h/v1/x", "Body": "", "PublishToGrid": False})
            assert (await c.post("/v1/cache/upsert", data=upsert)).status == 401
            assert (await c.post("/v1/cache/upsert", data=upsert, headers={KEY_HEADER: "route-key"})).status == 401
            r = await c.post("/v1/cache/upsert", data=upsert, headers={KEY_HEADER: "ck"})
            assert r.status == 200
            tid = (await r.json())["TaskId"]
            assert (await c.get(f"/v1/taskmanagement/task/{tid}", headers={KEY_HEADER: "ck"})).status == 200
            assert (await c.get("/metrics", headers={KEY_HEADER: "ck"})).status == 200
            assert (await c.get("/metrics")).status == 401
        finally:
            await c.close()

    run(go())
    cp.close()


def test_openapi_lists_every_route():
    cp, gw = _gateway("gk")

    async def go():
        c = TestClient(TestServer(gw.app))
        await c.start_server()
        try:
            return await (await c.get("/openapi.json")).json()
        finally:
            await c.close()

    doc = run(go())
    cp.close()
    assert doc["openapi"].startswith("3.")
    for r in gw.routes.routes:
        assert r.prefix in doc["paths"] and "post" in doc["paths"][r.prefix]
    for p in ("/v1/taskmanagement/task/{taskId}", "/v1/taskmanagement/task/{taskId}/result",
              "/v1/taskmanagement/task/{taskId}/trace", "/"):
        assert p in doc["paths"]
    assert doc["paths"]["/v1/echo"]["post"]["x-ai4e"]["mode"] == "sync"
    assert "application/json" in doc["paths"]["/v1/echo"]["post"]["requestBody"]["content"]
    assert doc["components"]["securitySchemes"]["subscriptionKey"]["name"] == KEY_HEADER
    task = doc["components"]["schemas"]["APITask"]["properties"]
    assert list(task) == ["TaskId", "Timestamp", "Status", "BackendStatus", "Endpoint", "Body", "PublishToGrid",
                          "EndpointPath"]


def _port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_https_platform_with_frontend_parity(tmp_path):
    """serve.py with a TLS certificate, a global key, a keyed route and one ingest front-end on the same port:
    a TLS round trip per request (fresh connection each, so requests land on either process), and every
    request class gets the same status on both paths."""
    doc = yaml.safe_load(open(os.path.join(ROOT, "examples", "platform_cpu.yaml")))
    doc["routes"] = [
        {"prefix": "/v1/tiny/async", "mode": "async", "backend": "inproc:tiny", "max_content_length": 4096},
        {"prefix": "/v1/tiny/keyed", "mode": "async", "backend": "inproc:tiny", "keys": ["tiny-key"],
         "content_types": ["application/octet-stream"]},
        {"prefix": "/v1/tiny/sync", "mode": "sync", "backend": "inproc:tiny"},
    ]
    cfgp = tmp_path / "platform.yaml"
    cfgp.write_text(yaml.safe_dump(doc))
    port = _port()
    env = dict(os.environ, PYTHONPATH=ROOT, AI4E_FRONTEND_PROCESSES="1", AI4E_TLS_CERT=CERT, AI4E_TLS_KEY=KEY,
               AI4E_SUBSCRIPTION_KEYS="gk")
    proc = subprocess.Popen([sys.executable, "-m", "aiforearth_api_platform_amd.serve", "--config", str(cfgp),
                             "--port", str(port)], cwd=ROOT, env=env, stdout=open(tmp_path / "serve.log", "w"),
                            stderr=subprocess.STDOUT)
    base = f"https://127.0.0.1:{port}"
    s = requests.Session()
    s.verify = CERT
    s.trust_env = False  # (a CA bundle from the environment would override the session's verify)
    try:
        deadline = time.time() + 240
        while True:
            try:
                if s.get(base + "/", timeout=1).status_code == 200:
                    break
            except requests.exceptions.ConnectionError:
                time.sleep(0.2)
            if time.time() > deadline:
                raise AssertionError("server did not come up: " + (tmp_path / "serve.log").read_text()[-2000:])
        time.sleep(3.0)  # the front-end's interpreter starts and binds the shared port
        with pytest.raises(requests.exceptions.SSLError):  # clients that do not trust the cert are refused
            requests.get(base + "/", timeout=5, verify=True)
        img = np.zeros((4, 4, 3), np.uint8)
        img[..., 2] = 90
        ob = {"Content-Type": "application/octet-stream", "Connection": "close"}
        cases = [  # (path, headers, body, expected status)
            ("/v1/tiny/async", ob, img.tobytes(), 401),
            ("/v1/tiny/async", dict(ob, **{KEY_HEADER: "wrong"}), img.tobytes(), 401),
            ("/v1/tiny/async", dict(ob, **{KEY_HEADER: "gk"}), img.tobytes(), 200),
            ("/v1/tiny/async", dict(ob, **{KEY_HEADER: "gk"}), b"\x00" * 5000, 413),
            ("/v1/tiny/keyed", dict(ob, **{KEY_HEADER: "tiny-key"}), img.tobytes(), 200),
            ("/v1/tiny/keyed", dict(ob, **{KEY_HEADER: "gk", "Content-Type": "image/png"}), img.tobytes(), 401),
        ]
        ids = []
        for _ in range(6):  # fresh connections: the kernel spreads them over the two listeners
            for path, hdr, body, want in cases:
                r = s.post(base + path, data=body, headers=hdr)
                assert r.status_code == want, (path, hdr, r.status_code, r.text)
                if want == 200:
                    ids.append(r.json()["TaskId"])
        deadline = time.time() + 60
        pending = set(ids)
        while pending and time.time() < deadline:
            for t in list(pending):
                r = s.get(f"{base}/v1/taskmanagement/task/{t}", headers={KEY_HEADER: "gk", "Connection": "close"})
                if r.status_code == 200 and r.json()["BackendStatus"] == "completed":
                    pending.discard(t)
            time.sleep(0.05)
        assert not pending
        r = s.get(f"{base}/v1/taskmanagement/task/{ids[0]}/result", headers={KEY_HEADER: "gk"})
        assert r.json()["Result"]["classes"][0] == 2
        assert s.get(f"{base}/v1/taskmanagement/task/{ids[0]}").status_code == 401
        doc = s.get(base + "/openapi.json").json()
        assert "/v1/tiny/keyed" in doc["paths"] and doc["servers"][0]["url"].startswith("https://")
    finally:
        proc.terminate()
        try:
            proc.wait(20)
        except subprocess.TimeoutExpired:
            proc.kill()


def test_gateway_refuses_oversized_declared_length():
    """A declared Content-Length above the route's max_content_length — or, with none set, above the global 1 GiB
    body cap — is answered 413 from the headers, before any of the body is read (the native front-end's rule)."""
    cp, gw = _gateway("")

    async def go():
        c = TestClient(TestServer(gw.app))
        await c.start_server()
        try:
            r, w = await asyncio.open_connection("127.0.0.1", c.server.port)
            w.write(b"POST /v1/open HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
                    b"Content-Length: 999999999999\r\n\r\n")
            await w.drain()
            head = await asyncio.wait_for(r.readline(), 10)
            w.close()
            assert b" 413 " in head
            ok = await c.post("/v1/open", data=json.dumps({"a": 1}), headers={"Content-Type": "application/json"})
            assert ok.status == 200
        finally:
            await c.close()

    run(go())
    cp.close()
