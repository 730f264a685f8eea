"""JPEG frames prepared into payload-ring slots (runtime/jpeg_gpu.py, runtime/model_endpoint.py, runtime/engine.py,
runtime/gpu_worker.py): the front-end parses the headers and copies the entropy-coded bytes into the request's slot and
marks it with the ring's key; the worker decodes marked slots into the model input (on the GPU; on CPU workers with the
kernels' span decoder run sequentially + the numpy reconstruction, which is what runs here).

* the ring's key lives in the segment's tail; a raw payload (which fills its slot) is never taken for a prepared one;
* the CPU decode of a prepared frame is bit-exact to ``decode_image`` (the CPU path the endpoints use);
* through a worker pool, a JPEG request gives exactly the result of the same frame decoded on the CPU and submitted as
  pixels; a prepared frame whose entropy-coded data is cut short fails its task as an invalid payload; frames outside the
  GPU envelope (progressive) are decoded by the front-end as before.
"""
import io
import json
import time

import numpy as np
import pytest
from PIL import Image

from aiforearth_api_platform_amd import _ai4e_core as core
from aiforearth_api_platform_amd.config import Config
from aiforearth_api_platform_amd.gateway.control import ControlPlane
from aiforearth_api_platform_amd.runtime import jpeg_gpu as jg
from aiforearth_api_platform_amd.runtime.decode import decode_image
from aiforearth_api_platform_amd.runtime.model_endpoint import ModelEndpoint
from aiforearth_api_platform_amd.runtime.worker_pool import ModelSpec, SharedPayloadRing, WorkerPool

SHAPE = (192, 256, 3)  # (the slot must hold the 18.7 KB header + the frame's scan)


def frame(h, w, q=90, seed=0, **kw):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (max(h // 8, 1), max(w // 8, 1), 3), dtype=np.uint8)
    b = io.BytesIO()
    Image.fromarray(base).resize((w, h), Image.BILINEAR).save(b, "JPEG", quality=q, **kw)
    return b.getvalue()


def test_ring_tail_key_and_slot_marks():
    on = SharedPayloadRing(4, SHAPE, jpeg_slots=True)
    off = SharedPayloadRing(4, SHAPE, jpeg_slots=False)
    try:
        item = int(np.prod(SHAPE))
        assert on.jpeg_key != 0 and off.jpeg_key == 0
        assert jg.ring_key(on.shm.buf, 4 * item) == on.jpeg_key
        body = frame(480, 640)
        assert jg.prepare_into_slot(body, on.buf[1].data_ptr(), item, SHAPE, on.jpeg_key)
        on.buf[2].copy_(on.buf[1])  # a raw payload that happens to equal a prepared slot's first bytes ...
        on.buf[2].view(-1)[-jg.TRAILER_BYTES:] = 7  # ... but fills the slot, trailer included
        u8 = on.buf.view(4, -1).numpy()
        frames = jg.slot_frames(u8, [0, 1, 2, 3], on.jpeg_key)
        assert [j for j, _ in frames] == [1]
        assert jg.slot_frames(u8, [1], on.jpeg_key ^ 1) == []  # another ring's key
        hdr = jg.parse_header(u8[1, :160].tobytes())
        assert jg.header_sane(hdr, frames[0][1])
        assert not jg.header_sane(dict(hdr, nblocks=hdr["nblocks"] + 1), frames[0][1])
        assert not jg.header_sane(hdr, 1000)
        # progressive / too large for the slot: left to the CPU decoder
        assert not jg.prepare_into_slot(frame(480, 640, progressive=True), on.buf[0].data_ptr(), item, SHAPE,
                                        on.jpeg_key)
        assert not jg.prepare_into_slot(frame(1200, 1600, q=98), on.buf[0].data_ptr(), item, SHAPE, on.jpeg_key)
        assert not jg.prepare_into_slot(body, on.buf[0].data_ptr(), item, SHAPE, 0)
    finally:
        on.close()
        off.close()


@pytest.mark.parametrize("hw,shape", [((480, 640), SHAPE), ((480, 640), (224, 224, 3)), ((300, 400), (300, 400, 3))])
def test_prepared_cpu_decode_bit_exact(hw, shape):
    body = frame(*hw, seed=hw[0])
    buf = np.zeros(4 << 20, np.uint8)
    st, used = core.jpeg_scan_prepare(body, buf.ctypes.data, buf.nbytes)
    assert st == 0
    got = jg.decode_prepared_cpu(buf[:used], shape)
    if hw == (300, 400) and shape[:2] == hw:  # 4:2:0 at full scale needs upsampling: outside the plan
        assert got is None
        return
    np.testing.assert_array_equal(got, decode_image(body, "image/jpeg", shape))


def _wait(cond, t=120.0):
    d = time.time() + t
    while time.time() < d:
        if cond():
            return True
        time.sleep(0.02)
    return False


def test_jpeg_requests_through_a_worker_pool():
    cp = ControlPlane(Config.load(env={}))
    spec = ModelSpec("aiforearth_api_platform_amd.models.toy:tiny_classifier", SHAPE, max_batch=8, topk=6,
                     use_graphs=False)
    pool = WorkerPool(cp, "http://127.0.0.1/v1/jpg/classify", spec, ["cpu"], max_delay_s=0.001, jpeg_slots=True)
    ep = ModelEndpoint(cp, "/v1/jpg/classify", worker=pool)
    try:
        pool.start(wait_ready_s=120)
        bodies = [frame(480, 640, seed=s) for s in range(3)]
        cut = frame(480, 640, seed=9)
        bad = cut[:len(cut) // 2] + b"\xff\xd9"  # entropy-coded data cut short (PIL: "image file is truncated")
        prog = frame(480, 640, seed=5, progressive=True)
        jpeg_ids = [json.loads(ep.submit(b, "image/jpeg"))["TaskId"] for b in bodies + [bytes(bad), prog]]
        raw_ids = ep.submit_many(np.stack([decode_image(b, "image/jpeg", SHAPE) for b in bodies + [prog]]))
        assert _wait(lambda: all(cp.store.get_record(t)["BackendStatus"] in ("completed", "failed")
                                 for t in jpeg_ids + raw_ids))
        for a, b in zip(jpeg_ids[:3] + jpeg_ids[4:], raw_ids):
            ra, rb = ep.result(a), ep.result(b)
            assert ra is not None and ra == rb, (ra, rb)
        rec = cp.store.get_record(jpeg_ids[3])
        assert rec["BackendStatus"] == "failed", rec
    finally:
        ep.stop()
        cp.close()


def test_native_frontend_prepares_jpeg_into_slots(tmp_path):
    """A native front-end (csrc/ingest/ingestd.cpp) takes a JPEG POST straight into a ring slot (headers + scan, the
    ring's key in the trailer); a progressive JPEG goes to the serving process with its body and is decoded there.
    Both give the result of the same frame decoded on the CPU and posted as pixels."""
    import os
    import socket
    import subprocess
    import sys

    import requests
    import yaml

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    doc = yaml.safe_load(open(os.path.join(root, "examples", "platform_cpu.yaml")))
    doc["endpoints"]["tiny"].update(item_shape=list(SHAPE), topk=6, devices=["cpu"])
    doc["routes"] = [{"prefix": "/v1/tiny/async", "mode": "async", "backend": "inproc:tiny"}]
    cfgp = tmp_path / "platform.yaml"
    cfgp.write_text(yaml.safe_dump(doc))
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ, PYTHONPATH=root, AI4E_FRONTEND_PROCESSES="1", AI4E_FRONTEND_IMPL="native",
               AI4E_JPEG_SLOTS="1")
    proc = subprocess.Popen([sys.executable, "-m", "aiforearth_api_platform_amd.serve", "--config", str(cfgp),
                             "--port", str(port)], cwd=root, env=env, stdout=subprocess.DEVNULL,
                            stderr=subprocess.DEVNULL)
    base = f"http://127.0.0.1:{port}"
    s = requests.Session()
    s.trust_env = False
    try:
        for _ in range(600):
            try:
                if s.get(base + "/", timeout=1).status_code == 200:
                    break
            except requests.ConnectionError:
                time.sleep(0.1)
        else:
            raise AssertionError("server did not come up")
        time.sleep(2.0)
        bodies = [frame(480, 640, seed=s_) for s_ in range(3)] + [frame(480, 640, seed=7, progressive=True)]
        pairs = []
        for b in bodies:
            r1 = s.post(base + "/v1/tiny/async", data=b, headers={"Content-Type": "image/jpeg"})
            r2 = s.post(base + "/v1/tiny/async", data=decode_image(b, "image/jpeg", SHAPE).tobytes(),
                        headers={"Content-Type": "application/octet-stream"})
            assert r1.status_code == 200 and r2.status_code == 200, (r1.text, r2.text)
            assert r1.headers.get("Server", "").startswith("ai4e-ingestd")
            pairs.append((r1.json()["TaskId"], r2.json()["TaskId"]))

        # a client that waits for 100-continue before its body, on a body the front-end proxies (progressive JPEG)
        import socket as _socket

        prog = bodies[-1]
        with _socket.create_connection(("127.0.0.1", port), timeout=30) as so:
            so.sendall((f"POST /v1/tiny/async HTTP/1.1\r\nHost: x\r\nContent-Type: image/jpeg\r\n"
                        f"Content-Length: {len(prog)}\r\nExpect: 100-continue\r\n\r\n").encode())
            head = so.recv(4096)
            assert head.startswith(b"HTTP/1.1 100"), head
            so.sendall(prog)
            resp = b""
            while b"\r\n\r\n" not in resp:
                resp += so.recv(65536)
            assert resp.startswith(b"HTTP/1.1 200"), resp[:200]

        def result(t):
            r = s.get(f"{base}/v1/taskmanagement/task/{t}/result")
            return r.json().get("Result") if r.status_code == 200 else None

        assert _wait(lambda: all(result(a) is not None and result(b) is not None for a, b in pairs), 120)
        for a, b in pairs:
            assert result(a) == result(b)
    finally:
        proc.terminate()
        try:
            proc.wait(20)
        except subprocess.TimeoutExpired:
            proc.kill()
