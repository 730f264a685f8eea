"""End-to-end: launch the platform CLI (CPU config) as a process, drive it over real HTTP."""
import os
import socket
import subprocess
import sys
import time

import numpy as np
import requests

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_platform_cli_end_to_end():
    port = _port()
    env = dict(os.environ, PYTHONPATH=ROOT)
    proc = subprocess.Popen([sys.executable, "-m", "aiforearth_api_platform_amd.serve", "--config",
                             os.path.join(ROOT, "examples", "platform_cpu.yaml"), "--port", str(port)],
                            cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    base = f"http://127.0.0.1:{port}"
    try:
        for _ in range(600):
            try:
                if requests.get(base + "/", timeout=1).status_code == 200:
                    break
            except requests.ConnectionError:
                time.sleep(0.1)
        else:
            raise AssertionError("server did not come up")
        img = np.zeros((4, 4, 3), np.uint8)
        img[..., 2] = 50
        ids = []
        for _ in range(20):
            r = requests.post(base + "/v1/tiny/async", data=img.tobytes(),
                              headers={"Content-Type": "application/octet-stream"})
            assert r.status_code == 200
            ids.append(r.json()["TaskId"])
        deadline = time.time() + 60
        done = set()
        while time.time() < deadline and len(done) < len(ids):
            for t in ids:
                if t not in done and requests.get(f"{base}/v1/taskmanagement/task/{t}").json()["BackendStatus"] == \
                        "completed":
                    done.add(t)
            time.sleep(0.05)
        assert len(done) == len(ids)
        res = requests.get(f"{base}/v1/taskmanagement/task/{ids[0]}/result").json()["Result"]
        assert res["classes"][0] == 2
        r = requests.post(base + "/v1/tiny/sync", data=img.tobytes())
        assert r.status_code == 200 and r.json()["classes"][0] == 2
        assert requests.post(base + "/v1/echo", data=b"hello").content == b"hello"
        t = requests.post(base + "/v1/generic", json={"x": 1}).json()
        for _ in range(100):
            if requests.get(f"{base}/v1/taskmanagement/task/{t['TaskId']}").json()["BackendStatus"] != "created":
                break
            time.sleep(0.05)
        # generic async backends are delivered by the queue dispatcher (BackendQueueProcessor); echo returns 200
        assert "tiny" in requests.get(base + "/metrics").text
    finally:
        proc.terminate()
        try:
            proc.wait(20)
        except subprocess.TimeoutExpired:
            proc.kill()
