"""The shipped server's control plane sharded by GPU (runtime/worker_pool.py ShardedWorkerPool): launch the platform
CLI with 4 fake-GPU (CPU) workers and 2 native ingest front-ends, drive it over HTTP, and check that

* every pool endpoint runs one scheduler shard per device (its own dispatch queue ``<queue>-s<k>``),
* the front-ends and the gateway spread tasks over the shards (a task id's last hex digit names its shard),
* every task id returned by either ingest path resolves from the gateway (status, result) without a broadcast.
"""
import os
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np
import pytest
import requests

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

YAML = """
settings:
  max_batch_delay_ms: 1.0
  frontend_processes: 2
  frontend_ring_slots: 64
  queue_logger_period_s: 0.5
endpoints:
  tiny:
    path: /v1/ai4e/tiny/classify
    factory: aiforearth_api_platform_amd.models.toy:tiny_classifier
    item_shape: [4, 4, 3]
    max_batch: 8
    topk: 2
    devices: [cpu, cpu, cpu, cpu]
    mode: pool
    hip_graphs: false
routes:
  - {prefix: /v1/tiny/async, mode: async, backend: "inproc:tiny"}
  - {prefix: /v1/tiny/sync, mode: sync, backend: "inproc:tiny"}
"""


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _native_available():
    sys.path.insert(0, ROOT)
    from aiforearth_api_platform_amd.runtime import native_frontend

    return native_frontend.available()


@pytest.mark.skipif(not _native_available(), reason="ai4e_ingestd not buildable here")
def test_sharded_serve_four_workers_every_task_resolvable():
    port = _port()
    with tempfile.NamedTemporaryFile("w", suffix=".yaml", delete=False) as f:
        f.write(YAML)
        cfg = f.name
    env = dict(os.environ, PYTHONPATH=ROOT, AI4E_MAX_QUEUE_MS="0")  # (resolvability, not load refusals, is tested)
    proc = subprocess.Popen([sys.executable, "-m", "aiforearth_api_platform_amd.serve", "--config", cfg, "--port",
                             str(port)], cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    base = f"http://127.0.0.1:{port}"
    try:
        for _ in range(900):
            try:
                if requests.get(base + "/", timeout=1).status_code == 200:
                    break
            except requests.ConnectionError:
                time.sleep(0.1)
        else:
            raise AssertionError("server did not come up")
        time.sleep(1.0)  # the front-ends bind the shared port
        img = np.zeros((4, 4, 3), np.uint8)
        img[..., 2] = 50
        ids = []
        s = requests.Session()
        for _ in range(40):  # single payloads (front-end or gateway, whichever the kernel picks)
            r = s.post(base + "/v1/tiny/async", data=img.tobytes(), headers={"Content-Type": "application/octet-stream"})
            assert r.status_code == 200, r.text
            ids.append(r.json()["TaskId"])
        batch = np.broadcast_to(img, (6, 4, 4, 3)).tobytes()
        for _ in range(10):  # binary batches
            r = s.post(base + "/v1/tiny/async", data=batch, headers={"Content-Type": "application/x-ai4e-batch"})
            assert r.status_code == 200, r.text
            ids += r.json()["TaskIds"]
        assert len(set(ids)) == len(ids) == 100
        # ids are minted in their shard's task-store lock domain: 4 shards of an 8-way store own digits {k, k+4, ..}
        shards = {int(t[-1], 16) % 4 for t in ids}
        assert len(shards) >= 3, shards
        deadline = time.time() + 90
        done = set()
        while time.time() < deadline and len(done) < len(ids):
            for t in ids:
                if t in done:
                    continue
                r = s.get(f"{base}/v1/taskmanagement/task/{t}")
                assert r.status_code == 200, (t, r.status_code)
                if r.json()["BackendStatus"] == "completed":
                    done.add(t)
            time.sleep(0.05)
        assert len(done) == len(ids), f"{len(done)} of {len(ids)} completed"
        for t in ids[::7]:
            res = s.get(f"{base}/v1/taskmanagement/task/{t}/result").json()["Result"]
            assert res["classes"][0] == 2
        r = s.post(base + "/v1/tiny/sync", data=img.tobytes())
        assert r.status_code == 200 and r.json()["classes"][0] == 2
        stats = s.get(base + "/v1/platform/stats").json() if s.get(base + "/v1/platform/stats").status_code == 200 \
            else None
        if stats is not None:
            qnames = " ".join(map(str, stats.get("control_plane", stats).get("queues", {}).keys())) \
                if isinstance(stats, dict) else ""
            if qnames:
                assert "-s3" in qnames, qnames
    finally:
        proc.terminate()
        try:
            out, _ = proc.communicate(timeout=20)
        except subprocess.TimeoutExpired:
            proc.kill()
            out, _ = proc.communicate()
        os.unlink(cfg)
    assert b"Traceback" not in out, out.decode(errors="replace")[-3000:]


def test_sharded_pool_layout_cpu():
    """In process: 4 shards over 4 CPU 'devices', disjoint ring partitions, one queue each, ids owned per shard."""
    sys.path.insert(0, ROOT)
    from aiforearth_api_platform_amd.config import Config
    from aiforearth_api_platform_amd.gateway.control import ControlPlane
    from aiforearth_api_platform_amd.runtime.worker_pool import ModelSpec, ShardedWorkerPool

    cp = ControlPlane(Config.load(env={}))
    spec = ModelSpec("aiforearth_api_platform_amd.models.toy:tiny_classifier", (4, 4, 3), 8, 2, {}, False)
    pool = ShardedWorkerPool(cp, "http://127.0.0.1/v1/ai4e/tiny/classify", spec, ["cpu"] * 4, frontends=2,
                             frontend_slots=16)
    try:
        assert len(pool.control_shards) == 4
        parts = [(p.ring.base, p.ring.length) for p in pool.control_shards]
        parts += [(b, n) for p in pool.control_shards for b, n, _ in p.frontend_partitions]
        parts.sort()
        for (b0, n0), (b1, _) in zip(parts, parts[1:]):
            assert b0 + n0 <= b1, parts
        assert parts[-1][0] + parts[-1][1] <= pool.ring.nslots
        assert len({id(p.queue) for p in pool.control_shards}) == 4
        assert sorted(cp.queues()) == sorted({p.queue.name for p in pool.control_shards} | set(cp.queues()))
        pool.start(wait_ready_s=120)
        imgs = np.zeros((24, 4, 4, 3), np.uint8)
        ids = []
        for _ in range(4):
            ids += pool.submit_many(imgs)
        by_shard = {}
        for t in ids:
            by_shard.setdefault(cp.store.shard_index(t) % 4, []).append(t)
        assert len(by_shard) == 4, {k: len(v) for k, v in by_shard.items()}
        deadline = time.time() + 60
        while time.time() < deadline and pool.images < len(ids):
            time.sleep(0.02)
        assert pool.images == len(ids)
        assert all(pool.result(t)["classes"] for t in ids[::5])
        st = pool.stats()
        assert st["control_plane_shards"] == 4 and len(st["workers"]) == 4
        assert pool.queue.stats()["ready"] == 0
    finally:
        pool.stop()
        cp.close()
