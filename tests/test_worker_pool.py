"""Multi-process worker pool on CPU: batching across workers, fail-over requeue, restart, elastic resize."""
import time

import numpy as np
import pytest

from aiforearth_api_platform_amd.config import Config
from aiforearth_api_platform_amd.gateway.control import ControlPlane
from aiforearth_api_platform_amd.runtime.worker_pool import ModelSpec, WorkerPool

SPEC = ModelSpec("aiforearth_api_platform_amd.models.toy:tiny_classifier", (4, 4, 3), max_batch=8, topk=2,
                 use_graphs=False)
EP = "http://127.0.0.1/v1/ai4e/tiny/classify"


def _wait(cond, t=60):
    d = time.time() + t
    while time.time() < d:
        if cond():
            return True
        time.sleep(0.02)
    return False


def _imgs(n):
    a = np.zeros((n, 4, 4, 3), np.uint8)
    a[np.arange(n), :, :, np.arange(n) % 3] = 100
    return a


@pytest.fixture
def cp():
    c = ControlPlane(Config.load(env={}, max_delivery_count=5))
    yield c
    c.close()


def test_pool_two_workers_complete_all(cp):
    pool = WorkerPool(cp, EP, SPEC, ["cpu", "cpu"], heartbeat_interval_s=0.1).start()
    try:
        ids = pool.submit_many(_imgs(40))
        assert _wait(lambda: cp.store.zcard("/v1/ai4e/tiny/classify_completed") == 40)
        for i, t in enumerate(ids):
            assert pool.result(t)["classes"][0] == i % 3
        pool.refresh()
        assert sum(1 for w in pool.workers if w.batches > 0) >= 1
    finally:
        pool.stop()


def test_pool_worker_crash_requeues_and_restarts(cp, monkeypatch):
    monkeypatch.setenv("AI4E_FAULT_INJECTION", "exit_after=1@0")
    pool = WorkerPool(cp, EP, SPEC, ["cpu", "cpu"], heartbeat_interval_s=0.1, max_restarts=1).start()
    try:
        pool.submit_many(_imgs(64))
        assert _wait(lambda: cp.store.zcard("/v1/ai4e/tiny/classify_completed") == 64, 120)
        ev = [e for _, e, r in pool.events]
        assert "worker_failed" in ev
    finally:
        pool.stop()


def test_pool_hung_worker_heartbeat_timeout(cp, monkeypatch):
    monkeypatch.setenv("AI4E_FAULT_INJECTION", "hang_after=0@1,delay_ms=100@0")
    pool = WorkerPool(cp, EP, SPEC, ["cpu", "cpu"], heartbeat_interval_s=0.1, heartbeat_timeout_s=1.0,
                      max_restarts=0).start()
    try:
        assert _wait(lambda: all(w.ready for w in pool.workers))
        pool.submit_many(_imgs(32))
        assert _wait(lambda: cp.store.zcard("/v1/ai4e/tiny/classify_completed") == 32, 120)
        # "removed" follows the kill + join of the hung process, which may end after the requeued tasks complete
        assert _wait(lambda: any(e == "removed" and r == 1 for _, e, r in pool.events), 30), pool.events
    finally:
        pool.stop()


def test_pool_elastic_resize(cp):
    pool = WorkerPool(cp, EP, SPEC, ["cpu"], heartbeat_interval_s=0.1).start()
    try:
        pool.submit_many(_imgs(8))
        assert _wait(lambda: cp.store.zcard("/v1/ai4e/tiny/classify_completed") == 8)
        pool.resize(2)
        assert _wait(lambda: sum(w.ready for w in pool.workers if not w.stop.is_set()) == 2)
        pool.submit_many(_imgs(24))
        assert _wait(lambda: cp.store.zcard("/v1/ai4e/tiny/classify_completed") == 32)
        pool.resize(1)
        pool.submit_many(_imgs(8))
        assert _wait(lambda: cp.store.zcard("/v1/ai4e/tiny/classify_completed") == 40)
    finally:
        pool.stop()
