"""Competing consumers across control-plane shards (runtime/worker_pool.py ShardedWorkerPool + csrc/core/scheduler.h
``set_peers``): any live worker finishes any queued task, as every replica of the reference consumes the one Service
Bus queue of its API (``ProcessManager/BackendQueueProcessor/BackendQueueProcessor.cs:54-64``, ``host.json:3-11``).

* a shard whose only worker dies for good (restarts exhausted) has its queue drained by the other shards, every task
  completes exactly once;
* shrinking the pool below one worker per shard (4 -> 2) under load loses no task;
* a sharded sync endpoint with a journal (explicit-upsert ids in any lock domain) answers every request;
* the shard's published load counters return to zero backlog once the work is done (every terminal outcome counts).
"""
import json
import os
import tempfile
import threading
import time

import numpy as np
import pytest

from aiforearth_api_platform_amd.config import Config
from aiforearth_api_platform_amd.gateway.control import ControlPlane
from aiforearth_api_platform_amd.runtime.worker_pool import ModelSpec, ShardedWorkerPool

SPEC = ModelSpec("aiforearth_api_platform_amd.models.toy:tiny_classifier", (4, 4, 3), max_batch=8, topk=2,
                 use_graphs=False)
EP = "http://127.0.0.1/v1/ai4e/tiny/classify"
DONE_INDEX = "/v1/ai4e/tiny/classify_completed"


def _wait(cond, t=90.0):
    d = time.time() + t
    while time.time() < d:
        if cond():
            return True
        time.sleep(0.02)
    return False


def _imgs(n, off=0):
    a = np.zeros((n, 4, 4, 3), np.uint8)
    a[np.arange(n), :, :, (np.arange(n) + off) % 3] = 100
    return a


@pytest.fixture
def cp():
    c = ControlPlane(Config.load(env={}, max_delivery_count=10))
    yield c
    c.close()


def _submit_spread(pool, total, chunk):
    ids = []
    for i in range(0, total, chunk):
        ids += pool.submit_many(_imgs(min(chunk, total - i), i))
    return ids


def test_dead_shard_drained_by_peers(cp, monkeypatch):
    # every batch takes 15 ms, so 1000 tasks are still queued on every shard when shard 1's worker dies
    monkeypatch.setenv("AI4E_FAULT_INJECTION", "delay_ms=15")
    pool = ShardedWorkerPool(cp, EP, SPEC, ["cpu"] * 4, heartbeat_interval_s=0.1, max_restarts=0, frontends=1,
                             frontend_slots=8, ring_slots=400)
    try:
        pool.start(wait_ready_s=120)
        assert [p.sched.live_workers() for p in pool.pools] == [1, 1, 1, 1]
        ids = _submit_spread(pool, 1000, 40)
        shard_of = {t: cp.store.shard_index(t) % 4 for t in ids}
        assert sorted(set(shard_of.values())) == [0, 1, 2, 3]
        assert pool.pools[1].queue.depth() > 0  # work is queued on the shard about to lose its worker
        victim = pool.pools[1].workers[0]
        victim.proc.kill()
        assert _wait(lambda: any(e == "removed" for _, e, _ in pool.pools[1].events), 30), pool.pools[1].events
        assert _wait(lambda: cp.store.zcard(DONE_INDEX) == 1000, 120), cp.store.zcard(DONE_INDEX)
        time.sleep(0.3)
        assert pool.images == 1000  # every task completed exactly once (no duplicate completion)
        assert pool.pools[1].sched.live_workers() == 0
        assert pool.stats()["stolen_items"] > 0
        for i, t in enumerate(ids[::37]):
            rec = json.loads(cp.get(t)[1])
            assert rec["BackendStatus"] == "completed", rec
        for p in pool.pools:  # terminal outcomes balance what was queued, nothing is left in flight
            enq, done, pending, live, inflight = p.sched.stat_counters()[:5]
            assert enq == done and inflight == 0 and pending == 0, (p.shard.index, p.sched.stat_counters())
            assert p.queue.depth() == 0
        # new ingest avoids the dead shard
        more = pool.submit_many(_imgs(16))
        assert all(cp.store.shard_index(t) % 4 != 1 for t in more)
        assert _wait(lambda: cp.store.zcard(DONE_INDEX) == 1016, 60)
    finally:
        pool.stop()


def test_shrink_below_one_worker_per_shard_under_load(cp, monkeypatch):
    monkeypatch.setenv("AI4E_FAULT_INJECTION", "delay_ms=10")
    pool = ShardedWorkerPool(cp, EP, SPEC, ["cpu"] * 4, heartbeat_interval_s=0.1, ring_slots=400)
    try:
        pool.start(wait_ready_s=120)
        ids = _submit_spread(pool, 800, 40)
        pool.resize(2)
        assert pool.active() == 2
        assert sorted(p.sched.live_workers() for p in pool.pools) == [0, 0, 1, 1]
        ids += _submit_spread(pool, 200, 20)
        assert _wait(lambda: cp.store.zcard(DONE_INDEX) == 1000, 120), cp.store.zcard(DONE_INDEX)
        time.sleep(0.2)
        assert pool.images == 1000
        assert len(set(ids)) == 1000
        pool.resize(4)  # and back
        assert _wait(lambda: sum(p.sched.live_workers() for p in pool.pools) == 4, 60)
        pool.submit_many(_imgs(40))
        assert _wait(lambda: cp.store.zcard(DONE_INDEX) == 1040, 60)
    finally:
        pool.stop()


def test_sharded_sync_with_journal_every_waiter_fires():
    from aiforearth_api_platform_amd.runtime.model_endpoint import ModelEndpoint

    with tempfile.TemporaryDirectory() as d:
        cp = ControlPlane(Config.load(env={}, journal_path=os.path.join(d, "j.log")))
        pool = ShardedWorkerPool(cp, EP, SPEC, ["cpu"] * 4, heartbeat_interval_s=0.1)
        ep = ModelEndpoint(cp, "/v1/ai4e/tiny/classify", worker=pool)
        try:
            pool.start(wait_ready_s=120)
            fired, lock = [], threading.Lock()
            ev = threading.Event()
            n = 48

            def cb(t):
                with lock:
                    fired.append(t)
                    if len(fired) == n:
                        ev.set()

            img = _imgs(1)[0].tobytes()
            tids = []
            for i in range(n):
                # half with an upstream taskId (the explicit-upsert path), half journaled payloads
                rec = json.loads(ep.submit(img, task_id=(f"upstream-{i:04d}" if i % 2 else ""), on_done=cb))
                tids.append(rec["TaskId"])
            assert ev.wait(60), f"{len(fired)} of {n} sync waiters fired"
            assert sorted(fired) == sorted(tids)
        finally:
            pool.stop()
            cp.close()


def test_batch_larger_than_a_shard_partition_is_413(cp):
    from aiforearth_api_platform_amd.runtime.decode import PayloadError
    from aiforearth_api_platform_amd.runtime.model_endpoint import ModelEndpoint

    pool = ShardedWorkerPool(cp, EP, SPEC, ["cpu"] * 2, ring_slots=16)
    ep = ModelEndpoint(cp, "/v1/ai4e/tiny/classify", worker=pool)
    try:
        item = 4 * 4 * 3
        ep.begin_stream_batch(16 * item)  # fits one partition
        with pytest.raises(PayloadError) as e:
            ep.begin_stream_batch(17 * item)  # fits the whole ring (32), not one partition
        assert e.value.status == 413
    finally:
        pool.stop()
