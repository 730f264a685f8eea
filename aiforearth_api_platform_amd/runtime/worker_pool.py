"""Per-GPU worker pool: one process per MI355X, heartbeats, fail-over requeue, elastic resize.

Replaces the reference's replica scaling (``APIs/Charts/templates/async-gpu/autoscaler.yaml`` HPA
1..10 replicas, ``routing.yml`` ROUND_ROBIN, ``deploy_aks.sh`` cluster autoscaler) with a fixed
node: the gateway process owns the task store, the dispatch queue and a shared-memory payload ring;
each GPU worker process (``HIP_VISIBLE_DEVICES``-style pinning via ``cuda:<i>``) maps the ring,
registers it as pinned host memory, and runs batches handed to it over a pipe. Placement is
least-loaded by construction: each worker's dispatcher thread pulls the next batch from the shared
endpoint queue only when its GPU has a free pipeline slot.

Failure handling (survey §5.3): a worker that exits, or whose heartbeat stops for
``heartbeat_timeout_s``, has its in-flight batches abandoned back to the queue (redelivered to the
surviving workers, bounded by the queue's max delivery count -> task failed with a reason), and is
restarted up to ``max_restarts`` times; ``resize(n)`` grows or shrinks the active GPU set without
losing queued tasks. ``AI4E_FAULT_INJECTION`` drives the failure tests:
``exit_after=<batches>[@<rank>]``, ``hang_after=<batches>[@<rank>]``, ``delay_ms=<ms>``.
"""
from __future__ import annotations

import importlib
import multiprocessing as mp
import os
import threading
import time
from dataclasses import dataclass, field
from multiprocessing import shared_memory
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..store import STATE_COMPLETED, STATE_FAILED, STATE_RUNNING
from .engine import PayloadRing
from .serving import ResultStore


@dataclass
class ModelSpec:
    factory: str                      # "package.module:function" -> callable(u8 [b,H,W,C]) -> logits
    item_shape: Tuple[int, int, int]
    max_batch: int = 250  # whole waves of workgroups on 256 CUs for ResNet-50 (bench.py)
    topk: int = 5
    kwargs: Dict[str, Any] = field(default_factory=dict)
    use_graphs: bool = True
    buckets: Tuple[int, ...] = ()      # captured batch sizes (config.bucket_list); () = max_batch only


class SharedPayloadRing(PayloadRing):
    """PayloadRing whose buffer lives in POSIX shared memory (children map it read-only by name)."""

    def __init__(self, nslots: int, item_shape: Sequence[int]):
        self.nslots = int(nslots)
        self.item_shape = tuple(item_shape)
        nbytes = self.nslots * int(np.prod(self.item_shape))
        self.shm = shared_memory.SharedMemory(create=True, size=max(nbytes, 1))
        self.buf = torch.frombuffer(self.shm.buf, dtype=torch.uint8, count=nbytes).view(self.nslots, *self.item_shape)
        self._head = 0
        self._used = 0
        self._free = [False] * self.nslots
        self._mu = threading.Condition()

    @staticmethod
    def attach(name: str, nslots: int, item_shape: Sequence[int]):
        shm = shared_memory.SharedMemory(name=name)
        nbytes = nslots * int(np.prod(item_shape))
        buf = torch.frombuffer(shm.buf, dtype=torch.uint8, count=nbytes).view(nslots, *item_shape)
        return shm, buf

    def close(self) -> None:
        del self.buf
        try:
            self.shm.close()
            self.shm.unlink()
        except FileNotFoundError:
            pass


def _load_factory(path: str):
    mod, fn = path.split(":")
    return getattr(importlib.import_module(mod), fn)


def _parse_fault(rank: int) -> Dict[str, int]:
    out = {}
    spec = os.environ.get("AI4E_FAULT_INJECTION", "")
    for item in filter(None, spec.split(",")):
        k, v = item.split("=")
        tgt = None
        if "@" in v:
            v, tgt = v.split("@")
        if tgt is None or int(tgt) == rank:
            out[k.strip()] = int(v)
    return out


def _child_main(rank: int, device: str, spec: ModelSpec, shm_name: str, nslots: int, conn, hb_interval: float):
    """GPU worker process body."""
    from .engine import InferenceEngine

    dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    shm, buf = SharedPayloadRing.attach(shm_name, nslots, spec.item_shape)
    registered = False
    if dev.type == "cuda":
        try:  # pin the shared ring in place so H2D DMA reads it directly
            rc = torch.cuda.cudart().cudaHostRegister(buf.data_ptr(), buf.numel(), 0)
            registered = int(rc) == 0 if not isinstance(rc, tuple) else int(rc[0]) == 0
        except Exception:
            registered = False
    model = _load_factory(spec.factory)(device=device, **spec.kwargs)
    engine = InferenceEngine(model, spec.item_shape, spec.max_batch, device=dev, topk=spec.topk,
                             use_graphs=spec.use_graphs, head_fn=getattr(model, "topk_u8", None),
                             buckets=list(spec.buckets) or None)
    engine.warmup()
    fault = _parse_fault(rank)
    send_mu = threading.Lock()
    alive = threading.Event()
    alive.set()

    def send(msg):
        with send_mu:
            conn.send(msg)

    def heartbeat():
        while alive.is_set():
            try:
                send(("hb", rank, time.time()))
            except (BrokenPipeError, EOFError, OSError):
                return
            time.sleep(hb_interval)

    threading.Thread(target=heartbeat, daemon=True).start()
    send(("ready", rank, registered))
    pending: List[Tuple[int, Any]] = []
    nbatches = 0
    while True:
        # retire finished batches in order (the parent keeps at most `depth` outstanding)
        while pending and (pending[0][1].done.query() or len(pending) > 2):
            bid, res = pending.pop(0)
            res.done.synchronize()
            send(("done", bid, res.top_idx.numpy().copy(), res.top_prob.numpy().copy()))
        if not conn.poll(0.0005 if pending else 0.05):
            continue
        msg = conn.recv()
        if msg[0] == "stop":
            break
        if msg[0] == "batch":
            _, bid, slots = msg
            nbatches += 1
            if "exit_after" in fault and nbatches > fault["exit_after"]:
                os._exit(17)
            if "hang_after" in fault and nbatches > fault["hang_after"]:
                alive.clear()
                time.sleep(3600)
            if fault.get("delay_ms"):
                time.sleep(fault["delay_ms"] / 1e3)
            pending.append((bid, engine.submit(buf, slots)))
    alive.clear()
    for bid, res in pending:
        res.done.synchronize()
    del buf
    shm.close()


class _WorkerHandle:
    def __init__(self, rank: int, device: str):
        self.rank = rank
        self.device = device
        self.proc: Optional[mp.Process] = None
        self.conn = None
        self.last_hb = 0.0
        self.ready = False
        self.outstanding: Dict[int, Tuple[List[str], List[int], List[int]]] = {}
        self.restarts = 0
        self.thread: Optional[threading.Thread] = None
        self.stop = threading.Event()
        self.batches = 0
        self.images = 0


class WorkerPool:
    def __init__(self, control_plane, endpoint: str, spec: ModelSpec, devices: Sequence[str], ring_slots: int = 0,
                 max_delay_s: float = 0.0005, heartbeat_interval_s: float = 0.5, heartbeat_timeout_s: float = 10.0,
                 max_restarts: int = 2, pipeline_depth: int = 2, results: Optional[ResultStore] = None):
        self.cp = control_plane
        self.endpoint = endpoint
        self.queue = control_plane.queue_for(endpoint)
        self.store = control_plane.store
        self.spec = spec
        self.devices = list(devices)
        self.ring = SharedPayloadRing(ring_slots or spec.max_batch * (pipeline_depth + 2) * max(1, len(devices)),
                                      spec.item_shape)
        self.max_delay_s = max_delay_s
        self.hb_interval = heartbeat_interval_s
        self.hb_timeout = heartbeat_timeout_s
        self.max_restarts = max_restarts
        self.depth = pipeline_depth
        self.results = results or ResultStore()
        self.workers: List[_WorkerHandle] = []
        self.events: List[Tuple[float, str, int]] = []  # (time, event, rank) for tests/ops
        self._ctx = mp.get_context("spawn")
        self._bid = 0
        self._bmu = threading.Lock()
        self.on_batch_done = None

    # ------------------------------------------------------------ lifecycle
    def start(self, wait_ready_s: float = 300.0) -> "WorkerPool":
        for i, dev in enumerate(self.devices):
            self._spawn(_WorkerHandle(i, dev))
        deadline = time.time() + wait_ready_s
        while time.time() < deadline and not all(w.ready for w in self.workers):
            time.sleep(0.01)
        return self

    def _spawn(self, w: _WorkerHandle) -> None:
        parent, child = self._ctx.Pipe()
        w.conn = parent
        w.ready = False
        w.last_hb = time.time()
        w.proc = self._ctx.Process(target=_child_main, args=(w.rank, w.device, self.spec, self.ring.shm.name,
                                                             self.ring.nslots, child, self.hb_interval), daemon=True)
        w.proc.start()
        child.close()
        w.stop.clear()
        if w not in self.workers:
            self.workers.append(w)
        w.thread = threading.Thread(target=self._dispatch_loop, args=(w,), daemon=True,
                                    name=f"ai4e-pool-dispatch-{w.rank}")
        w.thread.start()
        self.events.append((time.time(), "spawn", w.rank))

    def resize(self, n: int, devices: Optional[Sequence[str]] = None) -> None:
        """Elastic: grow to / shrink to n active workers (queued tasks are never lost)."""
        active = [w for w in self.workers if not w.stop.is_set()]
        if n > len(active):
            devs = list(devices or self.devices)
            for i in range(len(active), n):
                self._spawn(_WorkerHandle(len(self.workers), devs[i % len(devs)]))
        else:
            for w in active[n:]:
                self._retire(w)

    def _retire(self, w: _WorkerHandle) -> None:
        w.stop.set()
        if w.thread is not None:
            w.thread.join(30)
        try:
            w.conn.send(("stop",))
        except (BrokenPipeError, OSError):
            pass
        if w.proc is not None:
            w.proc.join(30)
            if w.proc.is_alive():
                w.proc.kill()
        self.events.append((time.time(), "retire", w.rank))

    def stop(self) -> None:
        for w in self.workers:
            if not w.stop.is_set():
                self._retire(w)
        self.ring.close()

    # ------------------------------------------------------------ submission (ModelEndpoint-compatible)
    def submit_many(self, images_u8: np.ndarray) -> List[str]:
        n = images_u8.shape[0]
        slots = self.ring.alloc(n, timeout=60)
        for i, s in enumerate(slots):
            self.ring.buf[s].copy_(torch.from_numpy(np.require(images_u8[i], requirements=["C", "W"])))
        ids = self.store.create_many(self.endpoint, n)
        self.queue.send_many(ids, slots)
        return ids

    def result(self, task_id: str):
        return self.results.get(task_id)

    @property
    def images(self) -> int:
        return sum(w.images for w in self.workers)

    # ------------------------------------------------------------ per-worker dispatcher
    def _dispatch_loop(self, w: _WorkerHandle) -> None:
        while not w.stop.is_set():
            # drain worker messages
            try:
                while w.conn.poll(0):
                    self._on_msg(w, w.conn.recv())
            except (EOFError, OSError):
                pass
            if not w.proc.is_alive() or (w.ready and time.time() - w.last_hb > self.hb_timeout):
                self._fail_over(w)
                return
            if not w.ready or len(w.outstanding) >= self.depth:
                w.conn.poll(0.0005)
                continue
            msgs = self.queue.receive(self.spec.max_batch, 0.0005 if w.outstanding else 0.02, self.max_delay_s)
            if not msgs:
                continue
            ids = [m.task_id for m in msgs]
            seqs = [m.seq for m in msgs]
            slots = [m.ref for m in msgs]
            self.store.transition_many(ids, STATE_RUNNING, STATE_RUNNING)
            with self._bmu:
                bid = self._bid
                self._bid += 1
            w.outstanding[bid] = (ids, seqs, slots)
            try:
                w.conn.send(("batch", bid, slots))
            except (BrokenPipeError, OSError):
                self._fail_over(w)
                return

    def _on_msg(self, w: _WorkerHandle, msg) -> None:
        kind = msg[0]
        if kind == "hb":
            w.last_hb = time.time()
        elif kind == "ready":
            w.ready = True
            w.last_hb = time.time()
            self.events.append((time.time(), "ready", w.rank))
        elif kind == "done":
            _, bid, idx, prob = msg
            ids, seqs, slots = w.outstanding.pop(bid)
            self.ring.free(slots)
            self.results.put_batch(ids, idx, prob)
            self.store.transition_many(ids, STATE_COMPLETED, STATE_COMPLETED)
            self.queue.complete(seqs)
            w.batches += 1
            w.images += len(ids)
            if self.on_batch_done is not None:
                self.on_batch_done(ids)

    def _fail_over(self, w: _WorkerHandle) -> None:
        """Requeue the dead/hung worker's in-flight batches and restart it (bounded)."""
        self.events.append((time.time(), "worker_failed", w.rank))
        for bid, (ids, seqs, slots) in list(w.outstanding.items()):
            self.store.transition_many(ids, "created", "Awaiting service availability. Worker failed; requeued.")
            for s in seqs:
                self.queue.abandon(s, 0.0)
        w.outstanding.clear()
        dead = self.queue.take_deadletters()
        if dead:
            self.store.transition_many(dead, STATE_FAILED, "Task failed - maximum retries exceeded")
        if w.proc is not None and w.proc.is_alive():
            w.proc.kill()
            w.proc.join(10)
        if w.restarts < self.max_restarts and not w.stop.is_set():
            w.restarts += 1
            self.events.append((time.time(), "restart", w.rank))
            self._spawn(w)
        else:
            w.stop.set()
            self.events.append((time.time(), "removed", w.rank))
