"""Per-GPU worker pool: one process per MI355X behind the native NodeScheduler.

Replaces the reference's replica scaling (``APIs/Charts/templates/async-gpu/autoscaler.yaml`` HPA
1..10 replicas, ``routing.yml`` ROUND_ROBIN, ``deploy_aks.sh`` cluster autoscaler) with a fixed
node. The gateway process owns the task store, the endpoint's dispatch queue, the shared-memory
payload ring and the native scheduler; each GPU worker process (spawned here, or a ``torchrun``
rank that connects over TCP — :meth:`attach_remote`) maps the ring, registers it as pinned host
memory and executes batches the scheduler hands it. Placement is least-loaded by construction: a
worker's dispatcher thread pulls the next batch only when its GPU has a free pipeline slot. All
per-batch work (receive, running/completed transitions, result attachment, slot release) is C++.

Failure handling (survey §5.3): a worker that exits, or whose heartbeat stops for
``heartbeat_timeout_s``, has its in-flight batches requeued (redelivered to the surviving workers,
bounded by the queue's max delivery count -> task failed with a reason) and is restarted up to
``max_restarts`` times. ``resize(n)`` grows or shrinks the active GPU set without losing queued
tasks; :class:`runtime.autoscale.QueueDepthAutoscaler` drives it from queue depth (the HPA analogue).
In a :class:`ShardedWorkerPool` the shards' schedulers are competing consumers of each other's queues
(``NodeScheduler.set_peers``): a shard left without a live worker (restarts exhausted, or resized to zero) has its
queue drained by the others, and an idle shard helps a peer holding more than a full batch — any live GPU
finishes any queued task, as every replica of the reference consumes the one Service Bus queue
(``ProcessManager/BackendQueueProcessor/BackendQueueProcessor.cs:54-64``, ``host.json:3-11``).
Fault injection: ``AI4E_FAULT_INJECTION`` (see :mod:`runtime.gpu_worker`).
"""
from __future__ import annotations

import json
import multiprocessing as mp
import os
import threading
import time
from multiprocessing import shared_memory
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..store import native
from .gpu_worker import ModelSpec, follower_main, worker_main  # noqa: F401  (ModelSpec re-exported)
from .servable import format_result

__all__ = ["ModelSpec", "SharedPayloadRing", "WorkerPool"]


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _jpeg_slots_default(devices: Sequence[str], flag: Optional[bool]) -> bool:
    """Prepared JPEG slots are decoded on the GPU; a CPU worker would decode them with the slow numpy reference."""
    if flag is not None:
        return bool(flag)
    env = os.environ.get("AI4E_JPEG_SLOTS", "")
    if env:
        return env not in ("0", "false", "no")
    return any(str(d).startswith("cuda") for d in devices)


class SharedPayloadRing:
    """The node's payload ring in POSIX shared memory + the native slot allocator of this process's
    ingest partition ``[0, local_slots)``; slots beyond belong to remote ingest shards."""

    def __init__(self, nslots: int, item_shape: Sequence[int], local_slots: Optional[int] = None, durable=None,
                 jpeg_slots: bool = False):
        """``durable``: a :class:`runtime.durable_ring.DurableRing` (a task journal is configured): the ring is a
        crash-surviving segment with a per-slot task-id tag segment (``tags_name``) the schedulers write.
        ``jpeg_slots``: the ring's workers decode JPEG frames prepared into slots (runtime/jpeg_gpu.py): the segment's
        tail holds the key front-ends mark such slots with (``jpeg_key``; 0 when off)."""
        from .jpeg_gpu import RING_TAIL_BYTES, init_ring_tail

        self.nslots = int(nslots)
        self.item_shape = tuple(int(x) for x in item_shape)
        nbytes = self.nslots * int(np.prod(self.item_shape))
        self.durable = durable
        self.tags_name = ""
        if durable is not None:
            self.shm, self.tags_name = durable.create(self.nslots, self.item_shape)
        else:
            self.shm = shared_memory.SharedMemory(create=True, size=nbytes + RING_TAIL_BYTES)
        image = len(self.item_shape) == 3 and self.item_shape[2] == 3
        self.jpeg_key = init_ring_tail(self.shm.buf, nbytes, bool(jpeg_slots) and image)
        self.buf = torch.frombuffer(self.shm.buf, dtype=torch.uint8, count=nbytes).view(self.nslots, *self.item_shape)
        self.np_buf = self.buf.numpy()
        self.slots = native.SlotRing(int(local_slots or self.nslots), 0)

    @property
    def name(self) -> str:
        return self.shm.name

    @property
    def max_alloc(self) -> int:
        """The largest batch one allocation can hold (this process's ingest partition)."""
        return int(self.slots.capacity)

    def alloc(self, n: int, timeout: Optional[float] = None) -> List[int]:
        s = self.slots.alloc(int(n), -1.0 if timeout is None else float(timeout))
        if not s:
            raise TimeoutError("payload ring full")
        return s

    def free(self, slots: Sequence[int]) -> None:
        self.slots.free(list(slots))

    def write(self, slots: Sequence[int], images_u8: np.ndarray) -> None:
        """Copy decoded payloads into their slots (one copy per contiguous run of slots). A numpy copy: it runs on the
        calling thread with the GIL released (a torch copy of a large CPU tensor fans out over the intra-op pool, and
        with 16 request threads doing so at once the serving process oversubscribed its cores: 248 vs 3.9k requests/s
        of 640^2 images through the detector API, bench/jpeg_detect_bench.py raw mode)."""
        src = np.asarray(images_u8, dtype=np.uint8)
        dst = self.np_buf
        i, n = 0, len(slots)
        while i < n:
            j = i + 1
            while j < n and slots[j] == slots[j - 1] + 1:
                j += 1
            np.copyto(dst[slots[i]:slots[i] + (j - i)], src[i:j].reshape(j - i, *self.item_shape))
            i = j

    def close(self) -> None:
        self.slots.close()
        del self.buf, self.np_buf
        self.shm.close()
        if self.durable is not None:  # (its segments are unknown to the resource tracker)
            self.durable.close()
            return
        try:
            self.shm.unlink()
        except FileNotFoundError:
            pass


class RingPartition:
    """One control-plane shard's view of a node ring shared by several shards: the same shared memory
    (``name`` / ``nslots`` / ``buf``: workers address every slot by its global index) with its own native slot
    allocator over ``[base, base + length)``."""

    def __init__(self, ring: SharedPayloadRing, base: int, length: int):
        self.parent = ring
        self.nslots = ring.nslots
        self.item_shape = ring.item_shape
        self.buf = ring.buf
        self.np_buf = ring.np_buf
        self.base, self.length = int(base), int(length)
        self.slots = native.SlotRing(self.length, self.base)
        self.jpeg_key = ring.jpeg_key

    @property
    def name(self) -> str:
        return self.parent.name

    alloc = SharedPayloadRing.alloc
    free = SharedPayloadRing.free
    max_alloc = SharedPayloadRing.max_alloc
    write = SharedPayloadRing.write

    def close(self) -> None:  # (the owner of the shared memory closes it)
        self.slots.close()


class _WorkerHandle:
    def __init__(self, rank: int, device: str):
        self.rank = rank
        self.device = device
        self.proc: Optional[mp.Process] = None
        self.followers: List[mp.Process] = []  # the rest of a worker group
        self.group_devices: List[str] = [device]
        self.co: List["_WorkerHandle"] = []     # stage graph: the group's other leaders (spawned by this handle)
        self.owner: Optional["_WorkerHandle"] = None  # stage graph: the handle that spawns this leader's group
        self.restarts = 0
        self.stop = threading.Event()
        self.remote = False
        self.stats: dict = {}

    @property
    def ready(self) -> bool:
        return bool(self.stats.get("ready")) and bool(self.stats.get("alive"))

    @property
    def batches(self) -> int:
        return int(self.stats.get("batches", 0))

    @property
    def images(self) -> int:
        return int(self.stats.get("images", 0))


FRONTEND_RANK0 = 1 << 20  # scheduler connection ids of ingest front-ends (GPU worker ranks stay below)


def _sweep_stale_stats() -> None:
    """Unlink shard-counter segments (``ai4e_stat_<pid>_*``) left behind by serving processes that were killed."""
    try:
        names = os.listdir("/dev/shm")
    except OSError:
        return
    for n in names:
        if not n.startswith("ai4e_stat_"):
            continue
        try:
            pid = int(n.split("_")[2])
            os.kill(pid, 0)
        except ProcessLookupError:
            try:
                os.unlink(os.path.join("/dev/shm", n))
            except OSError:
                pass
        except (ValueError, IndexError, PermissionError):
            pass


class WorkerPool:
    def __init__(self, control_plane, endpoint: str, spec: ModelSpec, devices: Sequence[str], ring_slots: int = 0,
                 max_delay_s: float = 0.0005, heartbeat_interval_s: float = 0.5, heartbeat_timeout_s: float = 10.0,
                 max_restarts: int = 2, pipeline_depth: int = 3, retry_delay_s: float = 1.0,
                 remote_partitions: Sequence[Tuple[int, int, int]] = (), completion_feed: bool = False,
                 poll_s: float = 0.02, frontends: int = 0, frontend_slots: int = 0,
                 shard: Optional["ShardLayout"] = None, durable=None, busy_delay_s: float = 0.002,
                 jpeg_slots: Optional[bool] = None):
        """``max_delay_s``: how long a batch waits to fill when the worker is idle; ``busy_delay_s``: when it already
        has a batch in flight (its GPU is busy: a fuller batch costs no throughput, and arrivals of single images
        otherwise leave as many small batches, each in a padded graph bucket). ``shard``: this pool is one
        control-plane shard of a :class:`ShardedWorkerPool` (its own dispatch queue and scheduler, a partition of the
        shared ring, ids minted in its own task-store lock domains). ``jpeg_slots``: front-ends may prepare JPEG
        bodies into slots for the workers to decode on the GPU (runtime/jpeg_gpu.py; default: when the devices are
        GPUs, or AI4E_JPEG_SLOTS=1)."""
        if native is None:
            raise RuntimeError("the worker pool needs the native core (_ai4e_core)")
        self.cp = control_plane
        self.endpoint = endpoint
        self.shard = shard
        self.queue = control_plane.queue_for(endpoint, shard=None if shard is None else shard.index)
        self.store = control_plane.store
        if not isinstance(self.store, native.TaskStore) or not isinstance(self.queue, native.DispatchQueue):
            raise RuntimeError("the worker pool needs the native store/queue backend (AI4E_STORE_BACKEND=native)")
        # dead workers are found by heartbeat and their batches requeued by the scheduler; a peek-lock expiry
        # redelivery would give a batch's ring slots to a second worker while the first still holds them
        self.queue.set_lock_duration(0.0)
        self.spec = spec
        self.devices = list(devices)
        # 3 batches in flight per worker: two overlap on the GPU's two compute streams while the third is
        # already copied in, so a finishing batch never leaves the GPU waiting for the next H2D
        # (ResNet-50 @250: 67.4-69.5k -> 75.7-77.7k images/s, p50 10.6 -> 9.1-9.4 ms; profiles/r2_pool/)
        self.remote_partitions = [tuple(int(v) for v in p) for p in remote_partitions]  # (base, len, rank)
        if shard is not None:
            self.frontend_partitions = list(shard.frontend_parts)
            self.remote_partitions += list(shard.remote_parts) + self.frontend_partitions
            self.ring = RingPartition(shard.ring, shard.local[0], shard.local[1])
            total = shard.ring.nslots
        else:
            local = ring_slots or spec.max_batch * (pipeline_depth + 2) * max(1, len(self.devices))
            # ingest front-end processes (runtime/frontend.py): one ring partition each, after everything else
            end = max([local] + [b + n for b, n, _ in self.remote_partitions])
            fs = frontend_slots or spec.max_batch * 4
            self.frontend_partitions = [(end + i * fs, fs, FRONTEND_RANK0 + i) for i in range(int(frontends))]
            self.remote_partitions += self.frontend_partitions
            total = max([local] + [b + n for b, n, _ in self.remote_partitions])
            self.ring = SharedPayloadRing(total, spec.item_shape, local_slots=local, durable=durable,
                                          jpeg_slots=_jpeg_slots_default(devices, jpeg_slots))
        self.hb_interval = heartbeat_interval_s
        self.max_restarts = max_restarts
        self.sched = native.NodeScheduler(self.store, self.queue, endpoint, total, max_batch=spec.max_batch,
                                          linger_s=max_delay_s, depth=pipeline_depth, retry_delay_s=retry_delay_s,
                                          hb_timeout_s=heartbeat_timeout_s, poll_s=poll_s,
                                          busy_linger_s=busy_delay_s)
        self.sched.add_local_ring(self.ring.slots)
        tags = getattr(getattr(self.ring, "parent", self.ring), "tags_name", "")
        if tags and not self.sched.set_slot_tags(tags):
            raise RuntimeError(f"cannot map the payload ring's tag segment {tags}")
        # shard load (tasks queued / finished) in shm for the native front-ends' admission (unlinked with the scheduler)
        self.stat_name = ""
        if int(frontends) > 0 and hasattr(self.sched, "open_stat"):
            _sweep_stale_stats()
            name = f"ai4e_stat_{os.getpid()}_{id(self):x}"
            self.stat_name = name if self.sched.open_stat(name) else ""
        if shard is not None:
            self.sched.set_store_shards(list(shard.store_shards))
        if spec.stage_endpoints:
            self.sched.set_stage_endpoints(list(spec.stage_endpoints),
                                           ["running - stage %d" % (i + 2) for i in range(len(spec.stage_endpoints))])
        for base, n, rank in self.remote_partitions:
            self.sched.add_remote_partition(base, n, rank)
        self.workers: List[_WorkerHandle] = []
        self.events: List[Tuple[float, str, int]] = []  # (time, event, rank) for tests/ops
        self._ctx = mp.get_context("spawn")
        self._mu = threading.Lock()
        self._stop = threading.Event()
        self._monitor: Optional[threading.Thread] = None
        self._feed: Optional[threading.Thread] = None
        self._waiters: Dict[str, Callable[[str], None]] = {}
        self._wmu = threading.Lock()
        self.describe: dict = {}
        if completion_feed:
            self.enable_completion_feed()

    # ------------------------------------------------------------ lifecycle
    def start(self, wait_ready_s: float = 600.0) -> "WorkerPool":
        if self._monitor is not None:  # already started
            return self
        k = max(1, self.spec.group_size)
        nl = max(1, self.spec.group_leaders)
        if len(self.devices) % k:
            raise ValueError(f"{len(self.devices)} devices cannot form worker groups of {k}")
        if nl > 1 and nl >= k:
            raise ValueError(f"a stage graph of {k} GPUs needs fewer than {k} leaders, got {nl}")
        for i in range(len(self.devices) // k):
            devs = self.devices[i * k:(i + 1) * k]
            w = _WorkerHandle(i * nl, devs[0])
            w.group_devices = devs
            for j in range(1, nl if k > 1 else 1):  # the group's other leaders: own scheduler connections
                c = _WorkerHandle(i * nl + j, devs[j])
                c.owner = w
                w.co.append(c)
            self._spawn(w)
        self._monitor = threading.Thread(target=self._monitor_loop, daemon=True, name="ai4e-pool-monitor")
        self._monitor.start()
        self.wait_ready(wait_ready_s)
        return self

    def wait_ready(self, timeout_s: float = 600.0, n: Optional[int] = None) -> bool:
        deadline = time.time() + timeout_s
        while time.time() < deadline:
            self.refresh()
            active = [w for w in self.workers if not w.stop.is_set()]
            want = len(active) if n is None else n
            if sum(w.ready for w in active) >= want:
                return True
            if all(w.proc is not None and not w.proc.is_alive() for w in active if not w.remote) and active and \
                    not any(w.remote for w in active):
                return False
            time.sleep(0.02)
        return False

    def _spawn(self, w: _WorkerHandle) -> None:
        """Start a worker (or a whole worker group: its leaders, each with a scheduler connection, and its
        followers, all joined in one process group)."""
        port = _free_port() if self.spec.group_size > 1 else 0
        self._kill_followers(w)
        leaders = [w] + w.co
        conns = []
        for gr, h in enumerate(leaders):
            parent, child = self._ctx.Pipe(duplex=True)
            h.proc = self._ctx.Process(target=worker_main, args=(child, h.rank, h.device, self.spec, self.ring.name,
                                                                 self.ring.nslots, self.hb_interval),
                                       kwargs={"group_port": port, "group_rank": gr}, daemon=True,
                                       name=f"ai4e-gpu-worker-{h.rank}")
            h.proc.start()
            child.close()
            conns.append(parent)
        for g, dev in enumerate(w.group_devices[len(leaders):], start=len(leaders)):
            f = self._ctx.Process(target=follower_main, args=(dev, self.spec, g, self.spec.group_size, port),
                                  daemon=True, name=f"ai4e-gpu-worker-{w.rank}.{g}")
            f.start()
            w.followers.append(f)
        for h, parent in zip(leaders, conns):
            fd = os.dup(parent.fileno())
            parent.close()
            h.stop.clear()
            h.stats = {}
            h.spawned_at = time.time()
            with self._mu:
                if h not in self.workers:
                    self.workers.append(h)
            self.sched.attach(h.rank, fd, True)
            self.events.append((time.time(), "spawn", h.rank))

    @staticmethod
    def _kill_followers(w: _WorkerHandle, grace_s: float = 0.0) -> None:
        for f in w.followers:
            f.join(grace_s)
            if f.is_alive():
                f.kill()
                f.join(10)
        w.followers = []

    def attach_remote(self, rank: int, conn, device: str = "remote") -> None:
        """A worker process started elsewhere (a torchrun rank) that connected to this node scheduler."""
        w = _WorkerHandle(rank, device)
        w.remote = True
        fd = os.dup(conn.fileno())
        conn.close()
        with self._mu:
            self.workers.append(w)
        self.sched.attach(rank, fd, True)
        self.events.append((time.time(), "attach", rank))

    def attach_ingest(self, rank: int, conn) -> None:
        """An ingest front-end process (its ring partition declared via ``frontends``): SUBMIT_IDS in,
        SUBMITTED / FREE out; never given batches."""
        fd = os.dup(conn.fileno())
        conn.close()
        self.sched.attach(rank, fd, False)
        self.events.append((time.time(), "attach-ingest", rank))

    def _monitor_loop(self) -> None:
        suppress: Dict[int, float] = {}  # leaders killed by a group restart: their connection loss is expected
        while not self._stop.is_set():
            failed = self.sched.wait_failed(0.2)
            self.refresh()
            now = time.time()
            # a dead follower (no scheduler connection of its own) takes its group down too
            for w in list(self.workers):
                if w.owner is None and not w.stop.is_set() and any(f.exitcode is not None for f in w.followers):
                    failed.append(w.rank)
            for rank in failed:
                if suppress.get(rank, 0.0) > now:
                    suppress.pop(rank, None)
                    continue
                w = next((x for x in self.workers if x.rank == rank), None)
                if w is not None and w.owner is not None:
                    w = w.owner  # a stage-graph group restarts as a whole
                if w is None or w.stop.is_set():
                    continue
                self.events.append((time.time(), "worker_failed", rank))
                for h in [w] + w.co:
                    if h.proc is not None and h.proc.is_alive():
                        h.proc.kill()
                        h.proc.join(10)
                    if h.rank != rank:
                        suppress[h.rank] = now + 10.0
                self._kill_followers(w)
                if not w.remote and w.restarts < self.max_restarts and not self._stop.is_set():
                    w.restarts += 1
                    self.events.append((time.time(), "restart", rank))
                    self._spawn(w)
                else:
                    for h in [w] + w.co:
                        h.stop.set()
                    self.events.append((time.time(), "removed", rank))

    def resize(self, n: int, devices: Optional[Sequence[str]] = None) -> None:
        """Elastic: grow to / shrink to n active workers (queued tasks are never lost)."""
        if self.spec.group_leaders > 1:
            raise NotImplementedError("resize a stage-graph pool by whole groups (restart it with other devices)")
        active = [w for w in self.workers if not w.stop.is_set()]
        if n > len(active):
            devs = list(devices or self.devices)
            k = max(1, self.spec.group_size)
            for i in range(len(active), n):
                w = _WorkerHandle(max((w.rank for w in self.workers), default=-1) + 1, devs[(i * k) % len(devs)])
                w.group_devices = [devs[(i * k + j) % len(devs)] for j in range(k)]
                self._spawn(w)
        else:
            for w in active[n:]:
                self._retire(w)

    def active(self) -> int:
        return sum(1 for w in self.workers if not w.stop.is_set())

    def _retire(self, w: _WorkerHandle) -> None:
        for h in [w] + w.co:  # (a stage-graph group retires as a whole)
            h.stop.set()
            self.sched.detach(h.rank, 30.0)
        for h in [w] + w.co:
            if h.proc is not None:
                h.proc.join(30)
                if h.proc.is_alive():
                    h.proc.kill()
        self._kill_followers(w, 30.0)
        self.events.append((time.time(), "retire", w.rank))

    def stop(self) -> None:
        self._stop.set()
        for w in self.workers:
            if not w.stop.is_set():
                w.stop.set()
        self.sched.stop()
        if self.stat_name:
            self.sched.unlink_stat()
        for w in self.workers:
            if w.proc is not None:
                w.proc.join(30)
                if w.proc.is_alive():
                    w.proc.kill()
            self._kill_followers(w, 30.0)
        if self._monitor is not None:
            self._monitor.join(5)
        if self._feed is not None:
            self._feed.join(5)
        self.ring.close()

    # ------------------------------------------------------------ ingest (ModelEndpoint backend)
    def submit_slots(self, slots: Sequence[int], trace: str = "") -> List[str]:
        return self.sched.submit(list(slots), trace)

    def send_existing(self, task_id: str, slot: int) -> bool:
        """Queue a task whose record already exists (explicit TaskId, journal replay) for the payload in ``slot``."""
        return self.sched.send_existing([task_id], [int(slot)]) == 1

    @property
    def control_shards(self) -> List["WorkerPool"]:
        """The scheduler shards behind this endpoint (ingest front-ends attach to each): just this pool."""
        return [self]

    @property
    def durable(self):
        """The crash-surviving ring (:class:`runtime.durable_ring.DurableRing`) when a journal is configured."""
        return getattr(getattr(self.ring, "parent", self.ring), "durable", None)

    def queue_for_slot(self, slot: int):
        return self.queue

    def mint_digits(self) -> str:
        """Last hex digits the ids of this shard's tasks may end in: its task-store lock domains."""
        if self.shard is None:
            return "".join("%x" % d for d in range(min(16, max(1, self.store.nshards))))
        n = self.store.nshards
        return "".join("%x" % d for d in range(16) if d % n in set(self.shard.store_shards))

    def submit_many(self, images_u8: np.ndarray) -> List[str]:
        slots = self.ring.alloc(images_u8.shape[0], timeout=60)
        self.ring.write(slots, images_u8)
        return self.submit_slots(slots)

    # ------------------------------------------------------------ completion feed (sync routes)
    def enable_completion_feed(self) -> None:
        if self._feed is None:
            self.sched.enable_completion_feed(True)
            self._feed = threading.Thread(target=self._feed_loop, daemon=True, name="ai4e-pool-feed")
            self._feed.start()

    def add_waiter(self, task_id: str, cb: Callable[[str], None]) -> None:
        with self._wmu:
            self._waiters[task_id] = cb

    def pop_waiter(self, task_id: str) -> Optional[Callable[[str], None]]:
        with self._wmu:
            return self._waiters.pop(task_id, None)

    def _feed_loop(self) -> None:
        while not self._stop.is_set():
            ids = self.sched.wait_completed(0.2)
            if not ids or not self._waiters:
                continue
            with self._wmu:
                cbs = [(t, self._waiters.pop(t)) for t in ids if t in self._waiters]
            for t, cb in cbs:
                try:
                    cb(t)
                except Exception:
                    pass

    # ------------------------------------------------------------ results / stats
    def refresh(self) -> None:
        stats = {s["rank"]: s for s in self.sched.worker_stats()}
        for w in self.workers:
            s = stats.get(w.rank)
            if s is not None:
                w.stats = s
                if not self.describe and s.get("info"):
                    try:
                        self.describe = json.loads(s["info"])
                    except ValueError:
                        pass

    def result(self, task_id: str) -> Optional[dict]:
        if not self.describe:
            self.refresh()
        row = self.store.result(task_id)
        if row is None or not self.describe:
            return None
        return format_result(self.describe.get("kind", "raw"), self.describe.get("outputs", []), row)

    @property
    def images(self) -> int:
        return int(self.sched.images_done())

    def stats(self) -> dict:
        self.refresh()
        return {"workers": [dict(w.stats, device=w.device, restarts=w.restarts) for w in self.workers],
                "batch_histogram": self.sched.batch_histogram(), "images": self.images,
                "ring": {"slots": self.ring.nslots, "local_used": self.ring.slots.used()}}


# ---------------------------------------------------------------------------------------------------------------
# Control plane sharded by GPU
class ShardLayout:
    """Where one control-plane shard lives: shard ``index``, its partition ``local`` = (base, length) of the node ring
    ``ring`` (ingest from this process), the ring partitions of the ingest front-ends attached to it
    (base, length, scheduler rank) and the task-store lock domains it mints ids in."""

    def __init__(self, index: int, ring: SharedPayloadRing, local: Tuple[int, int],
                 frontend_parts: Sequence[Tuple[int, int, int]], store_shards: Sequence[int],
                 remote_parts: Sequence[Tuple[int, int, int]] = ()):
        self.index, self.ring, self.local = int(index), ring, (int(local[0]), int(local[1]))
        self.frontend_parts = [tuple(int(v) for v in p) for p in frontend_parts]
        self.store_shards = [int(v) for v in store_shards]
        # ingest partitions of remote worker processes (a torchrun rank that serves this shard and submits its own
        # clients' payloads over its scheduler connection): (base, length, rank)
        self.remote_parts = [tuple(int(v) for v in p) for p in remote_parts]


class _ShardedRing:
    """The endpoint's view of the node ring across shards (what :class:`ModelEndpoint` and the decode pool use):
    ``alloc`` picks the least-loaded shard with a live worker and returns global slot indices; ``free`` / ``write``
    route by slot range; ``name`` / ``nslots`` / ``buf`` are the one shared memory segment."""

    def __init__(self, ring: SharedPayloadRing, pools: Sequence["WorkerPool"]):
        self.parent, self.pools = ring, list(pools)
        self.nslots, self.item_shape, self.buf = ring.nslots, ring.item_shape, ring.buf
        self._rr = 0
        self._mu = threading.Lock()

    @property
    def name(self) -> str:
        return self.parent.name

    def pick(self) -> "WorkerPool":
        with self._mu:
            self._rr += 1
            start = self._rr
        k = len(self.pools)
        order = [self.pools[(start + i) % k] for i in range(k)]
        live = [p for p in order if p.active()] or order
        return min(live, key=lambda p: p.ring.slots.used() / max(1, p.ring.length))

    @property
    def max_alloc(self) -> int:
        return max(p.ring.length for p in self.pools)

    def owner(self, slot: int) -> "WorkerPool":
        for p in self.pools:
            if p.ring.base <= slot < p.ring.base + p.ring.length:
                return p
        raise ValueError(f"slot {slot} is not in any control-plane shard's local partition")

    def alloc(self, n: int, timeout: Optional[float] = None) -> List[int]:
        return self.pick().ring.alloc(n, timeout)

    def free(self, slots: Sequence[int]) -> None:
        for p, part in self._by_owner(slots):
            p.ring.free(part)

    def write(self, slots: Sequence[int], images_u8: np.ndarray) -> None:
        self.parent.write(slots, images_u8)

    def _by_owner(self, slots: Sequence[int]):
        groups: Dict[int, Tuple["WorkerPool", List[int]]] = {}
        for s in slots:
            p = self.owner(int(s))
            groups.setdefault(id(p), (p, []))[1].append(int(s))
        return list(groups.values())


class _QueueStats:
    """Aggregated dispatch-queue statistics of the shards (the autoscaler's queue-depth input)."""

    def __init__(self, pools: Sequence["WorkerPool"]):
        self.pools = list(pools)

    def stats(self) -> dict:
        out: Dict[str, float] = {}
        for p in self.pools:
            for k, v in p.queue.stats().items():
                if isinstance(v, (int, float)) and not isinstance(v, bool):
                    out[k] = out.get(k, 0) + v
        return out

    def depth(self) -> int:
        return sum(p.queue.depth() for p in self.pools)


class ShardedWorkerPool:
    """A pool-backed endpoint whose control plane scales with its GPUs: one scheduler shard per GPU (or worker
    group), each with its own dispatch queue, node scheduler threads, partition of the node's payload ring and
    task-store lock domains, behind the one gateway and the native front-ends.

    The reference scales an API as HPA replicas (``APIs/Charts/templates/async-gpu/autoscaler.yaml:11-21``) behind
    Istio's ROUND_ROBIN (``APIs/Charts/templates/routing.yml:26-28``); its single serial dispatch point
    (``ProcessManager/BackendQueueProcessor/host.json:3-11``) is what this layout avoids: every task of an N-GPU
    endpoint passes through the scheduler of ONE shard, and shards share nothing on the per-task path.

    * ingest picks a shard per request: least-loaded by the shard's ring partition (the native front-ends
      the same per front-end partition, ``csrc/ingest/ingestd.cpp`` ``pick_shard``);
    * a task id's last hex digit names its task-store lock domain and so its shard, so status / result / trace
      lookups go straight to one domain (no broadcast);
    * queue-length and ``CURRENT_REQUESTS`` metrics aggregate over shards (the store's merged indexes,
      :class:`_QueueStats`).
    """

    def __init__(self, control_plane, endpoint: str, spec: ModelSpec, devices: Sequence[str], shards: int = 0,
                 ring_slots: int = 0, frontends: int = 0, frontend_slots: int = 0, pipeline_depth: int = 3,
                 remote: Sequence[int] = (), remote_slots: int = 0, durable=None, jpeg_slots: Optional[bool] = None,
                 **kw):
        """``remote``: shards whose worker is a process started elsewhere (a torchrun rank of the multi-GPU bench) that
        attaches with ``control_shards[i].attach_remote(i, conn)`` and ingests into its own ``remote_slots`` partition
        (``remote_partition(i)``); nothing is spawned for those shards."""
        self.cp, self.endpoint, self.spec = control_plane, endpoint, spec
        self.devices = list(devices)
        k = max(1, spec.group_size)
        if len(self.devices) % k:
            raise ValueError(f"{len(self.devices)} devices cannot form worker groups of {k}")
        groups = [self.devices[i * k:(i + 1) * k] for i in range(len(self.devices) // k)]
        K = max(1, min(int(shards or len(groups)), len(groups)))
        nstore = control_plane.store.nshards
        if K > 16:
            raise ValueError("at most 16 control-plane shards (a task id's last hex digit names its shard)")
        if K > nstore:
            raise ValueError(f"{K} control-plane shards need a task store of >= {K} lock domains (has {nstore})")
        shard_devs = [[d for g in groups[i::K] for d in g] for i in range(K)]
        self.remote = sorted(set(int(i) for i in remote))
        if any(not 0 <= i < K for i in self.remote):
            raise ValueError(f"remote shards {self.remote} outside 0..{K - 1}")
        for i in self.remote:
            shard_devs[i] = []  # (its worker attaches from elsewhere)
        fs = frontend_slots or spec.max_batch * 4
        layout, base = [], 0
        for i in range(K):
            n_local = ring_slots or spec.max_batch * (pipeline_depth + 2) * max(1, len(shard_devs[i]))
            layout.append([(base, n_local)])
            base += n_local
        self._remote_parts: Dict[int, Tuple[int, int, int]] = {}
        for i in self.remote:
            self._remote_parts[i] = (base, int(remote_slots or spec.max_batch * 4), i)
            base += self._remote_parts[i][1]
        for i in range(K):
            parts = []
            for f in range(int(frontends)):
                parts.append((base, fs, FRONTEND_RANK0 + f))
                base += fs
            layout[i].append(parts)
        self._ring = SharedPayloadRing(base, spec.item_shape, local_slots=1, durable=durable,
                                       jpeg_slots=_jpeg_slots_default(self.devices, jpeg_slots))
        self.pools: List[WorkerPool] = []
        for i in range(K):
            lay = ShardLayout(i, self._ring, layout[i][0], layout[i][1], [s for s in range(nstore) if s % K == i],
                              [self._remote_parts[i]] if i in self._remote_parts else [])
            self.pools.append(WorkerPool(control_plane, endpoint, spec, shard_devs[i], pipeline_depth=pipeline_depth,
                                         frontends=frontends, frontend_slots=fs, shard=lay, **kw))
        self.ring = _ShardedRing(self._ring, self.pools)
        self.queue = _QueueStats(self.pools)
        # one waiter table for every shard: a task's completion may come from any shard's scheduler (a stolen batch,
        # or a task created outside its shard's lock domains), and each shard's feed loop drains into the same table
        self._waiters: Dict[str, Callable[[str], None]] = {}
        self._wmu = threading.Lock()
        for p in self.pools:
            p._waiters, p._wmu = self._waiters, self._wmu
        scheds = [p.sched for p in self.pools]
        for p in self.pools:
            p.sched.set_peers(scheds)

    # ------------------------------------------------------------ lifecycle
    def start(self, wait_ready_s: float = 600.0) -> "ShardedWorkerPool":
        for p in self.pools:  # spawn every shard's workers first, then wait for all of them together
            p.start(wait_ready_s=0.0)
        self.wait_ready(wait_ready_s)
        return self

    def wait_ready(self, timeout_s: float = 600.0, n: Optional[int] = None) -> bool:
        deadline = time.time() + timeout_s
        ok = True
        for p in self.pools:
            ok = p.wait_ready(max(0.0, deadline - time.time())) and ok
        return ok

    def stop(self) -> None:
        for p in self.pools:
            p.stop()
        self._ring.close()

    def active(self) -> int:
        return sum(p.active() for p in self.pools)

    def resize(self, n: int, devices: Optional[Sequence[str]] = None) -> None:
        """Elastic: n local workers spread over the shards that have local devices (a remote shard's worker is a
        torchrun rank, not ours to spawn or retire). A shard resized to zero keeps its queue and ring partition; the
        live shards drain it (competing consumers) and new ingest skips it."""
        local = [p for i, p in enumerate(self.pools) if i not in self.remote and p.devices]
        if not local:
            return
        n = max(0, int(n))
        k = len(local)
        for i, p in enumerate(local):
            p.resize(n // k + (1 if i < n % k else 0))

    @property
    def workers(self) -> list:
        return [w for p in self.pools for w in p.workers]

    @property
    def events(self) -> list:
        return sorted(e for p in self.pools for e in p.events)

    @property
    def control_shards(self) -> List[WorkerPool]:
        return list(self.pools)

    @property
    def durable(self):
        return self._ring.durable

    def remote_partition(self, shard: int) -> Tuple[int, int, int]:
        """(base, length, rank) of a remote shard's ingest partition of the shared ring."""
        return self._remote_parts[int(shard)]

    # ------------------------------------------------------------ ingest
    def submit_slots(self, slots: Sequence[int], trace: str = "") -> List[str]:
        ids: List[str] = []
        for p, part in self.ring._by_owner(slots):
            ids += p.submit_slots(part, trace)
        return ids

    def submit_many(self, images_u8: np.ndarray) -> List[str]:
        p = self.ring.pick()
        slots = p.ring.alloc(images_u8.shape[0], timeout=60)
        p.ring.write(slots, images_u8)
        return p.submit_slots(slots)

    def queue_for_slot(self, slot: int):
        return self.ring.owner(int(slot)).queue

    def attach_ingest(self, rank: int, conn) -> None:
        raise TypeError("attach ingest front-ends per control-plane shard (ShardedWorkerPool.control_shards)")

    # ------------------------------------------------------------ completion feed / results / stats
    def enable_completion_feed(self) -> None:
        for p in self.pools:
            p.enable_completion_feed()

    def _owner_of(self, task_id: str) -> WorkerPool:
        return self.pools[self.cp.store.shard_index(task_id) % len(self.pools)]

    def add_waiter(self, task_id: str, cb: Callable[[str], None]) -> None:
        with self._wmu:
            self._waiters[task_id] = cb

    def pop_waiter(self, task_id: str) -> Optional[Callable[[str], None]]:
        with self._wmu:
            return self._waiters.pop(task_id, None)

    def send_existing(self, task_id: str, slot: int) -> bool:
        return self.ring.owner(int(slot)).send_existing(task_id, slot)

    def refresh(self) -> None:
        for p in self.pools:
            p.refresh()

    @property
    def describe(self) -> dict:
        for p in self.pools:
            if not p.describe:
                p.refresh()
            if p.describe:
                return p.describe
        return {}

    def result(self, task_id: str) -> Optional[dict]:
        return self._owner_of(task_id).result(task_id) if self.describe else None

    @property
    def images(self) -> int:
        return sum(p.images for p in self.pools)

    def stats(self) -> dict:
        per = [p.stats() for p in self.pools]
        hists = [s.get("batch_histogram") or [] for s in per]
        return {"workers": [dict(w, shard=i) for i, s in enumerate(per) for w in s["workers"]],
                "batch_histogram": [sum(h[i] for h in hists if i < len(h)) for i in range(max(map(len, hists)))],
                "images": self.images, "control_plane_shards": len(self.pools),
                "live_workers_per_shard": [p.sched.live_workers() for p in self.pools],
                "stolen_items": sum(p.sched.stolen_items() for p in self.pools),
                "ring": {"slots": self._ring.nslots, "local_used": sum(s["ring"]["local_used"] for s in per)}}

