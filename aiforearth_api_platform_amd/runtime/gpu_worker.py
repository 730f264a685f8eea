"""GPU worker process body: one process per MI355X, driven by the native NodeScheduler.

Replaces the reference's model container behind ``BackendQueueProcessor``
(``APIs/1.0/base-py/ai4e_service.py:180-213`` thread-per-request execution, fed by
``BackendQueueProcessor.cs:48-52`` HTTP POSTs): the worker maps the node's shared payload ring,
registers it as pinned host memory (``hipHostRegister``) so the H2D DMA reads request bytes where
the ingest wrote them, captures the model once per batch bucket in HIP graphs, and then only
executes BATCH frames (slot lists) and answers with DONE frames (item-major result rows).

Per-item isolation (survey §5.3, poison messages): slots outside the ring fail as invalid payloads
on their own; if a batch launch raises, the worker re-runs its items one by one, so only the items
that fail on their own are reported failed — the rest of the batch completes.

Fault injection (``AI4E_FAULT_INJECTION``, comma list, ``key=value[@rank]``):
``exit_after=<batches>``, ``hang_after=<batches>``, ``delay_ms=<ms>``, ``fail_batch=<batch index>``
(the launch of that batch raises; drives the isolation path), ``fail_item=<slot>`` (the isolated run
of that slot raises -> that item fails), ``fail_finalize=<n>`` (the n-th batch retirement raises -> its
items are returned for another delivery).
"""
from __future__ import annotations

import importlib
import os
import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import protocol as P
from .servable import as_servable, encode_rows, row_bytes


@dataclass
class ModelSpec:
    factory: str                      # "package.module:function" -> Servable or logits model
    item_shape: Tuple[int, ...]
    max_batch: int = 250  # whole waves of workgroups on 256 CUs for ResNet-50 (bench.py)
    topk: int = 5
    kwargs: Dict[str, Any] = field(default_factory=dict)
    use_graphs: bool = True
    buckets: Tuple[int, ...] = ()      # captured batch sizes (config.bucket_list); () = max_batch only
    # ensemble stages: endpoint of each later stage (the scheduler re-targets the batch's tasks there)
    stage_endpoints: Tuple[str, ...] = ()
    # worker group: each pool worker is `group_size` processes on consecutive devices joined in one
    # process group (RCCL on GPUs, gloo on CPU) — the leader talks to the scheduler, the followers serve
    # it (detector -> classifier pair over xGMI, spatial-parallel mosaic segmentation)
    group_size: int = 1
    # stage graph: the first `group_leaders` processes of a group each take batches from the scheduler (e.g. 7
    # detector GPUs), the rest serve them (e.g. 1 classifier GPU); 1 = one leader + followers
    group_leaders: int = 1


def load_factory(path: str):
    mod, fn = path.split(":")
    return getattr(importlib.import_module(mod), fn)


def parse_fault(rank: int) -> Dict[str, int]:
    out = {}
    for item in filter(None, os.environ.get("AI4E_FAULT_INJECTION", "").split(",")):
        k, v = item.split("=")
        tgt = None
        if "@" in v:
            v, tgt = v.split("@")
        if tgt is None or int(tgt) == rank:
            out[k.strip()] = int(v)
    return out


def attach_ring(shm_name: str, nslots: int, item_shape: Sequence[int], untrack: bool = False):
    """Map the node's payload ring. Processes with their own resource tracker (torchrun ranks) must
    ``untrack`` it, or their tracker unlinks the owner's segment when they exit; spawned children
    share the owner's tracker and must not."""
    from multiprocessing import resource_tracker, shared_memory

    if shm_name.startswith("ai4ej_"):  # a durable ring outlives a crash: never tracked (runtime/durable_ring.py)
        from .durable_ring import open_untracked

        shm = open_untracked(shm_name)
        untrack = False
    else:
        shm = shared_memory.SharedMemory(name=shm_name)
    if untrack:
        try:
            resource_tracker.unregister(shm._name, "shared_memory")  # type: ignore[attr-defined]
        except Exception:
            pass
    nbytes = int(nslots) * int(np.prod(item_shape))
    buf = torch.frombuffer(shm.buf, dtype=torch.uint8, count=nbytes).view(int(nslots), *item_shape)
    return shm, buf


def ring_jpeg_key(shm, nslots: int, item_shape: Sequence[int]) -> int:
    """The key marking slots that hold prepared JPEG frames (runtime/jpeg_gpu.py; 0: the ring has none)."""
    from .jpeg_gpu import ring_key

    return ring_key(shm.buf, int(nslots) * int(np.prod(item_shape)))


def pin_host(buf: torch.Tensor) -> bool:
    """Register the mapped ring as pinned host memory for direct DMA (hipHostRegister)."""
    try:
        rc = torch.cuda.cudart().cudaHostRegister(buf.data_ptr(), buf.numel(), 0)
        return (int(rc[0]) if isinstance(rc, tuple) else int(rc)) == 0
    except Exception:
        return False


class _Pending:
    __slots__ = ("bid", "n", "valid", "res", "t_recv", "status")

    def __init__(self, bid, n, valid, res, t_recv, status):
        self.bid, self.n, self.valid, self.res, self.t_recv, self.status = bid, n, valid, res, t_recv, status


class GpuWorker:
    """The loop of one worker process (also usable in a thread for tests)."""

    def __init__(self, conn: P.FrameConn, rank: int, device: str, spec: ModelSpec, ring_buf: torch.Tensor,
                 local_ring=None, hb_interval: float = 0.5, depth: int = 2, group_kwargs: Optional[dict] = None,
                 jpeg_key: int = 0):
        self.conn = conn
        self.rank = rank
        self.device = torch.device(device)
        self.spec = spec
        self.buf = ring_buf
        self.nslots = ring_buf.shape[0]
        self.jpeg_key = int(jpeg_key)  # slots holding prepared JPEG frames are decoded on the device (engine.py)
        self._ring_u8 = ring_buf.view(self.nslots, -1).numpy() if self.jpeg_key else None
        self.jpeg_frames = 0
        self.local_ring = local_ring  # native SlotRing of this process's ingest partition (FREE frames)
        self.hb_interval = hb_interval
        self.depth = depth
        self.fault = parse_fault(rank)
        self.servable = as_servable(load_factory(spec.factory)(device=device, **spec.kwargs, **(group_kwargs or {})),
                                    spec.topk)
        from .engine import InferenceEngine

        self.engine = InferenceEngine(None, spec.item_shape, spec.max_batch, device=self.device,
                                      use_graphs=spec.use_graphs, buckets=list(spec.buckets) or None,
                                      output_fn=self.servable, timing=self.device.type == "cuda")
        self.engine.warmup()
        self.row_bytes = row_bytes(self.servable.outputs)
        self.batches = 0
        self.isolated_batches = 0
        self.busy_ms = 0.0
        self._ready_sent = threading.Event()
        self.alive = threading.Event()
        self.alive.set()

    # ------------------------------------------------------------------ lifecycle
    def info(self) -> dict:
        d = self.servable.describe()
        d.update(device=str(self.device), max_batch=self.spec.max_batch, buckets=list(self.engine.buckets),
                 pid=os.getpid())
        if self.device.type == "cuda":
            d["gpu"] = torch.cuda.get_device_name(self.device)
        return d

    def _heartbeat(self) -> None:
        tel = None
        while self.alive.is_set():
            # GFX clock and power per heartbeat (fail-soft); amdsmi is initialised only once READY has gone out,
            # never concurrently with the main thread's HIP calls (an amdsmi_init racing them broke device lookup)
            if tel is None and self.device.type == "cuda" and self._ready_sent.is_set():
                from ..utils.gpu_telemetry import GpuTelemetry

                tel = GpuTelemetry(self.device.index or 0)
            used = total = 0
            if self.device.type == "cuda":
                try:
                    free, total = torch.cuda.mem_get_info(self.device)
                    used = total - free
                except Exception:
                    pass
            xg = getattr(self.servable, "xgmi_bytes", None)
            tx = rx = 0
            if callable(xg):
                b = xg()
                tx, rx = int(b.get("sent", 0)), int(b.get("received", 0))
            smp = tel.sample() if tel is not None else {}
            try:
                self.conn.heartbeat(time.monotonic(), used, total, self.busy_ms, self.batches, tx, rx,
                                    smp.get("gfx_mhz", 0.0), smp.get("power_w", 0.0))
            except (BrokenPipeError, EOFError, OSError):
                return
            time.sleep(self.hb_interval)

    def serve(self, pinned: bool = False) -> None:
        """Main thread: read frames and launch batches; a completion thread retires them in order
        (blocking event waits, no polling), so a DONE frame leaves as soon as its GPU work ends."""
        threading.Thread(target=self._heartbeat, daemon=True, name=f"ai4e-hb-{self.rank}").start()
        self._done_q: "queue.Queue[Optional[_Pending]]" = queue.Queue()
        self._idle = threading.Condition()
        self._inflight = 0
        fin = threading.Thread(target=self._completion_loop, daemon=True, name=f"ai4e-done-{self.rank}")
        fin.start()
        self.conn.ready(self.rank, pinned, self.info())
        self._ready_sent.set()
        try:
            while True:
                try:
                    buf = self.conn.recv()
                except (EOFError, OSError):
                    break
                t = P.frame_type(buf)
                if t == P.F_BATCH:
                    self._on_batch(buf)
                elif t == P.F_FREE:
                    if self.local_ring is not None:
                        self.local_ring.free(P.parse_slots(buf).tolist())
                elif t == P.F_STOP:
                    break
        finally:
            self._done_q.put(None)
            fin.join(60)
            self.alive.clear()
            close = getattr(self.servable, "close", None)  # e.g. release the group's followers
            if callable(close):
                close()

    def _completion_loop(self) -> None:
        while True:
            p = self._done_q.get()
            if p is None:
                return
            try:
                self._finalize(p)
            except (BrokenPipeError, EOFError, OSError):
                pass
            except Exception as e:  # never let the retire thread die: answer the batch, keep the count right
                self._fail_pending(p, e)
            finally:
                with self._idle:
                    self._inflight -= 1
                    self._idle.notify_all()

    def _fail_pending(self, p: _Pending, err: Exception) -> None:
        """A batch whose completion raised (device fault in the sync, an encode error): its valid items go
        back to the queue (IT_RETRY: another delivery, bounded by max-delivery) so no task stays 'running'
        until a lock expires. A device error is sticky (every later sync raises too): then the worker also
        stops heartbeating and exits, so the scheduler marks it dead and its restart path runs."""
        import sys

        print(f"[ai4e worker {self.rank}] batch {p.bid} completion failed ({err!r}); returning its items for retry",
              file=sys.stderr, flush=True)
        status = p.status.copy()
        status[p.valid] = P.IT_RETRY
        try:
            now = time.monotonic()
            self.conn.done(p.bid, status, bytes(p.n * self.row_bytes), self.row_bytes, (p.t_recv, now, now, 0, 0))
        except Exception:
            pass
        if self.device.type == "cuda" and not self._device_ok():
            self.alive.clear()
            print(f"[ai4e worker {self.rank}] device error is sticky; exiting", file=sys.stderr, flush=True)
            os._exit(19)

    def _device_ok(self) -> bool:
        try:
            torch.cuda.synchronize(self.device)
            return True
        except Exception:
            return False

    def _drain(self) -> None:
        with self._idle:
            self._idle.wait_for(lambda: self._inflight == 0, timeout=120)

    # ------------------------------------------------------------------ batches
    def _on_batch(self, buf: bytes) -> None:
        t_recv = time.monotonic()
        bid, slots = P.parse_batch(buf)
        n = slots.shape[0]
        self.batches += 1
        f = self.fault
        if "exit_after" in f and self.batches > f["exit_after"]:
            os._exit(17)
        if "hang_after" in f and self.batches > f["hang_after"]:
            self.alive.clear()  # heartbeats stop too
            time.sleep(3600)
        if f.get("delay_ms"):
            time.sleep(f["delay_ms"] / 1e3)
        status = np.zeros(n, np.uint8)
        valid = (slots >= 0) & (slots < self.nslots)
        status[~valid] = P.IT_INVALID
        vslots = slots[valid].tolist()
        if not vslots:
            self.conn.done(bid, status, bytes(n * self.row_bytes), self.row_bytes, (t_recv, t_recv, t_recv, 0, 0))
            return
        jpeg = self._jpeg_rows(vslots, status, valid)
        # the engine has 3 buffer sets: never launch a 3rd batch over one not yet retired
        with self._idle:
            self._idle.wait_for(lambda: self._inflight < self.engine.nbuf, timeout=120)
        try:
            if f.get("fail_batch") == self.batches:
                raise RuntimeError("injected batch launch failure")
            res = self.engine.submit(self.buf, vslots, jpeg=jpeg)
        except Exception as e:
            import sys

            print(f"[ai4e worker {self.rank}] batch {bid} launch failed ({e!r}); re-running its {len(vslots)} items "
                  "one by one", file=sys.stderr, flush=True)
            self.isolated_batches += 1
            self._drain()
            self._isolate(bid, slots, valid, status, t_recv)
            return
        with self._idle:
            self._inflight += 1
        self._done_q.put(_Pending(bid, n, valid, res, t_recv, status))

    def _jpeg_rows(self, vslots: List[int], status: np.ndarray, valid: np.ndarray):
        """[(batch row, prepared bytes, header, plan)] of the valid slots holding prepared JPEG frames; a marked slot
        whose header does not hold up is failed as an invalid payload (and its row computed from whatever it holds)."""
        if not self.jpeg_key:
            return None
        from .jpeg_gpu import header_sane, parse_header, plan_frame, slot_frames

        frames = slot_frames(self._ring_u8, vslots, self.jpeg_key)
        if not frames:
            return None
        h, w, c = self.spec.item_shape
        out = []
        vidx = np.nonzero(valid)[0]
        for j, used in frames:
            hdr = parse_header(self._ring_u8[vslots[j], :160].tobytes())
            plan = plan_frame(hdr, w, h, c) if header_sane(hdr, used) else None
            if plan is None:
                status[vidx[j]] = P.IT_INVALID
                continue
            out.append((j, used, hdr, plan))
        self.jpeg_frames += len(out)
        return out or None

    def _rows(self, n: int, valid: np.ndarray, outputs) -> bytes:
        nv = int(valid.sum())
        enc = encode_rows([o.numpy() if isinstance(o, torch.Tensor) else o for o in outputs], nv)
        if nv == n:
            return enc
        rows = np.zeros((n, self.row_bytes), np.uint8)
        rows[valid] = np.frombuffer(enc, np.uint8).reshape(nv, self.row_bytes)
        return rows.tobytes()

    def _finalize(self, p: _Pending) -> None:
        self._finalized = getattr(self, "_finalized", 0) + 1
        if self.fault.get("fail_finalize") == self._finalized:
            raise RuntimeError("injected completion failure")
        p.res.done.synchronize()
        t_done = time.monotonic()
        h2d_ms, comp_ms = p.res.gpu_ms()
        self.busy_ms += h2d_ms + comp_ms
        rows = self._rows(p.n, p.valid, p.res.outputs)
        self._mark_invalid(p.status, p.valid, p.res.outputs)
        bad = p.res.jpeg_failed()
        if bad:  # corrupt entropy-coded data in a prepared JPEG frame
            p.status[np.nonzero(p.valid)[0][bad]] = P.IT_INVALID
        if getattr(self.servable, "stages", 0):  # ensemble hop (AddPipelineTask) for this batch's tasks
            self.conn.stage(p.bid, 0)
        self.conn.done(p.bid, p.status, rows, self.row_bytes, (p.t_recv, p.res.t_launch, t_done, h2d_ms, comp_ms))

    def _mark_invalid(self, status: np.ndarray, valid: np.ndarray, outputs) -> None:
        """Servables that refuse single rows (``invalid_rows(outputs)`` -> bool per valid row, e.g. an extent record
        that did not come through the request decoder) fail those items alone as invalid payloads."""
        fn = getattr(self.servable, "invalid_rows", None)
        if fn is None:
            return
        bad = np.asarray(fn(outputs), bool)
        idx = np.nonzero(valid)[0]
        bad = bad[: idx.shape[0]]
        if bad.any():
            status[idx[bad]] = P.IT_INVALID

    def _isolate(self, bid: int, slots: np.ndarray, valid: np.ndarray, status: np.ndarray, t_recv: float) -> None:
        """Batch launch failed (pipeline already drained): run each valid item alone."""
        if self.device.type == "cuda":
            try:
                torch.cuda.synchronize(self.device)
            except Exception:
                pass
        n = slots.shape[0]
        rows = np.zeros((n, self.row_bytes), np.uint8)
        t_launch = time.monotonic()
        for i in np.nonzero(valid)[0].tolist():
            try:
                if self.fault.get("fail_item") == int(slots[i]):
                    raise RuntimeError("injected item failure")
                one = np.zeros(1, np.uint8)
                jpeg = self._jpeg_rows([int(slots[i])], one, np.ones(1, bool))
                res = self.engine.submit(self.buf, [int(slots[i])], jpeg=jpeg)
                res.done.synchronize()
                outs = [o.clone() for o in res.outputs]
                rows[i] = np.frombuffer(encode_rows([o.numpy() for o in outs], 1), np.uint8)
                self._mark_invalid(one, np.ones(1, bool), outs)
                if res.jpeg_failed():
                    one[0] = P.IT_INVALID
                status[i] = max(status[i], one[0])
            except Exception as e:  # this item fails on its own
                import sys
                print(f"[ai4e worker {self.rank}] item (slot {int(slots[i])}) failed alone: {e!r}", file=sys.stderr,
                      flush=True)
                status[i] = P.IT_ERROR
        if getattr(self.servable, "stages", 0):
            self.conn.stage(bid, 0)
        self.conn.done(bid, status, rows.tobytes(), self.row_bytes, (t_recv, t_launch, time.monotonic(), 0, 0))


def join_group(device: str, group_rank: int, group_size: int, port: int, n_leaders: int = 1):
    """Process group of one worker group (RCCL over xGMI between its GPUs; gloo on CPU). Stage-graph groups
    (``n_leaders`` > 1) also tell the factory its group rank and the number of leaders."""
    import datetime

    import torch.distributed as dist

    dev = torch.device(device)
    backend = "nccl" if dev.type == "cuda" else "gloo"
    kw = {"device_id": dev} if backend == "nccl" else {}
    dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=group_rank, world_size=group_size,
                            timeout=datetime.timedelta(seconds=600), **kw)
    kw = {"group": dist.group.WORLD, "role": "leader" if group_rank < n_leaders else "follower"}
    if n_leaders > 1:
        kw.update(group_rank=group_rank, n_leaders=n_leaders)
    return kw


def _share_cpu(dev: torch.device, spec: ModelSpec) -> None:
    """CPU worker groups (tests, CPU-only deployments): the group's processes share the host's cores instead of
    each running an intra-op pool as wide as the machine (8 processes x 8 threads on 8 cores thrash)."""
    if dev.type == "cpu" and spec.group_size > 1 and "OMP_NUM_THREADS" not in os.environ:
        torch.set_num_threads(max(1, (os.cpu_count() or 1) // spec.group_size))


def follower_main(device: str, spec: ModelSpec, group_rank: int, group_size: int, port: int) -> None:
    """A non-leader process of a worker group: builds its part of the model and serves the leader
    (``servable.serve_follower()`` returns when the leader releases the group)."""
    dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    _share_cpu(dev, spec)
    gk = join_group(device, group_rank, group_size, port, spec.group_leaders)
    part = load_factory(spec.factory)(device=device, **spec.kwargs, **gk)
    try:
        part.serve_follower()
    finally:
        import torch.distributed as dist

        if dist.is_initialized():
            dist.destroy_process_group()


def worker_main(conn, rank: int, device: str, spec: ModelSpec, shm_name: str, nslots: int, hb_interval: float,
                partition: Optional[Tuple[int, int]] = None, untrack: bool = False, local_ring=None,
                group_port: int = 0, ready_event: Optional[threading.Event] = None, group_rank: int = 0) -> None:
    """Entry point of a spawned worker process (and of ``torchrun`` worker ranks, which pass their
    ingest partition's ``local_ring`` and ``untrack=True``). With ``spec.group_size > 1`` this is the
    leader of a worker group (rendezvous on ``group_port``)."""
    dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    _share_cpu(dev, spec)
    group_kwargs = (join_group(device, group_rank, spec.group_size, group_port, spec.group_leaders)
                    if spec.group_size > 1 else None)
    shm, buf = attach_ring(shm_name, nslots, spec.item_shape, untrack=untrack)
    pinned = pin_host(buf) if dev.type == "cuda" else False
    if local_ring is None and partition is not None:
        from ..store import native

        local_ring = native.SlotRing(partition[1], partition[0])
    fc = conn if isinstance(conn, P.FrameConn) else P.FrameConn(conn)
    w = GpuWorker(fc, rank, device, spec, buf, local_ring=local_ring, hb_interval=hb_interval, group_kwargs=group_kwargs,
                  jpeg_key=ring_jpeg_key(shm, nslots, spec.item_shape))
    if ready_event is not None:  # graphs are captured: the hosting process may use the device again
        ready_event.set()
    try:
        w.serve(pinned)
    finally:
        if pinned:
            try:
                torch.cuda.cudart().cudaHostUnregister(buf.data_ptr())
            except Exception:
                pass
        del buf
        shm.close()
        if group_kwargs is not None:
            import torch.distributed as dist

            if dist.is_initialized():
                dist.destroy_process_group()
