"""Per-GPU inference engine: static device buffers, HIP-graph-captured forward, overlapped H2D/D2H.

One engine per MI355X (one process per GPU in the worker pool). The model forward (57 kernel
launches for ResNet-50) is captured once per (batch bucket, buffer) into a HIP graph
(``torch.cuda.CUDAGraph`` is hipGraph on ROCm), so a batch costs one graph launch instead of
dozens of Python-side launches. Inputs arrive as uint8 images in a pinned host ring
(:class:`PayloadRing`); contiguous slot runs are copied H2D on a dedicated copy stream while the
previous batch computes; only the top-k result (a few bytes per image) is copied back.
"""
from __future__ import annotations

import os
import threading
import time
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch


class PayloadRing:
    """Pinned host ring of fixed-shape request payloads (e.g. decoded uint8 images).

    ``alloc`` hands out slot indices in FIFO order so a batch received from the FIFO dispatch
    queue is (almost always) one contiguous run -> one DMA.
    """

    def __init__(self, nslots: int, item_shape: Sequence[int], dtype=torch.uint8, pin: bool = True):
        self.nslots = int(nslots)
        self.item_shape = tuple(item_shape)
        pin = pin and torch.cuda.is_available()
        self.buf = torch.empty((self.nslots, *self.item_shape), dtype=dtype, pin_memory=pin)
        self._head = 0
        self._used = 0
        self._free = [False] * self.nslots
        self._mu = threading.Condition()

    def alloc(self, n: int, timeout: Optional[float] = None) -> List[int]:
        with self._mu:
            if n > self.nslots:
                raise ValueError("request larger than the ring")
            if not self._mu.wait_for(lambda: self.nslots - self._used >= n, timeout):
                raise TimeoutError("payload ring full")
            start = (self._head + self._used) % self.nslots
            self._used += n
            return [(start + i) % self.nslots for i in range(n)]

    def free(self, slots: Sequence[int]) -> None:
        """Release slots; the ring head only advances over a contiguous freed prefix."""
        with self._mu:
            for s in slots:
                self._free[s] = True
            while self._used and self._free[self._head]:
                self._free[self._head] = False
                self._head = (self._head + 1) % self.nslots
                self._used -= 1
            self._mu.notify_all()

    def write(self, slot: int, data) -> None:
        self.buf[slot].copy_(torch.as_tensor(data))


def contiguous_runs(slots: Sequence[int]) -> List[Tuple[int, int, int]]:
    """[(dst_offset, src_start, length)] for runs of consecutive slot ids."""
    runs = []
    i = 0
    n = len(slots)
    while i < n:
        j = i + 1
        while j < n and slots[j] == slots[j - 1] + 1:
            j += 1
        runs.append((i, slots[i], j - i))
        i = j
    return runs


class _DoneEvent:
    def synchronize(self) -> None:
        return None

    def query(self) -> bool:
        return True


@dataclass
class BatchResult:
    outputs: List[torch.Tensor]  # per output: [n, ...] (pinned host views, valid after done)
    done: "torch.cuda.Event"
    n: int
    t_launch: float = 0.0        # host CLOCK_MONOTONIC at launch
    ev_copy0: Optional["torch.cuda.Event"] = None
    ev_copy1: Optional["torch.cuda.Event"] = None
    jpeg: Optional[Tuple[List[int], torch.Tensor]] = None  # (batch rows decoded from JPEG, their status, valid after done)

    def jpeg_failed(self) -> List[int]:
        """Batch rows whose prepared JPEG frame could not be decoded (corrupt data): their outputs are garbage."""
        if self.jpeg is None:
            return []
        idx, st = self.jpeg
        return [idx[k] for k in range(len(idx)) if int(st[k]) != 0]

    @property
    def top_idx(self) -> torch.Tensor:
        return self.outputs[0]

    @property
    def top_prob(self) -> torch.Tensor:
        return self.outputs[1]

    def gpu_ms(self) -> Tuple[float, float]:
        """(H2D copy ms, copy-end -> outputs-ready ms) once ``done`` has fired (0, 0 without timing)."""
        if self.ev_copy0 is None:
            return 0.0, 0.0
        return self.ev_copy0.elapsed_time(self.ev_copy1), self.ev_copy1.elapsed_time(self.done)


class InferenceEngine:
    """Runs ``output_fn(u8 [b,H,W,C] on device) -> tuple of [b, ...] tensors`` with HIP graphs and
    3-deep buffering. Without ``output_fn`` the engine is a classifier: ``head_fn`` (a fused top-k,
    e.g. ``FusedResNet.topk_u8``) or softmax/top-k over ``model_fn``'s logits."""

    def __init__(self, model_fn: Optional[Callable[[torch.Tensor], torch.Tensor]], item_shape: Sequence[int],
                 max_batch: int, device: Optional[torch.device] = None, topk: int = 5, use_graphs: bool = True,
                 nbuf: int = 4, buckets: Optional[Sequence[int]] = None,
                 head_fn: Optional[Callable[[torch.Tensor, int], Tuple[torch.Tensor, torch.Tensor]]] = None,
                 output_fn: Optional[Callable[[torch.Tensor], Sequence[torch.Tensor]]] = None, timing: bool = False):
        self.model_fn = model_fn
        self.head_fn = head_fn
        self.output_fn = output_fn
        self.device = torch.device(device or "cuda")
        self.item_shape = tuple(item_shape)
        self.max_batch = max_batch
        self.topk = topk
        self.use_graphs = use_graphs and self.device.type == "cuda"
        self.timing = timing and self.device.type == "cuda"
        self.nbuf = max(nbuf, int(os.environ.get("AI4E_ENGINE_NBUF", "0")))
        self.buckets = sorted(set(buckets or [max_batch]))
        if self.buckets[-1] != max_batch:
            self.buckets.append(max_batch)
        cuda = self.device.type == "cuda"
        self.copy_stream = torch.cuda.Stream(self.device) if cuda else None
        self.compute_stream = torch.cuda.Stream(self.device) if cuda else None
        # AI4E_ENGINE_STREAMS (default 2): consecutive batches replay on alternating compute streams, so the tail of
        # batch i (layer3/4 grids smaller than the 256-CU machine) can overlap the head of batch i+1
        # (ResNet-50 @250: +1.5-1.9 % images/s same-box A/B, p99 14.1 -> 10.9 ms; profiles/r2_pool/)
        ns = int(os.environ.get("AI4E_ENGINE_STREAMS", "2")) if cuda else 1
        self.compute_streams = [self.compute_stream] + [torch.cuda.Stream(self.device) for _ in range(ns - 1)]
        self.inputs = [torch.empty((max_batch, *self.item_shape), dtype=torch.uint8, device=self.device)
                       for _ in range(self.nbuf)]
        self.host_out: List[List[torch.Tensor]] = [[] for _ in range(self.nbuf)]  # allocated at warmup
        self.graphs: Dict[Tuple[int, int], torch.cuda.CUDAGraph] = {}
        self._graph_out: Dict[Tuple[int, int], Tuple[torch.Tensor, ...]] = {}
        self.compute_done: List[Optional[torch.cuda.Event]] = [None] * self.nbuf
        self._k = 0
        # JPEG frames prepared into ring slots (runtime/jpeg_gpu.py): decoded on the copy stream into the input rows
        self._jpeg = None
        self._jpeg_scan: List[Optional[torch.Tensor]] = [None] * self.nbuf
        self._jpeg_host: List[Optional[torch.Tensor]] = [None] * self.nbuf
        # (measured and removed in round 5: the phase-offset front/back split and the CU-partitioned pipeline,
        # both slower than two full-chip streams; profiles/r3_cusplit/, patches in profiles/r5_pruned/)

    # -------------------------------------------------------------- forward
    def _forward_into(self, buf: int, b: int) -> Tuple[torch.Tensor, ...]:
        x = self.inputs[buf][:b]
        if self.output_fn is not None:
            return tuple(self.output_fn(x))
        if self.head_fn is not None:
            i, p = self.head_fn(x, self.topk)
            return i, p
        logits = self.model_fn(x)
        p, i = torch.topk(torch.softmax(logits.float(), dim=1), self.topk, dim=1)
        return i.to(torch.int32), p

    def bucket_for(self, n: int) -> int:
        for b in self.buckets:
            if b >= n:
                return b
        raise ValueError(f"batch {n} > max_batch {self.max_batch}")

    def _alloc_host(self, outs: Sequence[torch.Tensor]) -> None:
        pin = self.device.type == "cuda"
        for buf in range(self.nbuf):
            self.host_out[buf] = [torch.empty((self.max_batch, *o.shape[1:]), dtype=o.dtype, pin_memory=pin)
                                  for o in outs]

    def warmup(self) -> None:
        """Run every (bucket, buffer) once eagerly (kernel load / allocator warm) then capture graphs."""
        if self.device.type != "cuda":
            return
        with torch.cuda.stream(self.compute_stream):
            for buf in range(self.nbuf):
                self.inputs[buf].zero_()
                for b in self.buckets:
                    outs = self._forward_into(buf, b)
        torch.cuda.synchronize(self.device)
        self._alloc_host(outs)
        if not self.use_graphs:
            return
        for buf in range(self.nbuf):
            for b in self.buckets:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=self.compute_stream):
                    outs = self._forward_into(buf, b)
                self.graphs[(buf, b)] = g
                self._graph_out[(buf, b)] = outs
        torch.cuda.synchronize(self.device)

    # -------------------------------------------------------------- submit
    def submit(self, host_src: torch.Tensor, slots: Sequence[int], jpeg=None) -> BatchResult:
        """Copy ``host_src[slots]`` to the next device buffer, run, and return an async result. ``jpeg``: [(batch row,
        prepared bytes, header, plan)] of the rows whose slot holds a prepared JPEG frame (runtime/jpeg_gpu.py): those
        are decoded on the copy stream straight into their input rows instead of copied."""
        n = len(slots)
        t_launch = time.monotonic()
        if self.device.type != "cuda":  # CPU path (tests / CPU-only hosts): synchronous
            x = host_src[list(slots)]
            st = None
            if jpeg:
                from .jpeg_gpu import decode_prepared_cpu

                x = x.clone()
                st = torch.zeros(len(jpeg), dtype=torch.int32)
                for k, (j, used, _, _) in enumerate(jpeg):
                    img = decode_prepared_cpu(host_src[slots[j]].reshape(-1)[:used].numpy(), self.item_shape)
                    if img is None:
                        st[k] = 2
                        x[j].zero_()
                    else:
                        x[j].copy_(torch.from_numpy(img))
            outs = self.run_sync(x)
            return BatchResult(list(outs), _DoneEvent(), n, t_launch,
                               jpeg=([j for j, _, _, _ in jpeg], st) if jpeg else None)
        if not self.host_out[0]:
            raise RuntimeError("InferenceEngine.warmup() must run before submit() on a GPU")
        buf = self._k % self.nbuf
        self._k += 1
        b = self.bucket_for(n)
        dev_in = self.inputs[buf]
        cs = self.copy_stream
        # the copy into `buf` must not overwrite an input the compute stream is still reading
        # (only the batch that last used this buffer; the previous batch keeps computing)
        if self.compute_done[buf] is not None:
            cs.wait_event(self.compute_done[buf])
        ev0 = ev1 = None
        if self.timing:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record(cs)
        jstatus = None
        with torch.cuda.stream(cs):
            if not jpeg:
                for dst, src, ln in contiguous_runs(list(slots)):
                    dev_in[dst:dst + ln].copy_(host_src[src:src + ln], non_blocking=True)
            else:
                jstatus = self._submit_jpeg(buf, host_src, slots, jpeg, dev_in, cs)
        ev = torch.cuda.Event(enable_timing=self.timing)
        ev.record(cs)
        if self.timing:
            ev1 = ev
        st = self.compute_streams[buf % len(self.compute_streams)]
        st.wait_event(ev)
        with torch.cuda.stream(st):
            if self.use_graphs and (buf, b) in self.graphs:
                self.graphs[(buf, b)].replay()
                outs = self._graph_out[(buf, b)]
            else:
                outs = self._forward_into(buf, b)
            host = self.host_out[buf]
            for h, o in zip(host, outs):
                h[:n].copy_(o[:n], non_blocking=True)
            jres = None
            if jstatus is not None:
                hs = self._jpeg_host[buf]
                if hs is None or hs.numel() < jstatus.numel():
                    hs = self._jpeg_host[buf] = torch.zeros(max(self.max_batch, jstatus.numel()), dtype=torch.int32,
                                                            pin_memory=True)
                hs[:jstatus.numel()].copy_(jstatus, non_blocking=True)
                jstatus.record_stream(st)  # (allocated on the copy stream, read here)
                jres = ([j for j, _, _, _ in jpeg], hs[:jstatus.numel()])
            done = torch.cuda.Event(enable_timing=self.timing)
            done.record(st)
        self.compute_done[buf] = done
        return BatchResult([h[:n] for h in self.host_out[buf]], done, n, t_launch, ev0, ev1, jres)

    def _submit_jpeg(self, buf: int, host_src: torch.Tensor, slots: Sequence[int], jpeg, dev_in: torch.Tensor, cs):
        """(on the copy stream) raw rows by contiguous runs; prepared JPEG rows: their bytes into a device scan area,
        then the decode kernels write the rows. Returns the per-frame status (device)."""
        from .jpeg_gpu import JpegLauncher, _align

        if self._jpeg is None:
            self._jpeg = JpegLauncher(self.device)
        jrows = {j for j, _, _, _ in jpeg}
        raw = [(j, s) for j, s in enumerate(slots) if j not in jrows]
        i = 0
        while i < len(raw):
            k = i + 1
            while k < len(raw) and raw[k][0] == raw[k - 1][0] + 1 and raw[k][1] == raw[k - 1][1] + 1:
                k += 1
            d0, s0 = raw[i]
            dev_in[d0:d0 + (k - i)].copy_(host_src[s0:s0 + (k - i)], non_blocking=True)
            i = k
        offs, total = [], 0
        for _, used, _, _ in jpeg:
            offs.append(total)
            total += _align(used)
        scan = self._jpeg_scan[buf] = self._jpeg.grow(self._jpeg_scan[buf], total)
        flat = host_src.view(host_src.shape[0], -1)
        for (j, used, _, _), o in zip(jpeg, offs):
            scan[o:o + used].copy_(flat[slots[j], :used], non_blocking=True)
        base = scan.data_ptr()
        frames = [(hdr, plan, base + o, dev_in[j].data_ptr()) for (j, _, hdr, plan), o in zip(jpeg, offs)]
        status, _keep = self._jpeg.launch(frames, cs)
        return status

    def run_sync(self, images_u8: torch.Tensor) -> Tuple[torch.Tensor, ...]:
        """Convenience (sync API / tests): images already on host or device."""
        if self.device.type != "cuda":
            self.inputs[0][: images_u8.shape[0]].copy_(images_u8)
            return tuple(o.cpu() for o in self._forward_into(0, images_u8.shape[0]))
        host = images_u8.cpu().pin_memory() if not images_u8.is_pinned() else images_u8
        res = self.submit(host, list(range(images_u8.shape[0])))
        res.done.synchronize()
        return tuple(o.clone() for o in res.outputs)
