"""Detector -> classifier ensemble over RCCL send/recv (BASELINE config #5; ``AddPipelineTask``).

The reference chains APIs by re-publishing the same TaskId to the next endpoint
(``APIs/1.0/Common/task_management/distributed_api_task.py:67-100``,
``CacheConnectorUpsert.cs:144-176``): every hop is queue -> HTTP -> JSON. Here the stages are
GPU ranks of one node and the hand-off is a tensor over xGMI (:class:`StageGraphPipeline`, N detector GPUs : M
classifier GPUs of one group; 1:1 is the pair form):

* detector ranks run Faster-RCNN on a batch, pick the confident animal boxes, crop + bilinear-resize
  them on the GPU to uint8 ``[N, 224, 224, 3]`` (``crop_resize_u8``, K5/K7: 147 KiB per crop, the
  classifier's own input format, half the bytes of fp16 and a sixth of a bf16x8 stem tensor) and
  send a fixed-size message to their classifier rank over RCCL: a device-side header (crop count, capacity)
  and the capacity-sized crop buffer, valid crops first. The detector never reads the count on the host: its
  hand-off is stream-ordered behind its graph replay, so consecutive replays never drain to the host;
* classifier ranks ``recv`` the header, the crops, run the crop classifier (fused ResNet-50, bf16 or fp16) on
  the valid prefix and send back ``[capacity, 2]`` (class, probability), whose receive the detector posted
  with its send;
* a detector keeps one batch in flight: it sends batch i, starts detecting batch i+1, then collects batch
  i's classifications — compute and transfer overlap; message order per pair is fixed (header, payload,
  results) so the pairing can never deadlock;
* the task record keeps one TaskId across both stages (``stage_transition`` /
  ``TaskStore.retarget_many``): created@detector -> running -> created@classifier
  ("AddPipelineTask") -> running -> completed.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..ops.debug import crumb
from ..ops.detection import crop_resize_u8
from ..store import STATE_COMPLETED, STATE_CREATED, STATE_RUNNING

STOP = -1


@dataclass
class PipelineConfig:
    crop_hw: Tuple[int, int] = (224, 224)
    score_thresh: float = 0.5
    class_id: Optional[int] = 1    # MegaDetector "animal"; None = every class
    max_crops_per_image: int = 8
    # crops on the RCCL wire between detector and classifier GPUs: "uint8" (3 B/px, exact classifier
    # input) or "float16" (6 B/px, rounded back to uint8 on receipt)
    wire_dtype: str = "uint8"


def stage_transition(store, task_ids: Sequence[str], next_endpoint: str, status: str = "running - classifying"):
    """AddPipelineTask analogue: same TaskIds re-targeted at the next stage's endpoint."""
    for t in task_ids:
        store.upsert(t, STATE_CREATED, STATE_CREATED, next_endpoint, None, False)
    store.transition_many(list(task_ids), STATE_RUNNING, status)


# ----------------------------------------------------------------------------------------------------------
# N:M stage graph (config 5 at node scale): L detector GPUs feed M classifier GPUs of one RCCL group.
# ----------------------------------------------------------------------------------------------------------
def stage_assignment(n_leaders: int, world: int) -> List[List[int]]:
    """Classifier c (group rank n_leaders + c) serves detectors d with d % M == c (M = world - n_leaders):
    a fixed map, so each detector always talks to one classifier and the P2P pairs (and RCCL's per-pair
    communicators) never change. Ratio: sized by measured stage rates, e.g. 7:1 on an 8-GPU node when one
    GPU classifies the crops of seven detectors (bench/api_bench.py --model ensemble_group)."""
    m = world - n_leaders
    if n_leaders < 1 or m < 1:
        raise ValueError(f"stage graph needs >= 1 detector and >= 1 classifier rank, got {n_leaders}:{m}")
    return [[d for d in range(n_leaders) if d % m == c] for c in range(m)]


def _fault_at() -> int:
    """AI4E_FAULT_INJECTION=xgmi_fail_batch=<k>: the k-th hand-off of a detector fails before anything is on the
    wire (a lost / refused P2P transfer; survey §5.3)."""
    for item in filter(None, os.environ.get("AI4E_FAULT_INJECTION", "").split(",")):
        k, _, v = item.partition("=")
        if k.strip() == "xgmi_fail_batch":
            return int(v.split("@")[0])
    return 0


class _Arrivals:
    """Event-driven completion of posted receives, one form for every backend: ``post(d, work)`` hands the receive
    of detector ``d`` to a waiter thread and ``next()`` blocks until any posted receive has landed. On gloo the waiter
    blocks in ``work.wait()`` (gloo completes a receive only there); on RCCL the work is made a dependency of a
    per-detector side stream and the waiter sleeps in a blocking-sync HIP event recorded behind it (no NCCL call off
    the serving thread, no polling)."""

    def __init__(self, device: torch.device, blocking_wait: bool):
        import queue
        import threading

        self.device, self.blocking = device, blocking_wait
        self.ready: "queue.Queue" = queue.Queue()
        self._threading = threading
        self._streams: dict = {}

    def post(self, d: int, work) -> None:
        if self.blocking or self.device.type != "cuda":
            target = work.wait
        else:
            s = self._streams.get(d)
            if s is None:
                s = self._streams[d] = torch.cuda.Stream(device=self.device)
            with torch.cuda.stream(s):
                work.wait()  # (RCCL: the side stream waits for the receive)
            ev = torch.cuda.Event(blocking=True)
            ev.record(s)
            target = ev.synchronize

        def waiter():
            err = None
            try:
                target()
            except Exception as e:  # (surfaced by next() on the serving thread)
                err = e
            self.ready.put((d, err))
        self._threading.Thread(target=waiter, daemon=True).start()

    def next(self) -> int:
        d, err = self.ready.get()
        if err is not None:
            raise err
        return d


def plan_ensemble(gpus: int, det_images_per_s: float, cls_crops_per_s: float, crops_per_image: float,
                  colocated_images_per_s: Optional[float] = None) -> dict:
    """Placement of config 5 on ``gpus`` GPUs from measured stage rates (bench/stage_rates.py): every N:M stage
    graph (N detector GPUs, M = gpus - N classifier GPUs; node rate = min(N x detector rate, M x classifier rate /
    crops per image)) against the colocated form (both stages on every GPU, DP; per GPU 1 / (1/det + c/cls), or
    the measured colocated rate). Returns the fastest as {"form": "stage" | "colocated", "leaders", "classifiers",
    "images_per_s"} plus every candidate's estimate."""
    c = max(float(crops_per_image), 1e-9)
    cands = []
    for n in range(1, gpus):
        m = gpus - n
        cands.append({"form": "stage", "leaders": n, "classifiers": m,
                      "images_per_s": min(n * det_images_per_s, m * cls_crops_per_s / c)})
    per_gpu = colocated_images_per_s or 1.0 / (1.0 / det_images_per_s + c / cls_crops_per_s)
    cands.append({"form": "colocated", "leaders": gpus, "classifiers": 0, "images_per_s": gpus * per_gpu})
    best = max(cands, key=lambda x: x["images_per_s"])
    return dict(best, candidates=cands)


class _GraphRunner:
    """One static-shape callable captured per input size in HIP graphs (CUDA graphs on ROCm); eager on CPU."""

    def __init__(self, fn: Callable, device: torch.device, warmup: int = 2):
        self.fn, self.device, self.warmup = fn, device, warmup
        self.graphs: dict = {}

    def __call__(self, x: torch.Tensor):
        if self.device.type != "cuda":
            return self.fn(x)
        key = tuple(x.shape)
        g = self.graphs.get(key)
        if g is None:
            # the engine's capture pattern (runtime/engine.py warmup): eager warmup on the capture stream
            # itself, the device drained, then the capture on that same stream
            static_in = x.clone()
            s = torch.cuda.Stream(device=self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                for _ in range(self.warmup):
                    self.fn(static_in)
            torch.cuda.synchronize(self.device)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=s):
                static_out = self.fn(static_in)
            torch.cuda.synchronize(self.device)
            g = self.graphs[key] = (graph, static_in, static_out)
        graph, static_in, static_out = g
        # stream-ordered: back-to-back replays need no host sync (the round-3/4 replay fault was the library's
        # multi-block top-k inside the detector graph, now rpn_topk; profiles/r4_replay/, tests/test_graph_replay_gpu.py).
        # Every sort in the captured forward is a HIP row sort (rpn_topk, sort_select); a shape past their limit makes
        # the capture itself raise (ops.detection._graph_safe_fallback) instead of capturing a library sort, so no
        # graph reaching this replay holds library temporaries (tests/test_detector_cpu.py pins the default shapes)
        static_in.copy_(x)
        graph.replay()
        return static_out


class StageGraphPipeline:
    """Group ranks [0, L) detect + crop, ranks [L, L + M) classify crops (stage_assignment).

    Detector rank: ``run_batches`` per image batch — a captured graph does detection, crop selection
    (``models.zoo.select_crops_padded``: the first ``max_crops`` confident boxes per image), the uint8 224^2
    crop-resize (K5/K7) and the compaction of the valid crops to a prefix; the count comes back to the host,
    ``n`` and the ``n`` crops go to the rank's classifier over RCCL P2P (xGMI), one batch in flight.
    Classifier rank: ``serve`` posts a header ``irecv`` for every detector it serves and handles whichever
    arrives first (no head-of-line blocking behind an idle detector), runs the classifier on the crops in a
    graph captured per bucket size and sends back ``[n, 2]`` (class, probability). A detector's STOP header
    retires it; the classifier returns when all of its detectors have stopped.
    """

    BUCKETS = (8, 16, 32, 64, 128, 256, 512, 1024)

    def __init__(self, detector: Optional[Callable], classifier: Optional[Callable], device: torch.device,
                 cfg: PipelineConfig, group=None, n_leaders: int = 1, crop_dtype: torch.dtype = torch.uint8):
        self.detector, self.classifier, self.device, self.cfg, self.group = detector, classifier, device, cfg, group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.n_leaders = n_leaders
        self.is_detector = self.rank < n_leaders
        if self.world == 1:  # both stages in this process (no wire)
            self.assign, self.peer, self.serves = [], None, []
        else:
            self.assign = stage_assignment(n_leaders, self.world)
            m = self.world - n_leaders
            self.peer = n_leaders + self.rank % m if self.is_detector else None
            self.serves = self.assign[self.rank - n_leaders] if not self.is_detector else []
        self.wire_dtype = getattr(torch, cfg.wire_dtype)
        self.bytes_sent = self.bytes_received = 0
        self._handoffs, self._fail_at = 0, _fault_at()
        self._det_graph = _GraphRunner(self._detect_crop_compact, device) if self.is_detector else None
        self._cls_graph = _GraphRunner(self._classify_static, device) if classifier is not None else None

    # ------------------------------------------------------------ detector stage
    def _detect_crop_compact(self, images: torch.Tensor):
        from ..models.zoo import select_crops_padded

        b, m = images.shape[0], self.cfg.max_crops_per_image
        dets = self.detector(images)
        crumb("pipe.detected", dets[0])
        boxes, scores, valid = select_crops_padded(dets, m, self.cfg.score_thresh, self.cfg.class_id)
        crumb("pipe.selected", boxes)
        img = torch.arange(b, device=boxes.device, dtype=torch.float32)[:, None, None].expand(b, m, 1)
        crops = crop_resize_u8(images[..., :3].contiguous() if images.shape[-1] != 3 else images,
                               torch.cat([img, boxes], -1).reshape(b * m, 5), self.cfg.crop_hw)
        crumb("pipe.cropped", crops)
        flat = valid.reshape(-1)
        # (a 2-D innermost-dim cumsum: the library's own scan kernel; a 1-D cumsum goes to a device-wide library scan
        # with temporaries, kept out of captured graphs, profiles/r4_replay/)
        pos = torch.cumsum(flat.int().reshape(1, -1), 1).reshape(-1) - 1
        dst = torch.where(flat, pos, torch.full_like(flat, b * m, dtype=torch.int32))
        h, w = self.cfg.crop_hw
        packed = torch.zeros(b * m + 1, h, w, 3, dtype=torch.uint8, device=crops.device)
        packed.index_copy_(0, dst.long(), crops)           # valid crops first, in (image, score) order
        count = flat.sum().reshape(1).to(torch.int64)
        crumb("pipe.compacted", count)
        return dets, boxes, scores, valid, packed[: b * m].to(self.wire_dtype), count

    def _send(self, crops: torch.Tensor, count: torch.Tensor):
        """Non-blocking, and without the crop count on the host: a device-side header [count, capacity] and the
        whole capacity-sized crop buffer (valid crops first) go to the classifier, and the receive of its
        [capacity, 2] answer is posted right behind. The crops leave through a pair of preallocated wire buffers used
        alternately (batch i in buffer i % 2): the detector graph's static output is rewritten by the next replay
        while this send may still read, and batch i + 2 waits (stream-side on RCCL) for batch i's send before it
        reuses the buffer — one device copy into a resident buffer per batch, no allocation. Returns the works to
        wait for and the answer tensor."""
        self._handoffs += 1
        if self._fail_at and self._handoffs == self._fail_at:
            raise RuntimeError(f"injected xGMI hand-off failure (batch {self._handoffs})")
        cap = crops.shape[0]
        hdr = torch.empty(2, dtype=torch.int64, device=self.device)
        hdr[:1].copy_(count.reshape(1))
        hdr[1:].fill_(cap)
        k = self._handoffs % 2
        wire = self._wire_buffer(crops)
        for w in self._buf_works[k]:  # batch i - 2's send out of this buffer has finished reading it
            w.wait()
        wire.copy_(crops)
        sends = [dist.isend(hdr, group_dst=self.peer, group=self.group),
                 dist.isend(wire, group_dst=self.peer, group=self.group)]
        self._buf_works[k] = sends
        self._hdr_keep[k] = hdr  # (alive until its send is done)
        self.bytes_sent += hdr.numel() * 8 + wire.numel() * wire.element_size()
        res = torch.empty(cap, 2, device=self.device)
        rw = dist.irecv(res, group_src=self.peer, group=self.group)
        return rw, res

    def _wire_buffer(self, crops: torch.Tensor) -> torch.Tensor:
        """The ping-pong wire buffer of this hand-off (sized to the detector batch's crop capacity)."""
        if not hasattr(self, "_wire") or self._wire[0].shape != crops.shape or self._wire[0].dtype != crops.dtype:
            for ws in getattr(self, "_buf_works", [[], []]):  # (the old buffers' sends finish before they go)
                for w in ws:
                    w.wait()
            self._wire = [torch.empty_like(crops), torch.empty_like(crops)]
            self._buf_works, self._hdr_keep = [[], []], [None, None]
        return self._wire[self._handoffs % 2]

    def run_batches(self, batches: Sequence[torch.Tensor], padded: bool = False) -> List[Tuple]:
        """Detector rank: per batch (boxes [B, M, 4], det scores [B, M], valid [B, M], classes [n, 2] for the
        valid crops in (image, score) order), one batch's crops on the wire while the next one is detected.
        ``padded``: (boxes, scores, valid, classes [B * M, 2] — the valid crops' rows first —, count [1]) with no
        host synchronization at all (the serving path: every tensor stays stream-ordered on the device)."""
        out, pending = [], None

        def finish(p):
            boxes, scores, valid, count, rw, res = p
            rw.wait()  # (RCCL: stream-ordered; gloo: blocks)
            self.bytes_received += res.numel() * res.element_size()
            if padded:
                return boxes, scores, valid, res, count
            return boxes, scores, valid, res[: int(count.item())]

        for imgs in batches:
            _, boxes, scores, valid, crops, count = self._det_graph(imgs)
            boxes, scores, valid = boxes.clone(), scores.clone(), valid.clone()  # (graph outputs are reused)
            if self.world == 1:
                if padded:
                    res = torch.zeros(crops.shape[0], 2, device=self.device)
                    n = int(count.item())
                    res[:n] = self.classify(crops[:n])
                    out.append((boxes, scores, valid, res, count.clone()))
                else:
                    out.append((boxes, scores, valid, self.classify(crops[: int(count.item())])))
                continue
            rw, res = self._send(crops, count)
            if pending is not None:
                out.append(finish(pending))
            pending = (boxes, scores, valid, count.clone(), rw, res)
        if pending is not None:
            out.append(finish(pending))
        return out

    def stop(self) -> None:
        if self.world > 1 and self.is_detector:
            for ws in getattr(self, "_buf_works", []):
                for w in ws:
                    w.wait()
            dist.send(torch.tensor([STOP, 0], dtype=torch.int64, device=self.device), group_dst=self.peer,
                      group=self.group)

    # ------------------------------------------------------------ classifier stage
    def _classify_static(self, crops_u8: torch.Tensor) -> torch.Tensor:
        p = torch.softmax(self.classifier(crops_u8).float(), 1)
        prob, cls = p.max(1)
        return torch.stack([cls.float(), prob], 1)

    def classify(self, crops: torch.Tensor) -> torch.Tensor:
        n = crops.shape[0]
        if n == 0:
            return torch.zeros(0, 2, device=self.device)
        crops = crops if crops.dtype == torch.uint8 else crops.round().clamp(0, 255).to(torch.uint8)
        bucket = next((b for b in self.BUCKETS if b >= n), None)
        if bucket is None:  # (more crops than the largest captured bucket: in bucket-sized chunks)
            return torch.cat([self.classify(crops[i:i + self.BUCKETS[-1]]) for i in range(0, n, self.BUCKETS[-1])])
        if bucket != n:
            pad = torch.zeros(bucket, *crops.shape[1:], dtype=crops.dtype, device=crops.device)
            pad[:n] = crops
            crops = pad
        return self._cls_graph(crops)[:n].clone()

    def _headers(self):
        """Yield (detector, count, capacity) as headers arrive from the detectors this rank serves: one posted
        ``irecv`` per detector, completed event-driven (``_Arrivals``), so an idle detector never blocks a busy one.
        A detector's next header is posted only after its crops were received, so every posted receive matches a
        header."""
        arrivals = _Arrivals(self.device, dist.get_backend(self.group) == "gloo")
        hdrs = {d: torch.zeros(2, dtype=torch.int64, device=self.device) for d in self.serves}

        def post(d):
            arrivals.post(d, dist.irecv(hdrs[d], group_src=d, group=self.group))
        for d in self.serves:
            post(d)
        live = len(self.serves)
        while live:
            d = arrivals.next()
            n, cap = (int(v) for v in hdrs[d].tolist())
            yield d, n, cap  # (the crops are received before this detector's next header is posted)
            if n == STOP:
                live -= 1
            else:
                post(d)

    def serve(self) -> int:
        """Classifier rank loop; returns the number of crops classified."""
        h, w = self.cfg.crop_hw
        total = 0
        for d, n, cap in self._headers():
            if n == STOP:
                continue
            crops = torch.empty(cap, h, w, 3, dtype=self.wire_dtype, device=self.device)
            dist.recv(crops, group_src=d, group=self.group)
            self.bytes_received += crops.numel() * crops.element_size()
            res = torch.zeros(cap, 2, device=self.device)
            if n:
                res[:n] = self.classify(crops[:n])
            dist.send(res, group_dst=d, group=self.group)
            self.bytes_sent += res.numel() * res.element_size()
            total += n
        return total
