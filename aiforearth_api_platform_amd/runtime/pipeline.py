"""Detector -> classifier ensemble over RCCL send/recv (BASELINE config #5; ``AddPipelineTask``).

The reference chains APIs by re-publishing the same TaskId to the next endpoint
(``APIs/1.0/Common/task_management/distributed_api_task.py:67-100``,
``CacheConnectorUpsert.cs:144-176``): every hop is queue -> HTTP -> JSON. Here the stages are
GPU ranks of one node and the hand-off is a tensor over xGMI:

* detector ranks run Faster-RCNN on a batch, pick the animal boxes, crop + resize + normalise them
  on the GPU (``crop_resize_nhwc``, K5) and ``send`` a count header then the bf16 crops
  ``[N, 224, 224, 8]`` (≈0.8 MiB per crop) to their paired classifier rank over RCCL;
* classifier ranks ``recv`` the count, the crops, run the crop classifier (fused ResNet-50 on
  K1) and send back ``[N, 2]`` (class, probability);
* the detector side keeps one batch in flight: it sends batch i, starts detecting batch i+1, then
  collects batch i's classifications — compute and transfer overlap; message order is fixed
  (header, payload, results) so the pairing can never deadlock;
* the task record keeps one TaskId across both stages (``stage_transition``): created@detector ->
  running -> created@classifier ("AddPipelineTask") -> running -> completed.

Pairing: with ``world`` ranks, rank 2i (detector) talks to rank 2i+1 (classifier). ``world == 1``
runs both stages on one GPU with a local hand-off (no RCCL), same code path otherwise.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..ops.detection import crop_resize_nhwc
from ..store import STATE_COMPLETED, STATE_CREATED, STATE_RUNNING

STOP = -1


@dataclass
class PipelineConfig:
    crop_hw: Tuple[int, int] = (224, 224)
    score_thresh: float = 0.5
    class_id: Optional[int] = 1    # MegaDetector "animal"; None = every class
    max_crops_per_image: int = 8
    # dtype of the crops on the RCCL wire between detector and classifier GPUs (BASELINE config #5: fp16);
    # the classifier computes in bf16 and converts on receipt. CPU ranks (gloo) keep fp32.
    wire_dtype: str = "float16"


def select_crops(dets, cfg: PipelineConfig) -> torch.Tensor:
    """Padded detections -> boxes [N, 5] (img, x1, y1, x2, y2) of confident target-class boxes."""
    boxes, scores, labels, n = dets
    B, D = scores.shape
    rank = torch.arange(D, device=scores.device)[None].expand(B, D)
    ok = (rank < n[:, None].long()) & (scores > cfg.score_thresh)
    if cfg.class_id is not None:
        ok &= labels == cfg.class_id
    # cap per image (detections are score-sorted)
    ok &= torch.cumsum(ok.int(), 1) <= cfg.max_crops_per_image
    img = torch.arange(B, device=scores.device, dtype=torch.float32)[:, None].expand(B, D)
    sel = torch.cat([img[..., None], boxes], -1)[ok]
    return sel


def stage_transition(store, task_ids: Sequence[str], next_endpoint: str, status: str = "running - classifying"):
    """AddPipelineTask analogue: same TaskIds re-targeted at the next stage's endpoint."""
    for t in task_ids:
        store.upsert(t, STATE_CREATED, STATE_CREATED, next_endpoint, None, False)
    store.transition_many(list(task_ids), STATE_RUNNING, status)


class DetectClassifyPipeline:
    def __init__(self, detector: Callable, classifier: Callable[[torch.Tensor], torch.Tensor], device: torch.device,
                 cfg: Optional[PipelineConfig] = None, group=None):
        self.detector = detector        # uint8 NHWC images -> padded detections tuple
        self.classifier = classifier    # normalized bf16 crops [N, h, w, 8] -> logits [N, K]
        self.device = device
        self.cfg = cfg or PipelineConfig()
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.is_detector = self.world == 1 or self.rank % 2 == 0
        self.peer = self.rank + 1 if self.rank % 2 == 0 else self.rank - 1
        if self.world > 1 and self.peer >= self.world:
            raise ValueError("pipeline needs an even number of ranks (detector/classifier pairs)")
        self.crop_dtype = torch.bfloat16 if device.type == "cuda" else torch.float32  # classifier compute dtype
        self.wire_dtype = getattr(torch, self.cfg.wire_dtype) if device.type == "cuda" else torch.float32

    # ------------------------------------------------------------ classifier stage
    def classify(self, crops: torch.Tensor) -> torch.Tensor:
        if crops.shape[0] == 0:
            return torch.zeros(0, 2, device=self.device)
        p = torch.softmax(self.classifier(crops).float(), 1)
        prob, cls = p.max(1)
        return torch.stack([cls.float(), prob], 1)

    def serve_classifier(self) -> int:
        """Classifier-rank loop: until the detector sends STOP. Returns #crops classified."""
        total = 0
        h, w = self.cfg.crop_hw
        hdr = torch.zeros(1, dtype=torch.int64, device=self.device)
        while True:
            dist.recv(hdr, self.peer, group=self.group)
            n = int(hdr.item())
            if n == STOP:
                return total
            crops = torch.empty(n, h, w, 8, dtype=self.wire_dtype, device=self.device)
            if n:
                dist.recv(crops, self.peer, group=self.group)
            res = self.classify(crops.to(self.crop_dtype))
            if n:
                dist.send(res.contiguous(), self.peer, group=self.group)
            total += n

    # ------------------------------------------------------------ detector stage
    def _detect_and_crop(self, images: torch.Tensor):
        dets = self.detector(images)
        boxes = select_crops(dets, self.cfg)
        crops = crop_resize_nhwc(images, boxes, self.cfg.crop_hw).to(self.crop_dtype)
        return dets, boxes, crops

    def _send(self, crops: torch.Tensor) -> list:
        """Non-blocking: the detector must be free to post the recv of the previous batch's results
        while these bytes move, or both sides block in send (rendezvous) and deadlock."""
        n = torch.tensor([crops.shape[0]], dtype=torch.int64, device=self.device)
        works = [(dist.isend(n, self.peer, group=self.group), n)]
        if crops.shape[0]:
            c = crops.contiguous()
            works.append((dist.isend(c, self.peer, group=self.group), c))
        return works

    def _recv_results(self, n: int) -> torch.Tensor:
        res = torch.empty(n, 2, device=self.device)
        if n:
            dist.recv(res, self.peer, group=self.group)
        return res

    def run_batches(self, batches: Sequence[torch.Tensor]) -> List[Tuple]:
        """Detector rank: process image batches with one batch in flight. Returns per batch
        (dets, crop boxes [N,5], classifications [N,2])."""
        out = []
        if self.world == 1:
            for imgs in batches:
                dets, boxes, crops = self._detect_and_crop(imgs)
                out.append((dets, boxes, self.classify(crops)))
            return out
        # only the hand-off goes through wire_dtype (fp16 on GPUs): one conversion each side of the RCCL send
        pending = None
        inflight: list = []
        for imgs in batches:
            dets, boxes, crops = self._detect_and_crop(imgs)
            works = self._send(crops.to(self.wire_dtype))  # hand batch i to the classifier ...
            if pending is not None:                 # ... then collect batch i-1 while it works
                pd, pb = pending
                out.append((pd, pb, self._recv_results(pb.shape[0])))
            for w, _ in inflight:                   # batch i-1's sends are done by now
                w.wait()
            inflight = works
            pending = (dets, boxes)
        if pending is not None:
            pd, pb = pending
            out.append((pd, pb, self._recv_results(pb.shape[0])))
        for w, _ in inflight:
            w.wait()
        return out

    def stop(self) -> None:
        if self.world > 1 and self.is_detector:
            dist.send(torch.tensor([STOP], dtype=torch.int64, device=self.device), self.peer, group=self.group)
