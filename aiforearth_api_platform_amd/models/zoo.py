"""Servable factories of the platform's model families (``ModelSpec.factory`` / platform YAML).

The reference deploys each model as its own container behind an API route: the camera-trap
detector (``APIs/Charts/camera-trap/detection-{async,sync}``, MegaDetector on TF 1.9) and the
land-cover service (``APIManagement/create_sync_api_management_api.sh:9-92``: classify /
classifybyextent / tile / tilebyextent), chained with ``AddPipelineTask`` for ensembles
(``APIs/1.0/Common/task_management/distributed_api_task.py:67-100``). Here each factory returns a
:class:`runtime.servable.Servable` that a GPU worker process runs on fixed-shape batches:

* :func:`resnet50_classifier` — the headline classifier (fused ResNet-50 + fused top-k head);
* :func:`megadetector` — Faster-RCNN R50-FPN (K1 convs, K4 NMS, K5 RoIAlign) -> detections;
* :func:`landcover` — U-Net over a tiled mosaic (K2 GroupNorm, K3 upsample, K6 stitch) -> class map;
* :func:`camera_trap_ensemble` — detector -> crop classifier on one GPU with static shapes (the whole
  two-stage batch is one HIP graph); the two-GPU RCCL form is :mod:`runtime.pipeline`.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..runtime.servable import (ClassifierServable, DetectorServable, EnsembleServable, OutputField,
                                ResizingServable, SegmenterServable)


def resnet50_classifier(device="cuda", seed: int = 0, num_classes: int = 1000, topk: int = 5,
                        resize_from_gpu: bool = False):
    """``resize_from_gpu``: payloads of any fixed frame size (the endpoint's item_shape) are resized
    to 224x224 on the GPU inside the graph (K7) instead of by the CPU decoder."""
    from .resnet import FusedResNet, resnet50

    m = FusedResNet(resnet50(num_classes=num_classes, seed=seed), device=device)
    s = ClassifierServable(m, topk, head=m.topk_u8)
    return ResizingServable(s, (224, 224)) if resize_from_gpu else s


def megadetector(device="cuda", seed: int = 0, max_dets: Optional[int] = None, model_hw=None, **cfg):
    """``model_hw``: detector resolution when the payload slots hold native camera frames (e.g. 1536x2048):
    the frames are resized on the GPU in the graph (K7) and boxes come back in frame coordinates."""
    from .faster_rcnn import DetectorConfig, FasterRCNN

    det = FasterRCNN(DetectorConfig(**cfg), seed=seed, device=device)
    s = DetectorServable(det, max_dets)
    return ResizingServable(s, tuple(model_hw), ("boxes",)) if model_hw else s


def landcover(device="cuda", height: int = 4096, width: int = 4096, tile: int = 512, stride: int = 448,
              tile_batch: int = 16, n_classes: int = 7, seed: int = 0, unet_width: int = 64):
    from ..ops.stitch import TileGrid
    from ..runtime.spatial import SpatialSegmenter
    from .unet import FusedUNet, unet_landcover

    f = FusedUNet(unet_landcover(n_classes=n_classes, seed=seed, width=unet_width), device=device)
    seg = SpatialSegmenter(f.forward_u8, TileGrid(height, width, tile, stride), f.n_classes, torch.device(device),
                           tile_batch=tile_batch, local=True)
    return SegmenterServable(seg.run, height, width, f.n_classes)


def landcover_extent(device="cuda", mosaics=None, tile: int = 512, stride: int = 448, max_extent=(2048, 2048),
                     tile_batch: int = 16, n_classes: int = 7, seed: int = 0, unet_width: int = 64):
    """``/v2/landcover/classifybyextent`` and ``tilebyextent`` (create_sync_api_management_api.sh:52-92): the
    registered ``mosaics`` (name -> {height, width, channels, geotransform, path | seed}) stay resident in this
    worker's HBM; each task is a 64-byte extent record (runtime/extent.py) and returns the window's class map,
    identical to that window of the full-mosaic ``classify`` with the same tile grid."""
    from ..runtime.extent import ExtentSegmenter, ExtentServable, MosaicSpec
    from .unet import FusedUNet, unet_landcover

    f = FusedUNet(unet_landcover(n_classes=n_classes, seed=seed, width=unet_width), device=device)
    seg = ExtentSegmenter(f.forward_u8, MosaicSpec.parse(mosaics or {}), tile, stride, f.n_classes, device,
                          tile_batch=tile_batch)
    return ExtentServable(seg, tuple(max_extent), f.n_classes)


def select_crops_padded(dets, max_crops: int, score_thresh: float, class_id: Optional[int]):
    """Static-shape crop selection: the first ``max_crops`` confident detections of each image
    (score order) -> boxes [B, M, 4], scores [B, M], valid [B, M] (no host sync, graph-capturable)."""
    boxes, scores, labels, n = dets
    B, D = scores.shape
    M = max_crops
    rank = torch.arange(D, device=scores.device)[None].expand(B, D)
    ok = (rank < n[:, None].long()) & (scores > score_thresh)
    if class_id is not None:
        ok &= labels == class_id
    pos = torch.cumsum(ok.int(), 1) - 1
    keep = ok & (pos < M)
    dst = torch.where(keep, pos, torch.full_like(pos, M)).long()  # slot M = discard
    sel_b = torch.zeros(B, M + 1, 4, device=boxes.device)
    sel_s = torch.zeros(B, M + 1, device=boxes.device)
    sel_b.scatter_(1, dst[..., None].expand(B, D, 4), boxes.float())
    sel_s.scatter_(1, dst, scores.float())
    valid = torch.arange(M, device=boxes.device)[None] < keep.sum(1, keepdim=True)
    return sel_b[:, :M], sel_s[:, :M], valid


class StaticEnsemble:
    """Detector -> crop + resize (uint8, K5/K7) -> crop classifier, all static shapes."""

    def __init__(self, detector, classifier, max_crops: int, score_thresh: float, class_id: Optional[int],
                 crop_hw=(224, 224)):
        self.detector, self.classifier = detector, classifier
        self.max_crops, self.score_thresh, self.class_id, self.crop_hw = max_crops, score_thresh, class_id, crop_hw

    def __call__(self, images_u8: torch.Tensor):
        from ..ops.detection import crop_resize_u8

        B = images_u8.shape[0]
        M = self.max_crops
        dets = self.detector(images_u8)
        boxes, scores, valid = select_crops_padded(dets, M, self.score_thresh, self.class_id)
        img = torch.arange(B, device=boxes.device, dtype=torch.float32)[:, None, None].expand(B, M, 1)
        flat = torch.cat([img, boxes], -1).reshape(B * M, 5)
        crops = crop_resize_u8(images_u8[..., :3].contiguous(), flat, self.crop_hw)
        prob = torch.softmax(self.classifier(crops).float(), 1)
        p, c = prob.max(1)
        species = torch.where(valid, c.reshape(B, M).to(torch.int32), torch.full((B, M), -1, dtype=torch.int32,
                                                                                  device=c.device))
        sp_prob = torch.where(valid, p.reshape(B, M), torch.zeros_like(p.reshape(B, M)))
        count = valid.sum(1, keepdim=True).to(torch.int32)
        return boxes.contiguous(), (scores * valid).contiguous(), species, sp_prob, count


class _EnsembleServable(EnsembleServable):
    stages = 1  # the worker reports the detector -> classifier hop (AddPipelineTask) per batch

    def __init__(self, model: StaticEnsemble):
        super().__init__(None, model.max_crops)
        self.model = model

    def __call__(self, images_u8):
        return self.model(images_u8)


def camera_trap_ensemble(device="cuda", seed: int = 0, max_crops: int = 4, score_thresh: float = 0.5,
                         class_id: Optional[int] = 1, num_species: int = 200, **det_cfg):
    from .faster_rcnn import DetectorConfig, FasterRCNN
    from .resnet import FusedResNet, resnet50

    det = FasterRCNN(DetectorConfig(**det_cfg), seed=seed, device=device)
    cls = FusedResNet(resnet50(num_classes=num_species, seed=seed + 1), device=device)
    return _EnsembleServable(StaticEnsemble(det, cls.forward_u8, max_crops, score_thresh, class_id))


# ------------------------------------------------------------------ worker-group (multi-GPU) forms
class _Follower:
    def __init__(self, serve):
        self.serve_follower = serve


def camera_trap_ensemble_pair(device="cuda", group=None, role: str = "leader", **kw):
    """The detector -> classifier GPU pair (``ModelSpec.group_size=2``): the 1:1 stage graph."""
    return camera_trap_ensemble_group(device, group, role, group_rank=0, n_leaders=1, **kw)


class _StageGraphEnsembleServable(EnsembleServable):
    """One detector leader of an N:M stage graph (runtime/pipeline.py StageGraphPipeline): detection + crops in
    this process's HIP graph, classification on the group's classifier GPU over RCCL P2P."""

    stages = 1

    def __call__(self, images_u8):
        # no host synchronization: the answer rows come back padded to the crop capacity, valid crops first
        boxes, scores, valid, res, _ = self.pipeline.run_batches([images_u8], padded=True)[0]
        b, m = valid.shape
        flat = valid.reshape(-1)
        # valid slot s was packed at position (number of valid slots before it): its answer row
        pos = (torch.cumsum(flat.int().reshape(1, -1), 1).reshape(-1) - 1).clamp(min=0).long()
        rows = res.index_select(0, pos)
        species = torch.where(flat, rows[:, 0].to(torch.int32), torch.full_like(pos, -1, dtype=torch.int32))
        prob = torch.where(flat, rows[:, 1].float(), torch.zeros_like(rows[:, 1]))
        count = valid.sum(1, keepdim=True).to(torch.int32)
        return (boxes.float().contiguous(), (scores * valid).float().contiguous(), species.reshape(b, m),
                prob.reshape(b, m), count)

    def xgmi_bytes(self) -> dict:
        return {"sent": self.pipeline.bytes_sent, "received": self.pipeline.bytes_received}

    def close(self) -> None:
        self.pipeline.stop()


def camera_trap_ensemble_group(device="cuda", group=None, role: str = "leader", group_rank: int = 0,
                               n_leaders: int = 1, seed: int = 0, max_crops: int = 4, score_thresh: float = 0.5,
                               class_id: Optional[int] = 1, num_species: int = 200, wire_dtype: str = "uint8",
                               classifier_dtype: str = "bf16", **det_cfg):
    """Config 5 as an N:M stage graph (``ModelSpec.group_size`` = N + M, ``group_leaders`` = N): every leader is
    a detector GPU taking its own batches from the scheduler, the followers classify the crops of the detectors
    assigned to them (``runtime.pipeline.stage_assignment``), each stage in HIP graphs. ``classifier_dtype``:
    "bf16" (the fused ResNet-50 chains) or "fp16" (the per-conv K1 graph with f16 MFMA, ops/conv.py)."""
    from ..runtime.pipeline import PipelineConfig, StageGraphPipeline

    cfg = PipelineConfig(score_thresh=score_thresh, class_id=class_id, max_crops_per_image=max_crops,
                         wire_dtype=wire_dtype)
    dev = torch.device(device)
    if role == "leader":
        from .faster_rcnn import DetectorConfig, FasterRCNN

        det = FasterRCNN(DetectorConfig(**det_cfg), seed=seed, device=device)
        pipe = StageGraphPipeline(det.forward_u8, None, dev, cfg, group=group, n_leaders=n_leaders)
        return _StageGraphEnsembleServable(pipe, max_crops)
    cls = crop_classifier(device, num_species, seed + 1, classifier_dtype)
    pipe = StageGraphPipeline(None, cls, dev, cfg, group=group, n_leaders=n_leaders)
    return _Follower(pipe.serve)


def crop_classifier(device, num_species: int, seed: int, dtype: str = "bf16"):
    """uint8 crops [N, 224, 224, 3] -> logits: the fused ResNet-50 (bf16), or its per-conv K1 graph in fp16."""
    from .resnet import FusedResNet, resnet50

    m = FusedResNet(resnet50(num_classes=num_species, seed=seed), device=device,
                    dtype=torch.float16 if dtype in ("fp16", "float16") else torch.bfloat16)
    return m.forward_u8


class _SpatialSegmenterServable(SegmenterServable):
    def __init__(self, seg, height, width, n_classes):
        super().__init__(seg.run, height, width, n_classes)
        self.seg = seg

    def xgmi_bytes(self) -> dict:
        return {"sent": self.seg.bytes_sent, "received": self.seg.bytes_received}

    def close(self) -> None:
        self.seg.stop()


def landcover_spatial(device="cuda", group=None, role: str = "leader", height: int = 4096, width: int = 4096,
                      tile: int = 512, stride: int = 448, tile_batch: int = 16, n_classes: int = 7, seed: int = 0):
    """Worker group of k GPUs segmenting ONE mosaic together (tiles split evenly over the group, mosaic bands
    scattered from the leader, halo logits over RCCL P2P, class bands gathered on the leader) — BASELINE
    config #4 (spatial parallel) as an API."""
    from ..ops.stitch import TileGrid
    from ..runtime.spatial import SpatialSegmenter
    from .unet import FusedUNet, unet_landcover

    from ..parallel.dist import broadcast_tensors

    # weights are the leader's: loaded (here: seeded) once there, replicated over the group's links in one bucketed
    # broadcast per dtype (survey C1). Followers start from DIFFERENT weights, so the group's outputs equal the
    # single-GPU model only because of that broadcast (tests/test_worker_groups.py checks the equality)
    f = FusedUNet(unet_landcover(n_classes=n_classes, seed=seed if role == "leader" else seed + 7919), device=device)
    broadcast_tensors(f.tensors(), src=0, group=group)
    seg = SpatialSegmenter(f.forward_u8, TileGrid(height, width, tile, stride), f.n_classes, torch.device(device),
                           tile_batch=tile_batch, group=group, tile_graphs=True)
    if role == "leader":
        return _SpatialSegmenterServable(seg, height, width, f.n_classes)
    return _Follower(seg.serve_follower)


__all__ = ["resnet50_classifier", "camera_trap_ensemble_pair", "landcover_spatial", "megadetector", "landcover",
           "landcover_extent", "camera_trap_ensemble", "camera_trap_ensemble_group", "crop_classifier",
           "select_crops_padded",
           "StaticEnsemble", "OutputField"]
