"""MegaDetector-style Faster-RCNN R50-FPN (BASELINE config #3) on NHWC bf16 with the HIP kernels.

The reference's camera-trap detection API (``APIs/Charts/camera-trap/detection-async``, TF 1.9
MegaDetector) is re-built as a torchvision-layout Faster-RCNN: ResNet-50 backbone (BN folded, K1),
FPN (lateral 1x1 convs whose epilogue adds the nearest-upsampled top-down path, 3x3 output convs,
P6 by stride-2 max-pool), RPN (3x3 conv + one fused 1x1 objectness/box-delta conv), proposals
(top-k per level, decode, clip, NMS 0.7 via the K4 bitmask kernel — batched over images and
levels), multi-level RoIAlign (K5, level picked in-kernel), the TwoMLPHead + predictor as 1x1
convs through K1, and batched per-class NMS post-processing.

Every stage runs on fixed, padded shapes ([B, post_nms_top_n] proposals, [B, detections] outputs
+ counts), so one forward has no host synchronisation and can be captured in a HIP graph.
Weights are random-init (no checkpoint offline); classes = background + animal, person, vehicle.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from ..ops.conv import conv2d_head_nhwc, conv2d_nhwc, pack_conv
from ..ops.debug import crumb
from ..ops.detection import (det_decode, gather_keep, nms_batched_sorted, roi_align_fpn, rpn_decode_into, rpn_topk,
                              sort_select)
from ..ops.pool import maxpool2d_nhwc, preprocess_s2d_u8
from .resnet import FusedResNet, resnet50

MEGADETECTOR_CLASSES = ("background", "animal", "person", "vehicle")


@dataclass
class DetectorConfig:
    num_classes: int = 4
    fpn_channels: int = 256
    anchor_sizes: Tuple[int, ...] = (32, 64, 128, 256, 512)
    aspect_ratios: Tuple[float, ...] = (0.5, 1.0, 2.0)
    pre_nms_top_n: int = 1000
    post_nms_top_n: int = 1000
    rpn_nms_thresh: float = 0.7
    rpn_min_size: float = 1e-3
    box_score_thresh: float = 0.05
    box_nms_thresh: float = 0.5
    detections_per_img: int = 100
    box_reg_weights: Tuple[float, ...] = (10.0, 10.0, 5.0, 5.0)
    representation: int = 1024


def _rand_conv(cout, cin, k, g, std=None):
    std = std if std is not None else math.sqrt(2.0 / (cin * k * k))
    return torch.randn(cout, cin, k, k, generator=g) * std


def _nearest_up2(x: torch.Tensor, hw: Tuple[int, int]) -> torch.Tensor:
    """Nearest-neighbour upsample of NHWC x to spatial size hw (FPN top-down path)."""
    n, h, w, c = x.shape
    ih = (torch.arange(hw[0], device=x.device) * h // hw[0])
    iw = (torch.arange(hw[1], device=x.device) * w // hw[1])
    return x[:, ih][:, :, iw].contiguous()


class FasterRCNN:
    def __init__(self, cfg: Optional[DetectorConfig] = None, seed: int = 0, device="cpu",
                 backbone: Optional[nn.Module] = None):
        self.cfg = cfg = cfg or DetectorConfig()
        self.device = d = torch.device(device)
        g = torch.Generator().manual_seed(seed)
        self.backbone = FusedResNet(backbone if backbone is not None else resnet50(seed=seed), device=d)
        stage_out = (256, 512, 1024, 2048)
        C = cfg.fpn_channels
        self.lateral = [pack_conv(_rand_conv(C, ci, 1, g), torch.zeros(C)).to(d) for ci in stage_out]
        self.fpn_out = [pack_conv(_rand_conv(C, C, 3, g), torch.zeros(C), pad=1).to(d) for _ in stage_out]
        A = len(cfg.aspect_ratios)
        self.num_anchors = A
        self.rpn_conv = pack_conv(_rand_conv(C, C, 3, g, 0.01), torch.zeros(C), pad=1).to(d)
        head_out = (A + 4 * A + 3) // 4 * 4
        w = torch.zeros(head_out, C, 1, 1)
        w[: A + 4 * A] = torch.randn(A + 4 * A, C, 1, 1, generator=g) * 0.01
        self.rpn_head = pack_conv(w, torch.zeros(head_out)).to(d)
        rep = cfg.representation
        self.fc6 = pack_conv(torch.randn(rep, C * 49, 1, 1, generator=g) * math.sqrt(1.0 / (C * 49)),
                             torch.zeros(rep)).to(d)
        self.fc7 = pack_conv(torch.randn(rep, rep, 1, 1, generator=g) * math.sqrt(1.0 / rep), torch.zeros(rep)).to(d)
        nc = cfg.num_classes
        pred_out = (nc + 4 * nc + 3) // 4 * 4
        wp = torch.zeros(pred_out, rep, 1, 1)
        wp[:nc] = torch.randn(nc, rep, 1, 1, generator=g) * 0.01
        wp[nc: nc + 4 * nc] = torch.randn(4 * nc, rep, 1, 1, generator=g) * 0.001
        self.predictor = pack_conv(wp, torch.zeros(pred_out)).to(d)
        self._anchor_cache: Dict[Tuple, List[torch.Tensor]] = {}

    def sort_rows(self, img_hw: Tuple[int, int]) -> Dict[str, int]:
        """Row lengths of the two NMS-stage sorts at an input size: the all-level proposal sort (sum of the per-level
        pre-NMS top-k) and the detections' sort (post-NMS proposals x foreground classes). Both must fit the HIP row
        sort (ops.detection.ROW_SORT_MAX) for a graph-captured forward (tests/test_detector_cpu.py pins the defaults)."""
        cfg = self.cfg
        A = len(cfg.aspect_ratios)
        h, w = img_hw
        rpn = 0
        for s in (4, 8, 16, 32, 64):  # P2..P6
            rpn += min(cfg.pre_nms_top_n, -(-h // s) * -(-w // s) * A)
        return {"rpn": rpn, "detections": cfg.post_nms_top_n * (cfg.num_classes - 1)}

    # ------------------------------------------------------------------ backbone + FPN
    def backbone_stages(self, x: torch.Tensor) -> List[torch.Tensor]:
        """C2..C5 of the ResNet-50 backbone: fused stem + max-pool (K1s) and the bottleneck chains (K1c)."""
        bb = self.backbone
        return bb.stage_features(bb.stem_input(x))

    def fpn(self, feats: List[torch.Tensor]) -> List[torch.Tensor]:
        inner = conv2d_nhwc(feats[-1], self.lateral[-1])
        results = [conv2d_nhwc(inner, self.fpn_out[-1])]
        for i in range(len(feats) - 2, -1, -1):
            hw = tuple(feats[i].shape[1:3])
            if hw == (2 * inner.shape[1], 2 * inner.shape[2]):
                # lateral + nearest-2x top-down merge in one launch: the epilogue reads the coarse map directly
                inner = conv2d_nhwc(feats[i], self.lateral[i], residual=inner, residual_up2=True)
            else:
                inner = conv2d_nhwc(feats[i], self.lateral[i], residual=_nearest_up2(inner, hw))
            results.insert(0, conv2d_nhwc(inner, self.fpn_out[i]))
        results.append(maxpool2d_nhwc(results[-1], 1, 2, 0))  # P6
        return results

    # ------------------------------------------------------------------ anchors
    def anchors(self, shapes: Sequence[Tuple[int, int]], strides: Sequence[int]) -> List[torch.Tensor]:
        key = (tuple(shapes), tuple(strides))
        if key not in self._anchor_cache:
            out = []
            for (h, w), s, size in zip(shapes, strides, self.cfg.anchor_sizes):
                r = torch.tensor(self.cfg.aspect_ratios)
                hr = torch.sqrt(r)
                wr = 1 / hr
                ws, hs = wr * size, hr * size
                base = torch.round(torch.stack([-ws, -hs, ws, hs], 1) / 2)
                sy, sx = torch.meshgrid(torch.arange(h) * s, torch.arange(w) * s, indexing="ij")
                shifts = torch.stack([sx, sy, sx, sy], -1).reshape(-1, 1, 4).float()
                out.append((shifts + base[None]).reshape(-1, 4).to(self.device))
            self._anchor_cache[key] = out
        return self._anchor_cache[key]

    # ------------------------------------------------------------------ RPN + proposals
    def proposals(self, P: List[torch.Tensor], img_hw: Tuple[int, int]
                  ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        cfg = self.cfg
        A = self.num_anchors
        B = P[0].shape[0]
        shapes = [p.shape[1:3] for p in P]
        strides = [img_hw[0] // s[0] for s in shapes]
        anchors = self.anchors(shapes, strides)
        ks = [min(cfg.pre_nms_top_n, p.shape[1] * p.shape[2] * A) for p in P]
        KT = sum(ks)
        boxes = torch.empty(B, KT, 4, device=P[0].device, dtype=torch.float32)
        scores = torch.empty(B, KT, device=P[0].device, dtype=torch.float32)
        lvl = torch.empty(B, KT, device=P[0].device, dtype=torch.float32)
        off = 0
        for li, (p, k) in enumerate(zip(P, ks)):
            # [B, h, w, 16]: A logits, 4A deltas; on the 256-wide tiles the head runs in the RPN conv's epilogue
            head = conv2d_head_nhwc(p, self.rpn_conv, self.rpn_head)
            idx = rpn_topk(head, A, k)                            # per-level pre-NMS top-k
            # decode + clip + sigmoid + min-size mask straight into the all-level buffers (one HIP launch)
            crumb(f"rpn.topk{li}", idx)
            rpn_decode_into(head, idx, anchors[li], A, boxes, scores, lvl, off, li, img_hw, cfg.rpn_min_size)
            off += k
        # batched NMS across levels via coordinate offsets; invalid (small) boxes sort last. Sort, gathers, level
        # offsets and the valid count in one launch (sort_select), the kept rows in another (gather_keep)
        _, boxes_s, boxes_off, _, valid = sort_select(scores, boxes, max(img_hw) + 1.0, groups=lvl)
        keep, count = nms_batched_sorted(boxes_off, cfg.rpn_nms_thresh, cfg.post_nms_top_n, valid)
        crumb("rpn.nms", keep)
        # the proposals [B, R, 4] and the same boxes as RoIAlign rows [B * R, 5] (image, box), one launch
        props, _, _, rois = gather_keep(keep, boxes=boxes_s, rois=True)
        return props, count, rois

    # ------------------------------------------------------------------ box head + postprocess
    def box_head(self, P: List[torch.Tensor], props: torch.Tensor, img_hw, rois: Optional[torch.Tensor] = None):
        """``rois``: the proposals as RoIAlign rows [B * R, 5] (from ``proposals``), else formed here."""
        B, R, _ = props.shape
        if rois is None:
            bidx = torch.arange(B, device=props.device, dtype=torch.float32)[:, None, None].expand(B, R, 1)
            rois = torch.cat([bidx, props], -1).reshape(B * R, 5)
        strides = [img_hw[0] // p.shape[1] for p in P[:4]]
        feats = roi_align_fpn(P[:4], [1.0 / s for s in strides], rois, (7, 7), 2)  # [B*R, 7, 7, C]
        crumb("box.roi_align", feats)
        x = feats.reshape(B * R, 1, 1, -1)
        # box-head FCs on K1 (the 256x256 tile, tuned per batch in conv_tiles.json)
        x = conv2d_nhwc(x, self.fc6, relu=True)
        x = conv2d_nhwc(x, self.fc7, relu=True)
        # [B, R, >= 5 nc]: nc class logits, then 4 nc box deltas
        return conv2d_nhwc(x, self.predictor).reshape(B, R, -1)

    def postprocess(self, props, count, pred, img_hw):
        cfg = self.cfg
        # softmax (background dropped) + per-class decode + clip + validity mask: one HIP launch
        boxes, scores, _ = det_decode(pred, props, count, cfg.num_classes, cfg.box_reg_weights, img_hw,
                                      cfg.box_score_thresh)
        # class label of entry j of the [R, nc - 1] layout = j % (nc - 1) + 1: per-class NMS by label offsets
        s_s, b_s, b_off, l_s, valid = sort_select(scores, boxes, max(img_hw) + 1.0, group_mod=cfg.num_classes - 1,
                                                  want_labels=True)
        keep, ndet = nms_batched_sorted(b_off, cfg.box_nms_thresh, cfg.detections_per_img, valid)
        crumb("post.nms", keep)
        det_boxes, det_scores, det_labels = gather_keep(keep, boxes=b_s, scores=s_s, labels=l_s)
        return det_boxes, det_scores, det_labels, ndet

    # ------------------------------------------------------------------ forward
    def forward(self, x: torch.Tensor):
        """x normalized NHWC [B, H, W, 8] (H, W multiples of 64). Returns padded detections:
        boxes [B, D, 4], scores [B, D], labels [B, D], counts [B]."""
        img_hw = (x.shape[1], x.shape[2]) if x.shape[-1] != 16 else (2 * x.shape[1], 2 * x.shape[2])
        feats = self.backbone_stages(x)
        crumb("backbone", feats[-1])
        P = self.fpn(feats)
        crumb("fpn", P[-1])
        props, count, rois = self.proposals(P, img_hw)
        pred = self.box_head(P, props, img_hw, rois)
        crumb("box.head", pred)
        return self.postprocess(props, count, pred, img_hw)

    def forward_u8(self, img_u8: torch.Tensor):
        return self.forward(preprocess_s2d_u8(img_u8))

    __call__ = forward_u8

    @staticmethod
    def to_list(dets) -> List[Dict[str, list]]:
        boxes, scores, labels, n = [t.cpu() for t in dets]
        return [{"boxes": boxes[i, : n[i]].tolist(), "scores": scores[i, : n[i]].tolist(),
                 "labels": [MEGADETECTOR_CLASSES[int(c)] for c in labels[i, : n[i]]]} for i in range(len(n))]
