"""Detection ops: NMS [K4], RoIAlign / multi-scale RoIAlign [K5], crop-and-resize, box coding.

GPU tensors run the HIP kernels of ``csrc/kernels/detection.hip``; CPU tensors run the PyTorch
reference implementations below (torchvision is not available in this image, so these references
are written out here and the GPU tests compare the kernels against them).
"""
from __future__ import annotations

import ctypes
import math
from typing import Optional, Sequence, Tuple

import torch

from . import _ext
from .pool import IMAGENET_MEAN, IMAGENET_STD


# ---------------------------------------------------------------------------------------------- boxes
def box_iou(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    area_a = (a[:, 2] - a[:, 0]).clamp(min=0) * (a[:, 3] - a[:, 1]).clamp(min=0)
    area_b = (b[:, 2] - b[:, 0]).clamp(min=0) * (b[:, 3] - b[:, 1]).clamp(min=0)
    lt = torch.max(a[:, None, :2], b[None, :, :2])
    rb = torch.min(a[:, None, 2:], b[None, :, 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    union = area_a[:, None] + area_b[None, :] - inter
    return torch.where(union > 0, inter / union, torch.zeros_like(inter))


def decode_boxes(anchors: torch.Tensor, deltas: torch.Tensor, weights=(1.0, 1.0, 1.0, 1.0),
                 clip: float = math.log(1000.0 / 16)) -> torch.Tensor:
    """Faster-RCNN box decoding (anchors [..., 4] xyxy, deltas [..., 4] dx,dy,dw,dh)."""
    wx, wy, ww, wh = weights
    w = anchors[..., 2] - anchors[..., 0]
    h = anchors[..., 3] - anchors[..., 1]
    cx = anchors[..., 0] + 0.5 * w
    cy = anchors[..., 1] + 0.5 * h
    dx, dy = deltas[..., 0] / wx, deltas[..., 1] / wy
    dw, dh = (deltas[..., 2] / ww).clamp(max=clip), (deltas[..., 3] / wh).clamp(max=clip)
    pcx, pcy = dx * w + cx, dy * h + cy
    pw, ph = torch.exp(dw) * w, torch.exp(dh) * h
    return torch.stack([pcx - 0.5 * pw, pcy - 0.5 * ph, pcx + 0.5 * pw, pcy + 0.5 * ph], dim=-1)


def clip_boxes(boxes: torch.Tensor, h: int, w: int) -> torch.Tensor:
    return torch.stack([boxes[..., 0].clamp(0, w), boxes[..., 1].clamp(0, h), boxes[..., 2].clamp(0, w),
                        boxes[..., 3].clamp(0, h)], dim=-1)


def rpn_decode_into(head: torch.Tensor, idx: torch.Tensor, anchors: torch.Tensor, num_anchors: int,
                    boxes: torch.Tensor, scores: torch.Tensor, lvl: torch.Tensor, off: int, level: int,
                    img_hw: Tuple[int, int], min_size: float, clip: float = math.log(1000.0 / 16)) -> None:
    """One FPN level's RPN proposals into columns [off, off + k) of the all-level buffers: deltas and anchors
    gathered by the top-k flat indices ``idx`` [B, k] (pos * A + a), decoded, clipped to the image; score =
    sigmoid(objectness), -1 for boxes narrower or shorter than ``min_size``; lvl = level.
    ``head`` [B, h, w, >= 5A] holds A objectness logits then 4A deltas per pixel."""
    B, k = idx.shape
    A = num_anchors
    hw = head.shape[1] * head.shape[2]
    if _ext.backend_for(head) == "hip" and head.dtype == torch.bfloat16 and head.is_contiguous():
        _ext.call("ai4e_rpn_decode", head.data_ptr(), idx.contiguous().data_ptr(), anchors.data_ptr(), boxes.data_ptr(),
                  scores.data_ptr(), lvl.data_ptr(), B, hw, head.shape[-1], A, k, boxes.shape[1], off, float(level),
                  float(img_hw[0]), float(img_hw[1]), float(min_size), float(clip), _ext.stream_ptr(head.device))
        return
    hf = head.float().reshape(B, hw, -1)
    obj = hf[..., :A].reshape(B, -1)
    deltas = hf[..., A: 5 * A].reshape(B, -1, 4)
    d = torch.gather(deltas, 1, idx[..., None].expand(B, k, 4))
    bx = clip_boxes(decode_boxes(anchors[idx], d, clip=clip), img_hw[0], img_hw[1])
    sc = torch.sigmoid(torch.gather(obj, 1, idx))
    wh = bx[..., 2:] - bx[..., :2]
    boxes[:, off:off + k] = bx
    scores[:, off:off + k] = sc.masked_fill((wh < min_size).any(-1), -1.0)
    lvl[:, off:off + k] = float(level)


ROW_SORT_MAX = 8192  # longest row the HIP sorts take (one workgroup's LDS bitonic network, csrc detection.hip)


def _graph_safe_fallback(what: str, t: torch.Tensor) -> None:
    """A library fallback (multi-kernel sort with temporaries) must never be captured into a HIP graph: replaying it
    after other allocations came and went faulted the GPU (profiles/r4_replay/). Refuse loudly instead."""
    if t.is_cuda and torch.cuda.is_current_stream_capturing():
        raise RuntimeError(f"{what}: shape {tuple(t.shape)} exceeds the HIP kernel's limit (rows <= {ROW_SORT_MAX}); "
                           "its library fallback is not graph-safe — run this configuration without HIP graphs")


def argsort_desc_rows(scores: torch.Tensor) -> torch.Tensor:
    """``scores.argsort(1, descending=True)`` for fp32 [B, N] rows; HIP (N <= 8192): one workgroup per row, a bitonic
    network in LDS, ties in index order (deterministic), no library temporaries (graph-safe, profiles/r4_replay/)."""
    B, N = scores.shape
    if _ext.backend_for(scores) == "hip" and scores.dtype == torch.float32 and N <= ROW_SORT_MAX:
        s = scores.contiguous()
        order = torch.empty(B, N, dtype=torch.long, device=scores.device)
        _ext.call("ai4e_row_sort_desc", s.data_ptr(), B, N, order.data_ptr(), _ext.stream_ptr(scores.device))
        return order
    _graph_safe_fallback("argsort_desc_rows", scores)
    return scores.argsort(dim=1, descending=True, stable=True)


def sort_select(scores: torch.Tensor, boxes: torch.Tensor, scale: float, groups: Optional[torch.Tensor] = None,
                group_mod: int = 0, want_labels: bool = False):
    """One NMS stage's sort + select: rows of fp32 ``scores`` [B, N] sorted descending (ties: lower index first) with
    their ``boxes`` [B, N, 4]; each box also offset by ``group * scale`` (batched NMS of several groups at once by
    coordinate offsets), the group being ``groups`` [B, N] (fp32, e.g. the FPN level) or, without it, the index's
    ``index % group_mod + 1`` (the class label of det_decode's [R, nc - 1] layout).

    Returns (scores_s [B, N], boxes_s [B, N, 4], boxes_off [B, N, 4], groups_s [B, N] fp32 or labels [B, N] int64 with
    ``want_labels``, valid [B] int32 = entries with score >= 0). HIP (N <= 8192): one launch (sort_select_kernel)."""
    B, N = scores.shape
    dev = scores.device
    if _ext.backend_for(scores) == "hip" and N <= ROW_SORT_MAX:
        sc = scores.float().contiguous()
        bx = boxes.float().contiguous()
        g = None if groups is None else groups.float().contiguous()
        s_s = torch.empty(B, N, dtype=torch.float32, device=dev)
        b_s = torch.empty(B, N, 4, dtype=torch.float32, device=dev)
        b_o = torch.empty(B, N, 4, dtype=torch.float32, device=dev)
        g_s = None if want_labels else torch.empty(B, N, dtype=torch.float32, device=dev)
        lab = torch.empty(B, N, dtype=torch.int64, device=dev) if want_labels else None
        valid = torch.empty(B, dtype=torch.int32, device=dev)
        _ext.call("ai4e_sort_select", sc.data_ptr(), bx.data_ptr(), _ext.ptr(g), int(group_mod), float(scale), B, N,
                  s_s.data_ptr(), b_s.data_ptr(), b_o.data_ptr(), _ext.ptr(g_s), _ext.ptr(lab), valid.data_ptr(),
                  _ext.stream_ptr(dev))
        return s_s, b_s, b_o, (lab if want_labels else g_s), valid
    _graph_safe_fallback("sort_select", scores)
    order = scores.float().argsort(dim=1, descending=True, stable=True)
    s_s = torch.gather(scores.float(), 1, order)
    b_s = torch.gather(boxes.float(), 1, order[..., None].expand(B, N, 4))
    if groups is not None:
        g_s = torch.gather(groups.float(), 1, order)
    else:
        g_s = (order % int(group_mod) + 1).float()
    b_o = b_s + (g_s * float(scale))[..., None]
    valid = (s_s >= 0).sum(1).to(torch.int32)
    return s_s, b_s, b_o, (g_s.long() if want_labels else g_s), valid


def gather_keep(keep: torch.Tensor, boxes: Optional[torch.Tensor] = None, scores: Optional[torch.Tensor] = None,
                labels: Optional[torch.Tensor] = None, rois: bool = False):
    """Rows kept by NMS (``keep`` [B, K] int32, -1 = padding): (boxes [B, K, 4], scores [B, K], labels [B, K]) gathered
    from [B, N, ...] sources (None where the source is None), zero at padding. HIP: one launch (gather_keep_kernel).
    ``rois``: a fourth result, the boxes as RoIAlign rows [B * K, 5] = (image, x1, y1, x2, y2), from the same launch."""
    B, K = keep.shape
    src = next(t for t in (boxes, scores, labels) if t is not None)
    N = src.shape[1]
    dev = keep.device
    if _ext.backend_for(keep) == "hip":
        kp = keep.to(torch.int32).contiguous()
        bs = None if boxes is None else boxes.float().contiguous()
        ss = None if scores is None else scores.float().contiguous()
        ls = None if labels is None else labels.long().contiguous()
        bo = None if bs is None else torch.empty(B, K, 4, dtype=torch.float32, device=dev)
        so = None if ss is None else torch.empty(B, K, dtype=torch.float32, device=dev)
        lo = None if ls is None else torch.empty(B, K, dtype=torch.int64, device=dev)
        ro = torch.empty(B * K, 5, dtype=torch.float32, device=dev) if rois else None
        if rois and bs is None:
            raise ValueError("gather_keep(rois=True) needs boxes")
        _ext.call("ai4e_gather_keep", kp.data_ptr(), B, K, N, _ext.ptr(bs), _ext.ptr(ss), _ext.ptr(ls), _ext.ptr(bo),
                  _ext.ptr(so), _ext.ptr(lo), _ext.ptr(ro), _ext.stream_ptr(dev))
        return (bo, so, lo, ro) if rois else (bo, so, lo)
    k = keep.clamp(min=0).long()
    pad = keep < 0
    bo = None if boxes is None else torch.gather(boxes.float(), 1, k[..., None].expand(B, K, 4)).masked_fill(
        pad[..., None], 0.0)
    so = None if scores is None else torch.gather(scores.float(), 1, k).masked_fill(pad, 0.0)
    lo = None if labels is None else torch.gather(labels.long(), 1, k).masked_fill(pad, 0)
    if rois:
        bidx = torch.arange(B, device=dev, dtype=torch.float32)[:, None, None].expand(B, K, 1)
        return bo, so, lo, torch.cat([bidx, bo], -1).reshape(B * K, 5)
    return bo, so, lo


def rpn_topk(head: torch.Tensor, num_anchors: int, k: int) -> torch.Tensor:
    """Flat indices ``pos * A + a`` [B, k] (int64) of the k largest objectness logits of one FPN level, read straight
    from the RPN head bf16 [B, h, w, >= A] (channels 0..A-1). HIP: one workgroup per image, radix select, a fixed
    deterministic output order (the proposals are re-sorted by score across levels afterwards) and graph-safe (no
    library temporaries: torch.topk's multi-block path faulted replaying in a graph, profiles/r4_replay/). Ties of
    the k-th value are taken lowest index first on every backend (elsewhere: a stable descending sort's first k)."""
    B = head.shape[0]
    hw = head.shape[1] * head.shape[2]
    if k > hw * num_anchors:
        raise ValueError(f"rpn_topk: k={k} > {hw * num_anchors} candidates")
    if _ext.backend_for(head) == "hip" and head.dtype == torch.bfloat16 and head.is_contiguous():
        idx = torch.empty(B, k, dtype=torch.long, device=head.device)
        _ext.call("ai4e_rpn_topk", head.data_ptr(), B, hw, head.shape[-1], num_anchors, k, idx.data_ptr(),
                  _ext.stream_ptr(head.device))
        return idx
    # the k largest by (value desc, index asc): the same SET as the HIP kernel's (ties by lowest flat index)
    return head[..., :num_anchors].reshape(B, -1).float().argsort(dim=1, descending=True, stable=True)[:, :k]


def det_decode(pred: torch.Tensor, props: torch.Tensor, count: torch.Tensor, num_classes: int,
               weights: Sequence[float], img_hw: Tuple[int, int], score_thresh: float,
               clip: float = math.log(1000.0 / 16)) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Box-head postprocess before the final NMS: softmax over the nc logits of each RoI, every foreground
    class's box decoded from the RoI's proposal (regression ``weights``) and clipped; score -1 unless the RoI
    is real (r < count[b]), the score clears ``score_thresh`` and the box is >= 1e-2 wide and high.
    pred [B, R, >= 5 nc] (logits, then 4 nc deltas), props [B, R, 4], count [B] ->
    boxes [B, R * (nc-1), 4], scores [B, R * (nc-1)], labels [B, R * (nc-1)] (int64, 1..nc-1)."""
    B, R, ldp = pred.shape
    nc = num_classes
    if _ext.backend_for(pred) == "hip":
        bf16 = pred.dtype == torch.bfloat16  # (read as bf16 in the kernel: no conversion launch)
        pred = pred.contiguous() if bf16 else pred.float().contiguous()
        boxes = torch.empty(B, R * (nc - 1), 4, device=pred.device, dtype=torch.float32)
        scores = torch.empty(B, R * (nc - 1), device=pred.device, dtype=torch.float32)
        labels = torch.empty(B, R * (nc - 1), device=pred.device, dtype=torch.int64)
        w4 = (ctypes.c_float * 4)(*[float(v) for v in weights])
        _ext.call("ai4e_det_decode", pred.data_ptr(), props.float().contiguous().data_ptr(),
                  count.to(torch.int32).contiguous().data_ptr(), boxes.data_ptr(), scores.data_ptr(), labels.data_ptr(),
                  B, R, ldp, nc, ctypes.addressof(w4), float(img_hw[0]), float(img_hw[1]), float(score_thresh),
                  float(clip), int(bf16), _ext.stream_ptr(pred.device))
        return boxes, scores, labels
    pred = pred.float()
    logits, deltas = pred[..., :nc], pred[..., nc: 5 * nc].reshape(B, R, nc, 4)
    scores = torch.softmax(logits, -1)[..., 1:]
    boxes = decode_boxes(props[:, :, None, :].expand(B, R, nc - 1, 4), deltas[:, :, 1:], weights, clip)
    boxes = clip_boxes(boxes, img_hw[0], img_hw[1])
    labels = torch.arange(1, nc, device=props.device).expand(B, R, nc - 1)
    roi_valid = (torch.arange(R, device=props.device)[None] < count[:, None].long())[..., None]
    wh = boxes[..., 2:] - boxes[..., :2]
    ok = roi_valid & (scores > score_thresh) & (wh >= 1e-2).all(-1)
    scores = scores.masked_fill(~ok, -1.0).reshape(B, -1)
    return boxes.reshape(B, -1, 4), scores, labels.reshape(B, -1)


# ---------------------------------------------------------------------------------------------- NMS
def nms_reference(boxes: torch.Tensor, scores: torch.Tensor, thr: float) -> torch.Tensor:
    """Greedy NMS (torchvision.ops.nms semantics): indices kept, in descending score order."""
    order = torch.argsort(scores, descending=True, stable=True)
    b = boxes[order]
    keep = []
    suppressed = torch.zeros(len(order), dtype=torch.bool)
    iou = box_iou(b, b)
    for i in range(len(order)):
        if suppressed[i]:
            continue
        keep.append(i)
        suppressed |= iou[i] > thr
        suppressed[i] = True
    return order[torch.tensor(keep, dtype=torch.long)] if keep else torch.zeros(0, dtype=torch.long)


def nms_batched_sorted(boxes: torch.Tensor, thr: float, max_out: int, valid: Optional[torch.Tensor] = None
                       ) -> Tuple[torch.Tensor, torch.Tensor]:
    """NMS over B images at once. boxes [B, N, 4] already sorted by descending score per image.

    Returns (keep [B, max_out] int32 indices into N (padded -1), count [B] int32).
    """
    B, N, _ = boxes.shape
    if _ext.backend_for(boxes) == "hip":
        boxes = boxes.float().contiguous()
        words = (N + 63) // 64
        mask = torch.empty(B, N, words, dtype=torch.int64, device=boxes.device)
        keep = torch.empty(B, max_out, dtype=torch.int32, device=boxes.device)  # (the reduce pads with -1)
        count = torch.empty(B, dtype=torch.int32, device=boxes.device)
        vptr = None if valid is None else valid.to(torch.int32).contiguous()
        st = _ext.stream_ptr(boxes.device)
        _ext.call("ai4e_nms_mask", boxes.data_ptr(), B, N, float(thr), mask.data_ptr(), st)
        _ext.call("ai4e_nms_reduce", mask.data_ptr(), _ext.ptr(vptr), B, N, max_out, keep.data_ptr(), count.data_ptr(),
                  st)
        return keep, count
    keep = torch.full((B, max_out), -1, dtype=torch.int32)
    count = torch.zeros(B, dtype=torch.int32)
    for b in range(B):
        n = N if valid is None else int(valid[b])
        scores = torch.arange(n, 0, -1, dtype=torch.float32)  # already sorted
        k = nms_reference(boxes[b, :n].float().cpu(), scores, thr)[:max_out]
        keep[b, :len(k)] = k.to(torch.int32)
        count[b] = len(k)
    return keep.to(boxes.device), count.to(boxes.device)


def batched_nms(boxes: torch.Tensor, scores: torch.Tensor, idxs: torch.Tensor, thr: float,
                max_out: int = 1000) -> torch.Tensor:
    """Per-class NMS for one image (coordinate-offset trick); returns kept indices (desc score)."""
    if boxes.numel() == 0:
        return torch.zeros(0, dtype=torch.long, device=boxes.device)
    off = idxs.to(boxes.dtype) * (boxes.max() + 1)
    b = boxes + off[:, None]
    order = torch.argsort(scores, descending=True)
    keep, count = nms_batched_sorted(b[order][None], thr, max_out)
    k = keep[0, :int(count[0])].long()
    return order[k]


# ---------------------------------------------------------------------------------------------- RoIAlign
def roi_align_reference(feat: torch.Tensor, rois: torch.Tensor, out_hw: Tuple[int, int], scale: float,
                        sampling: int = 2, aligned: bool = False) -> torch.Tensor:
    """torchvision.ops.roi_align on NHWC features (fp32 math). rois [R, 5] = (img, x1, y1, x2, y2)."""
    n, H, W, C = feat.shape
    PH, PW = out_hw
    f = feat.float()
    out = torch.zeros(rois.shape[0], PH, PW, C)
    off = 0.5 if aligned else 0.0
    for r in range(rois.shape[0]):
        img = int(rois[r, 0])
        x1, y1 = float(rois[r, 1]) * scale - off, float(rois[r, 2]) * scale - off
        rw, rh = float(rois[r, 3]) * scale - off - x1, float(rois[r, 4]) * scale - off - y1
        if not aligned:
            rw, rh = max(rw, 1.0), max(rh, 1.0)
        bh, bw = rh / PH, rw / PW
        gh = sampling if sampling > 0 else int(math.ceil(rh / PH))
        gw = sampling if sampling > 0 else int(math.ceil(rw / PW))
        cnt = max(gh * gw, 1)
        ys = torch.tensor([y1 + ph * bh + (iy + 0.5) * bh / gh for ph in range(PH) for iy in range(gh)])
        xs = torch.tensor([x1 + pw * bw + (ix + 0.5) * bw / gw for pw in range(PW) for ix in range(gw)])
        yy, xx = torch.meshgrid(ys, xs, indexing="ij")
        v = _bilinear(f[img], yy, xx)  # [PH*gh, PW*gw, C]
        out[r] = v.reshape(PH, gh, PW, gw, C).sum(dim=(1, 3)) / cnt
    return out


def _bilinear(f: torch.Tensor, y: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    H, W, C = f.shape
    valid = (y >= -1) & (y <= H) & (x >= -1) & (x <= W)
    y = y.clamp(min=0)
    x = x.clamp(min=0)
    y0 = y.floor().long()
    x0 = x.floor().long()
    ytop = y0 >= H - 1
    xtop = x0 >= W - 1
    y0 = torch.where(ytop, torch.full_like(y0, H - 1), y0)
    x0 = torch.where(xtop, torch.full_like(x0, W - 1), x0)
    y = torch.where(ytop, y0.float(), y)
    x = torch.where(xtop, x0.float(), x)
    y1 = torch.where(ytop, y0, y0 + 1).clamp(max=H - 1)
    x1 = torch.where(xtop, x0, x0 + 1).clamp(max=W - 1)
    ly, lx = (y - y0)[..., None], (x - x0)[..., None]
    v = (1 - ly) * (1 - lx) * f[y0, x0] + (1 - ly) * lx * f[y0, x1] + ly * (1 - lx) * f[y1, x0] + ly * lx * f[y1, x1]
    return v * valid[..., None]


def roi_align_nhwc(feat: torch.Tensor, rois: torch.Tensor, out_hw: Tuple[int, int], scale: float,
                   sampling: int = 2, aligned: bool = False) -> torch.Tensor:
    n, H, W, C = feat.shape
    R = rois.shape[0]
    if _ext.backend_for(feat) == "hip":
        feat = feat.contiguous()
        rois = rois.float().contiguous()
        out = torch.empty(R, out_hw[0], out_hw[1], C, device=feat.device, dtype=feat.dtype)
        _ext.call("ai4e_roi_align_nhwc", feat.data_ptr(), rois.data_ptr(), out.data_ptr(), H, W, C, R, out_hw[0],
                  out_hw[1], sampling, float(scale), int(aligned), 0, _ext.stream_ptr(feat.device))
        return out
    return roi_align_reference(feat, rois.cpu(), out_hw, scale, sampling, aligned).to(feat.dtype)


def map_levels(rois: torch.Tensor, k_min: int = 2, k_max: int = 5, canonical_scale: float = 224.0,
               canonical_level: int = 4) -> torch.Tensor:
    """FPN level assignment (Lin et al. eq. 1)."""
    area = (rois[:, 3] - rois[:, 1]).clamp(min=0) * (rois[:, 4] - rois[:, 2]).clamp(min=0)
    lvl = torch.floor(canonical_level + torch.log2(torch.sqrt(area) / canonical_scale + 1e-6))
    return lvl.clamp(k_min, k_max).long() - k_min


def multiscale_roi_align(feats: Sequence[torch.Tensor], scales: Sequence[float], rois: torch.Tensor,
                         out_hw=(7, 7), sampling: int = 2) -> torch.Tensor:
    levels = map_levels(rois, 2, 2 + len(feats) - 1)
    C = feats[0].shape[-1]
    out = torch.zeros(rois.shape[0], out_hw[0], out_hw[1], C, device=feats[0].device, dtype=feats[0].dtype)
    for lv, (f, s) in enumerate(zip(feats, scales)):
        idx = torch.nonzero(levels == lv).flatten()
        if idx.numel():
            out[idx] = roi_align_nhwc(f, rois[idx], out_hw, s, sampling)
    return out


def roi_align_fpn(feats: Sequence[torch.Tensor], scales: Sequence[float], rois: torch.Tensor, out_hw=(7, 7),
                  sampling: int = 2, aligned: bool = False) -> torch.Tensor:
    """Multi-level RoIAlign over P2..P5 with in-kernel level assignment (static shapes, graph-safe)."""
    if len(feats) != 4:
        raise ValueError("roi_align_fpn expects 4 levels (P2..P5)")
    if _ext.backend_for(feats[0]) == "hip":
        feats = [f.contiguous() for f in feats]
        C = feats[0].shape[-1]
        R = rois.shape[0]
        hw = (ctypes.c_int * 8)(*[v for f in feats for v in (f.shape[1], f.shape[2])])
        sc = (ctypes.c_float * 4)(*[float(s) for s in scales])
        rois = rois.float().contiguous()
        out = torch.empty(R, out_hw[0], out_hw[1], C, device=feats[0].device, dtype=feats[0].dtype)
        _ext.call("ai4e_roi_align_fpn_nhwc", *[f.data_ptr() for f in feats], ctypes.addressof(hw), ctypes.addressof(sc),
                  rois.data_ptr(), out.data_ptr(), C, R, out_hw[0], out_hw[1], sampling, int(aligned),
                  _ext.stream_ptr(feats[0].device))
        return out
    return multiscale_roi_align(feats, scales, rois, out_hw, sampling)


# ---------------------------------------------------------------------------------------------- crops
def crop_resize_reference(img_u8: torch.Tensor, boxes: torch.Tensor, out_hw: Tuple[int, int],
                          mean=IMAGENET_MEAN, std=IMAGENET_STD) -> torch.Tensor:
    n, H, W, C = img_u8.shape
    OH, OW = out_hw
    m8 = torch.tensor(list(mean) + [0.0] * (8 - len(mean)))
    s8 = torch.tensor(list(std) + [1.0] * (8 - len(std)))
    out = torch.zeros(boxes.shape[0], OH, OW, 8)
    for r in range(boxes.shape[0]):
        b = boxes[r].float()
        i = int(b[0])
        sx = (b[1] + (torch.arange(OW) + 0.5) * (b[3] - b[1]) / OW - 0.5).clamp(0, W - 1)
        sy = (b[2] + (torch.arange(OH) + 0.5) * (b[4] - b[2]) / OH - 0.5).clamp(0, H - 1)
        yy, xx = torch.meshgrid(sy, sx, indexing="ij")
        y0, x0 = yy.floor().long(), xx.floor().long()
        y1, x1 = (y0 + 1).clamp(max=H - 1), (x0 + 1).clamp(max=W - 1)
        ly, lx = (yy - y0)[..., None], (xx - x0)[..., None]
        f = img_u8[i].float()
        pix = (1 - ly) * ((1 - lx) * f[y0, x0] + lx * f[y0, x1]) + ly * ((1 - lx) * f[y1, x0] + lx * f[y1, x1])
        out[r, ..., :C] = (pix / 255.0 - m8[:C]) / s8[:C]
    return out


_NORM_CACHE = {}


def crop_resize_nhwc(img_u8: torch.Tensor, boxes: torch.Tensor, out_hw=(224, 224), mean=IMAGENET_MEAN,
                     std=IMAGENET_STD) -> torch.Tensor:
    """Crop boxes [R,5]=(img,x1,y1,x2,y2) from uint8 NHWC images, resize bilinear, normalize ->
    bf16 [R, OH, OW, 8] (ready for a classifier stem)."""
    n, H, W, C = img_u8.shape
    R = boxes.shape[0]
    if _ext.backend_for(img_u8) == "hip":
        key = (img_u8.device, tuple(mean), tuple(std))
        norm = _NORM_CACHE.get(key)
        if norm is None:
            norm = torch.tensor(list(mean) + [0.0] * (8 - len(mean)) + list(std) + [1.0] * (8 - len(std)),
                                dtype=torch.float32, device=img_u8.device)
            _NORM_CACHE[key] = norm
        out = torch.empty(R, out_hw[0], out_hw[1], 8, device=img_u8.device, dtype=torch.bfloat16)
        _ext.call("ai4e_crop_resize_nhwc", img_u8.contiguous().data_ptr(), boxes.float().contiguous().data_ptr(),
                  out.data_ptr(), norm.data_ptr(), H, W, C, R, out_hw[0], out_hw[1], 0, _ext.stream_ptr(img_u8.device))
        return out
    return crop_resize_reference(img_u8.cpu(), boxes.cpu(), out_hw, mean, std)


def crop_resize_u8_reference(img_u8: torch.Tensor, boxes: torch.Tensor, out_hw: Tuple[int, int]) -> torch.Tensor:
    """fp32 reference of :func:`crop_resize_u8` (same sampling grid as the normalized variant)."""
    n, H, W, C = img_u8.shape
    OH, OW = out_hw
    out = torch.zeros(boxes.shape[0], OH, OW, C, dtype=torch.uint8)
    for r in range(boxes.shape[0]):
        b = boxes[r].float().cpu()
        i = int(b[0])
        sx = (b[1] + (torch.arange(OW) + 0.5) * (b[3] - b[1]) / OW - 0.5).clamp(0, W - 1)
        sy = (b[2] + (torch.arange(OH) + 0.5) * (b[4] - b[2]) / OH - 0.5).clamp(0, H - 1)
        yy, xx = torch.meshgrid(sy, sx, indexing="ij")
        y0, x0 = yy.floor().long(), xx.floor().long()
        y1, x1 = (y0 + 1).clamp(max=H - 1), (x0 + 1).clamp(max=W - 1)
        ly, lx = (yy - y0)[..., None], (xx - x0)[..., None]
        f = img_u8[i].float().cpu()
        pix = (1 - ly) * ((1 - lx) * f[y0, x0] + lx * f[y0, x1]) + ly * ((1 - lx) * f[y1, x0] + lx * f[y1, x1])
        out[r] = (pix + 0.5).clamp(0, 255).to(torch.uint8)
    return out


def crop_resize_u8(img_u8: torch.Tensor, boxes: torch.Tensor, out_hw=(224, 224)) -> torch.Tensor:
    """Crop boxes [R,5]=(img,x1,y1,x2,y2) from uint8 NHWC images and bilinear-resize -> uint8
    [R, OH, OW, C] (K5/K7). The ensemble's detector->classifier wire format: 3 bytes per pixel."""
    n, H, W, C = img_u8.shape
    R = boxes.shape[0]
    if _ext.backend_for(img_u8) == "hip":
        out = torch.empty(R, out_hw[0], out_hw[1], C, device=img_u8.device, dtype=torch.uint8)
        _ext.call("ai4e_crop_resize_nhwc", img_u8.contiguous().data_ptr(), boxes.float().contiguous().data_ptr(),
                  out.data_ptr(), 0, H, W, C, R, out_hw[0], out_hw[1], 1, _ext.stream_ptr(img_u8.device))
        return out
    return crop_resize_u8_reference(img_u8, boxes, out_hw).to(img_u8.device)


def resize_u8(img_u8: torch.Tensor, out_hw: Tuple[int, int]) -> torch.Tensor:
    """Bilinear resize of uint8 NHWC images on the GPU (K7): one whole-image box per image."""
    n, H, W, _ = img_u8.shape
    boxes = torch.tensor([[i, 0.0, 0.0, float(W), float(H)] for i in range(n)], dtype=torch.float32,
                         device=img_u8.device)
    return crop_resize_u8(img_u8, boxes, out_hw)
