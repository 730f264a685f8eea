"""Servables: what a GPU worker runs for an endpoint and how its per-task result is encoded.

The reference's "drop-in model" is an arbitrary user function behind ``APIService``
(``APIs/1.0/base-py/ai4e_service.py:72-101``) that writes its result wherever it likes and reports
``CompleteTask(taskId, "completed - <result location>")``. Here a model endpoint's output is a
fixed tuple of per-image tensors, so a whole GPU batch travels back to the scheduler as one
item-major byte buffer (row ``r`` = every output of task ``r``) and is attached to the task records
natively; ``GET /v1/taskmanagement/task/{id}/result`` decodes the row with the endpoint's
:class:`OutputField` list and formats it.

Servables for the platform's model families:

* :class:`ClassifierServable` — logits model (or a fused top-k head) -> ``classes`` / ``probabilities``
  (ResNet-50, the camera-trap crop classifier);
* :class:`DetectorServable` — Faster-RCNN padded detections -> ``detections`` (boxes, scores, labels);
* :class:`SegmenterServable` — land-cover U-Net over a tiled mosaic -> class map (+ histogram);
* :class:`EnsembleServable` — detector -> crop classifier (one GPU: ``models.zoo.StaticEnsemble``; N:M GPUs over
  RCCL: :class:`runtime.pipeline.StageGraphPipeline`).
"""
from __future__ import annotations

import base64
import io
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch


@dataclass(frozen=True)
class OutputField:
    name: str
    dtype: str               # numpy dtype string, e.g. "int32"
    shape: Tuple[int, ...]   # per task

    @property
    def nbytes(self) -> int:
        return int(np.prod(self.shape, dtype=np.int64)) * np.dtype(self.dtype).itemsize

    def to_json(self) -> list:
        return [self.name, self.dtype, list(self.shape)]

    @staticmethod
    def from_json(x) -> "OutputField":
        return OutputField(str(x[0]), str(x[1]), tuple(int(v) for v in x[2]))


def row_bytes(fields: Sequence[OutputField]) -> int:
    return sum(f.nbytes for f in fields)


def encode_rows(outputs: Sequence[np.ndarray], n: int) -> bytes:
    """Item-major rows of a batch: row r = concat(out[r] for out in outputs) as raw bytes."""
    if not outputs:
        return b""
    cols = [np.ascontiguousarray(o[:n]).reshape(n, -1).view(np.uint8) for o in outputs]
    return np.concatenate(cols, axis=1).tobytes() if len(cols) > 1 else cols[0].tobytes()


def decode_row(row: bytes, fields: Sequence[OutputField]) -> Dict[str, np.ndarray]:
    out, off = {}, 0
    for f in fields:
        a = np.frombuffer(row, dtype=np.uint8, count=f.nbytes, offset=off).view(f.dtype).reshape(f.shape)
        out[f.name] = a
        off += f.nbytes
    return out


class Servable:
    """Base: ``__call__(u8 images [b, H, W, C] on device) -> tuple of [b, ...] tensors``.

    ``format`` is a staticmethod of the decoded fields only, so the scheduler process formats
    results for ``GET .../result`` without instantiating the model (``KINDS[kind].format``)."""

    kind = "raw"
    outputs: List[OutputField] = []

    def __call__(self, images_u8: torch.Tensor) -> Tuple[torch.Tensor, ...]:
        raise NotImplementedError

    @staticmethod
    def format(fields: Dict[str, np.ndarray]) -> dict:
        return {k: v.tolist() for k, v in fields.items()}

    def describe(self) -> dict:
        return {"kind": self.kind, "outputs": [f.to_json() for f in self.outputs]}


class ClassifierServable(Servable):
    """logits model or fused head -> top-k ``classes`` (int32) + ``probabilities`` (fp32)."""

    kind = "classifier"

    def __init__(self, model: Callable, topk: int = 5, head: Optional[Callable] = None):
        self.model = model
        self.topk = int(topk)
        self.head = head if head is not None else getattr(model, "topk_u8", None)
        self.outputs = [OutputField("classes", "int32", (self.topk,)), OutputField("probabilities", "float32",
                                                                                   (self.topk,))]

    def __call__(self, images_u8: torch.Tensor):
        if self.head is not None:
            i, p = self.head(images_u8, self.topk)
            return i, p
        logits = self.model(images_u8)
        p, i = torch.topk(torch.softmax(logits.float(), 1), self.topk, 1)
        return i.to(torch.int32), p

    @staticmethod
    def format(fields):
        return {"classes": fields["classes"].tolist(), "probabilities": [float(x) for x in fields["probabilities"]]}


class DetectorServable(Servable):
    """Faster-RCNN (``FasterRCNN.forward_u8``) padded detections -> JSON detections."""

    kind = "detector"

    def __init__(self, detector, max_dets: Optional[int] = None):
        self.detector = detector
        d = int(max_dets or detector.cfg.detections_per_img)
        self.max_dets = d
        self.outputs = [OutputField("boxes", "float32", (d, 4)), OutputField("scores", "float32", (d,)),
                        OutputField("labels", "int32", (d,)), OutputField("count", "int32", (1,))]

    def __call__(self, images_u8):
        boxes, scores, labels, n = self.detector.forward_u8(images_u8)
        d = self.max_dets
        return (boxes[:, :d].float().contiguous(), scores[:, :d].float().contiguous(),
                labels[:, :d].to(torch.int32).contiguous(), n.to(torch.int32).reshape(-1, 1))

    @staticmethod
    def format(fields):
        k = min(int(fields["count"][0]), fields["scores"].shape[0])
        return {"detections": [{"bbox": [round(float(v), 2) for v in fields["boxes"][i]],
                                "score": round(float(fields["scores"][i]), 4), "label": int(fields["labels"][i])}
                               for i in range(k)]}


def encode_class_map(cls: np.ndarray, encoding: str = "png") -> Tuple[str, str]:
    if encoding == "png":
        from PIL import Image

        buf = io.BytesIO()
        Image.fromarray(np.ascontiguousarray(cls), mode="L").save(buf, format="PNG", compress_level=1)
        return "png-base64", base64.b64encode(buf.getvalue()).decode()
    return "raw-base64", base64.b64encode(np.ascontiguousarray(cls).tobytes()).decode()


class SegmenterServable(Servable):
    """Land-cover U-Net over one mosaic per task (tiled + stitched on the GPU, K6) -> class map."""

    kind = "segmenter"

    def __init__(self, segmenter, height: int, width: int, n_classes: int):
        self.segmenter = segmenter  # uint8 [H, W, C] on device -> uint8 class map [H, W]
        self.n_classes = int(n_classes)
        self.outputs = [OutputField("class_map", "uint8", (height, width)),
                        OutputField("histogram", "int64", (self.n_classes,))]

    def __call__(self, images_u8):
        maps = [self.segmenter(images_u8[i]) for i in range(images_u8.shape[0])]
        cls = torch.stack(maps)
        # per-class pixel counts without a host sync (bincount sizes its output from the data), so the whole
        # servable can be captured in a HIP graph
        classes = torch.arange(self.n_classes, device=cls.device, dtype=cls.dtype)
        hist = (cls.reshape(cls.shape[0], 1, -1) == classes[None, :, None]).sum(-1)
        return cls, hist

    @staticmethod
    def format(fields):
        enc, data = encode_class_map(fields["class_map"])
        return {"shape": list(fields["class_map"].shape), "n_classes": int(fields["histogram"].shape[0]),
                "histogram": fields["histogram"].tolist(), "encoding": enc, "class_map": data}


class EnsembleServable(Servable):
    """Detector -> crop classifier on one GPU: detections + the species class of each crop."""

    kind = "ensemble"

    def __init__(self, pipeline, max_crops: int):
        self.pipeline = pipeline  # (subclasses: a StaticEnsemble or a StageGraphPipeline leader)
        self.max_crops = int(max_crops)
        m = self.max_crops
        self.outputs = [OutputField("boxes", "float32", (m, 4)), OutputField("det_scores", "float32", (m,)),
                        OutputField("species", "int32", (m,)), OutputField("species_prob", "float32", (m,)),
                        OutputField("count", "int32", (1,))]

    def __call__(self, images_u8):
        raise NotImplementedError  # (boxes, det_scores, species, species_prob, count) per image

    @staticmethod
    def format(fields):
        k = min(int(fields["count"][0]), fields["species"].shape[0])
        return {"animals": [{"bbox": [round(float(v), 2) for v in fields["boxes"][i]],
                             "detection_score": round(float(fields["det_scores"][i]), 4),
                             "species": int(fields["species"][i]),
                             "species_probability": round(float(fields["species_prob"][i]), 4)}
                            for i in range(k)]}


class ResizingServable(Servable):
    """K7 on the GPU: the endpoint's payload slots hold frames of the camera's native size and the
    bilinear uint8 resize to the model resolution runs inside the same captured graph (``resize_u8``,
    one whole-image crop-resize per frame) — the data-prep stage of the reference diagram
    (``Assets/platform_diagram.jpeg``: API1 data prep -> API2 inference) fused into the inference call.
    Box outputs are scaled back to native-frame coordinates."""

    def __init__(self, inner: Servable, model_hw: Tuple[int, int], box_fields: Sequence[str] = ()):
        self.inner = inner
        self.model_hw = tuple(model_hw)
        self.kind = inner.kind
        self.outputs = inner.outputs
        self.box_fields = tuple(box_fields)
        for k in ("stages",):
            if hasattr(inner, k):
                setattr(self, k, getattr(inner, k))

    def __call__(self, images_u8):
        from ..ops.detection import resize_u8

        h, w = images_u8.shape[1:3]
        x = images_u8 if (h, w) == self.model_hw else resize_u8(images_u8, self.model_hw)
        outs = list(self.inner(x))
        if self.box_fields and (h, w) != self.model_hw:
            sx, sy = w / self.model_hw[1], h / self.model_hw[0]
            scale = torch.tensor([sx, sy, sx, sy], device=outs[0].device, dtype=torch.float32)
            for i, f in enumerate(self.outputs):
                if f.name in self.box_fields:
                    outs[i] = outs[i] * scale
        return tuple(outs)

    def format(self, fields):
        return self.inner.format(fields)

    def describe(self) -> dict:
        return self.inner.describe()

    def close(self) -> None:
        close = getattr(self.inner, "close", None)
        if callable(close):
            close()


KINDS = {c.kind: c for c in (Servable, ClassifierServable, DetectorServable, SegmenterServable, EnsembleServable)}


def format_result(kind: str, fields_json: Sequence, row: Optional[bytes]) -> Optional[dict]:
    if row is None:
        return None
    fields = [OutputField.from_json(f) for f in fields_json]
    if kind not in KINDS and kind == "extent_segmenter":
        from . import extent  # noqa: F401  (registers its kind)
    return KINDS.get(kind, Servable).format(decode_row(row, fields))


def as_servable(obj, topk: int = 5) -> Servable:
    """Factories may return a Servable or a plain logits model (-> top-k classifier)."""
    return obj if isinstance(obj, Servable) else ClassifierServable(obj, topk)
