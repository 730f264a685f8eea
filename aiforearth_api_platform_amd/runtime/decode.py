"""Request-body decoding for the image endpoints (numpy + Pillow; torch only for resizing raw arrays).

Kept free of a torch import so the gateway's decode worker processes (:mod:`runtime.decode_pool`) start
in well under a second.
"""
from __future__ import annotations

import base64
import io
import json
from typing import Tuple

import numpy as np


class PayloadError(ValueError):
    """A request body that cannot be decoded into the endpoint's input (HTTP 400 / 415)."""

    def __init__(self, msg: str, status: int = 400):
        super().__init__(msg)
        self.status = status


def decode_image(body: bytes, content_type: str, shape: Tuple[int, int, int]) -> np.ndarray:
    """Decode a request body to uint8 HxWxC of ``shape`` (resizing if needed).

    Accepted: raw ``application/octet-stream`` (exactly H*W*C bytes), ``application/x-npy``
    (``numpy.load(allow_pickle=False)``), ``image/jpeg``/``image/png``/``image/tiff`` (PIL), and JSON
    ``{"image_b64": ..., "shape": [H, W, C]}`` with raw bytes.
    """
    h, w, c = shape
    ct = (content_type or "").split(";")[0].strip().lower()
    try:
        if ct in ("application/json", "text/json"):
            d = json.loads(body or b"{}")
            raw = base64.b64decode(d["image_b64"])
            shp = tuple(d.get("shape", shape))
            arr = np.frombuffer(raw, dtype=np.uint8).reshape(shp)
        elif ct == "application/x-npy":
            arr = np.load(io.BytesIO(body), allow_pickle=False)
        elif ct.startswith("image/"):
            from PIL import Image

            im = Image.open(io.BytesIO(body))
            if im.format == "JPEG" and (im.size[0] >= 2 * w or im.size[1] >= 2 * h):
                # decode straight to 1/2..1/8 scale in the DCT domain (camera frames -> model size: 2-4x less
                # decode work, bench/jpeg_ingest_bench.py)
                im.draft("L" if c == 1 else "RGB", (w, h))
            im = im.convert("RGB" if c == 3 else ("L" if c == 1 else "RGBA"))
            if im.size != (w, h):
                im = im.resize((w, h), Image.BILINEAR, reducing_gap=2.0)
            arr = np.asarray(im, dtype=np.uint8)
        elif ct in ("", "application/octet-stream"):
            if len(body) != h * w * c:
                raise PayloadError(f"raw payload must be {h * w * c} bytes (uint8 {h}x{w}x{c}), got {len(body)}")
            arr = np.frombuffer(body, dtype=np.uint8).reshape(h, w, c)
        else:
            raise PayloadError(f"unsupported content type {ct!r}", 415)
    except PayloadError:
        raise
    except Exception as e:  # malformed JSON / base64 / npy / image bytes
        raise PayloadError(f"cannot decode payload: {e}") from e
    if arr.dtype != np.uint8:
        arr = np.clip(arr, 0, 255).astype(np.uint8)
    if arr.ndim == 2:
        arr = arr[..., None]
    if arr.ndim != 3 or arr.shape[2] != c:
        raise PayloadError(f"expected {c} channels, got shape {arr.shape}")
    if arr.shape[:2] != (h, w):
        import torch

        t = torch.from_numpy(np.ascontiguousarray(arr)).permute(2, 0, 1)[None].float()
        t = torch.nn.functional.interpolate(t, size=(h, w), mode="bilinear", align_corners=False)
        arr = t[0].permute(1, 2, 0).round().clamp(0, 255).to(torch.uint8).numpy()
    return arr
