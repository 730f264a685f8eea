"""A GPU model exposed as an API endpoint: payload decode -> pinned ring slot -> task -> batch worker.

This is the "drop-in model" container of the reference (``APIs/Charts/templates/async-gpu``,
``APIs/1.0/base-py/ai4e_service.py``) collapsed into the node process: request bodies are decoded
once on the CPU straight into a slot of the pinned payload ring, the task record is created in the
native store and the slot index travels through the dispatch queue, so the GPU worker's H2D copy
reads the request bytes exactly where the front end put them.
"""
from __future__ import annotations

import base64
import io
import json
import threading
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..store import STATE_CREATED, STATE_FAILED, APITask
from .serving import GpuBatchWorker, ResultStore


class PayloadError(ValueError):
    pass


def decode_image(body: bytes, content_type: str, shape: Tuple[int, int, int]) -> np.ndarray:
    """Decode a request body to uint8 HxWxC of ``shape`` (resizing if needed).

    Accepted: raw ``application/octet-stream`` (exactly H*W*C bytes), ``application/x-npy``
    (``numpy.load(allow_pickle=False)``), ``image/jpeg``/``image/png``/``image/tiff`` (PIL), and JSON
    ``{"image_b64": ..., "shape": [H, W, C]}`` with raw bytes.
    """
    h, w, c = shape
    ct = (content_type or "").split(";")[0].strip().lower()
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
        im = im.convert("RGB" if c == 3 else ("L" if c == 1 else "RGBA"))
        if im.size != (w, h):
            im = im.resize((w, h), Image.BILINEAR)
        arr = np.asarray(im, dtype=np.uint8)
    else:
        if len(body) != h * w * c:
            raise PayloadError(f"raw payload must be {h * w * c} bytes (uint8 {h}x{w}x{c}), got {len(body)}")
        arr = np.frombuffer(body, dtype=np.uint8).reshape(h, w, c)
    if arr.dtype != np.uint8:
        arr = np.clip(arr, 0, 255).astype(np.uint8)
    if arr.ndim == 2:
        arr = arr[..., None]
    if arr.shape[2] != c:
        raise PayloadError(f"expected {c} channels, got {arr.shape[2]}")
    if arr.shape[:2] != (h, w):
        t = torch.from_numpy(np.ascontiguousarray(arr)).permute(2, 0, 1)[None].float()
        t = torch.nn.functional.interpolate(t, size=(h, w), mode="bilinear", align_corners=False)
        arr = t[0].permute(1, 2, 0).round().clamp(0, 255).to(torch.uint8).numpy()
    return arr


class ModelEndpoint:
    def __init__(self, control_plane, path: str, engine, ring, worker: Optional[GpuBatchWorker] = None,
                 decode: Optional[Callable[[bytes, str], np.ndarray]] = None, base_url: str = "http://127.0.0.1"):
        self.cp = control_plane
        self.path = path
        self.endpoint = base_url.rstrip("/") + path
        self.engine = engine
        self.ring = ring
        self.results: ResultStore = worker.results if worker is not None else ResultStore()
        self.worker = worker or GpuBatchWorker(control_plane, self.endpoint, engine, ring, results=self.results)
        self.worker.on_batch_done = self._on_done
        self.decode = decode or (lambda body, ct: decode_image(body, ct, ring.item_shape))
        self.queue = control_plane.queue_for(self.endpoint)
        self._waiters: Dict[str, Callable[[str], None]] = {}
        self._wmu = threading.Lock()

    # ------------------------------------------------------------- ingest
    def ingest(self, body: bytes, content_type: str) -> int:
        arr = self.decode(body, content_type)
        slot = self.ring.alloc(1, timeout=30)[0]
        self.ring.buf[slot].copy_(torch.from_numpy(np.require(arr, requirements=["C", "W"])))
        return slot

    def submit(self, body: bytes, content_type: str = "application/octet-stream", task_id: str = "",
               on_done: Optional[Callable[[str], None]] = None) -> str:
        """Async API: decode, create task (or adopt an upstream ``taskId``), enqueue. Returns task JSON."""
        slot = self.ingest(body, content_type)
        serialized, _ = self.cp.store.upsert(task_id, STATE_CREATED, STATE_CREATED, self.endpoint, None, True)
        tid = json.loads(serialized)["TaskId"]
        if on_done is not None:
            with self._wmu:
                self._waiters[tid] = on_done
        if not self.queue.send(tid, slot, ""):
            self.ring.free([slot])
            serialized, _ = self.cp.store.upsert(tid, "Failed - unable to send to backend service.", STATE_FAILED,
                                                 self.endpoint, None, True)
            with self._wmu:
                self._waiters.pop(tid, None)
        return serialized

    def submit_many(self, images_u8: np.ndarray) -> List[str]:
        """Bulk async submit of already-decoded images (batch clients / benchmarks)."""
        n = images_u8.shape[0]
        slots = self.ring.alloc(n, timeout=60)
        for i, s in enumerate(slots):
            self.ring.buf[s].copy_(torch.from_numpy(images_u8[i]))
        ids = self.cp.store.create_many(self.endpoint, n)
        self.queue.send_many(ids, slots)
        return ids

    def result(self, task_id: str) -> Optional[dict]:
        return self.results.get(task_id)

    def _on_done(self, ids: Sequence[str]) -> None:
        if not self._waiters:
            return
        with self._wmu:
            cbs = [(t, self._waiters.pop(t)) for t in ids if t in self._waiters]
        for t, cb in cbs:
            cb(t)

    def start(self) -> "ModelEndpoint":
        self.worker.start()
        return self

    def stop(self) -> None:
        self.worker.stop()
