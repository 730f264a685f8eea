"""Land-cover extent operations: ``classifybyextent`` / ``tilebyextent`` over registered mosaics.

The reference's land-cover API publishes four sync operations, ``POST /v2/{classify, classifybyextent, tile,
tilebyextent}`` (``APIManagement/create_sync_api_management_api.sh:52-92``): the ``*byextent`` forms name an area
(an extent) instead of uploading pixels, and the service cuts it from the imagery it already holds. Here:

* **registered mosaics** (``mosaics:`` in the endpoint kwargs): uint8 H x W x C rasters loaded once into every
  worker's HBM (an ``.npy`` file read with ``allow_pickle=False``, or a seeded synthetic raster when no imagery
  is available offline) with a GDAL-style geotransform ``(x0, dx, rx, y0, ry, dy)`` mapping pixel (col, row) to
  geo coordinates;
* **the request** (JSON ``{"mosaic": name, "extent": {"xmin", "ymin", "xmax", "ymax"}, "crs": "pixel" | "geo"}``)
  is converted at ingest into a fixed 64-byte record (pixel bbox; geo extents through the inverse geotransform)
  so it rides the payload ring like any other item;
* **the worker** (:class:`ExtentSegmenter`) takes the tiles of the mosaic's full tile grid that touch the extent
  — exactly the tiles the full-mosaic ``classify`` would run there — crops them from the resident mosaic on the
  GPU, runs the U-Net, stitches the sub-grid (K6) and cuts the extent out. The extent's class map therefore
  equals the same window of the full ``classify`` result (the blend at every extent pixel sums the same tiles in
  the same order). ``tilebyextent`` returns the whole tile-aligned region around the extent instead.

The result row holds a class-map canvas of the endpoint's maximum extent plus the returned window
(``window`` = x0, y0, width, height in mosaic pixels); the formatter encodes only the window.
"""
from __future__ import annotations

import json
import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .decode import PayloadError
from .servable import OutputField, Servable, encode_class_map

RECORD_BYTES = 64
_MAGIC = 0x45585431  # "EXT1"
OP_CLASSIFY, OP_TILE = 0, 1


@dataclass(frozen=True)
class GeoTransform:
    """GDAL affine geotransform: geo_x = x0 + col * dx + row * rx, geo_y = y0 + col * ry + row * dy."""

    x0: float = 0.0
    dx: float = 1.0
    rx: float = 0.0
    y0: float = 0.0
    ry: float = 0.0
    dy: float = 1.0

    @staticmethod
    def of(v: Optional[Sequence[float]]) -> "GeoTransform":
        return GeoTransform(*[float(x) for x in v]) if v else GeoTransform()

    def to_pixel(self, gx: float, gy: float) -> Tuple[float, float]:
        """Geo (x, y) -> pixel (col, row) through the inverse affine map."""
        det = self.dx * self.dy - self.rx * self.ry
        if det == 0:
            raise PayloadError("singular geotransform")
        ux, uy = gx - self.x0, gy - self.y0
        col = (self.dy * ux - self.rx * uy) / det
        row = (-self.ry * ux + self.dx * uy) / det
        return col, row


@dataclass(frozen=True)
class MosaicSpec:
    name: str
    height: int
    width: int
    channels: int = 4
    geotransform: GeoTransform = GeoTransform()
    path: str = ""      # .npy uint8 [H, W, C] (allow_pickle=False); empty = synthetic
    seed: int = 0

    @staticmethod
    def parse(mosaics: Dict[str, dict]) -> List["MosaicSpec"]:
        out = []
        for name, m in sorted((mosaics or {}).items()):
            out.append(MosaicSpec(name, int(m["height"]), int(m["width"]), int(m.get("channels", 4)),
                                  GeoTransform.of(m.get("geotransform")), str(m.get("path", "")),
                                  int(m.get("seed", 0))))
        return out

    def load(self, device) -> torch.Tensor:
        if self.path:
            a = np.load(self.path, allow_pickle=False)
            if a.dtype != np.uint8 or a.shape != (self.height, self.width, self.channels):
                raise ValueError(f"mosaic {self.name}: {self.path} is {a.dtype} {a.shape}, expected uint8 "
                                 f"{(self.height, self.width, self.channels)}")
            return torch.from_numpy(a).to(device)
        return synthetic_mosaic(self.height, self.width, self.channels, self.seed, device)


def synthetic_mosaic(h: int, w: int, c: int, seed: int, device) -> torch.Tensor:
    """Deterministic uint8 raster (the same on every worker and in the tests): smooth fields + noise, so the
    class map has structure."""
    dev = torch.device(device)
    g = torch.Generator(device=dev).manual_seed(seed)  # generated where it lives (an 8192^2 mosaic: no host copy)
    coarse = torch.randint(0, 256, (c, max(2, h // 64), max(2, w // 64)), generator=g, device=dev).float()
    out = torch.empty(h, w, c, dtype=torch.uint8, device=dev)
    for r0 in range(0, h, 1024):  # row bands: bounded fp32 temporaries
        r1 = min(h, r0 + 1024)
        smooth = torch.nn.functional.interpolate(coarse[None], size=(h, w), mode="bilinear",
                                                 align_corners=False)[0, :, r0:r1] if h * w <= 1 << 22 else None
        if smooth is None:  # large rasters: interpolate the band's rows only (same sampling as the full grid)
            ys = (torch.arange(r0, r1, device=dev, dtype=torch.float32) + 0.5) * coarse.shape[1] / h - 0.5
            xs = (torch.arange(w, device=dev, dtype=torch.float32) + 0.5) * coarse.shape[2] / w - 0.5
            gy = (ys / max(1, coarse.shape[1] - 1)) * 2 - 1
            gx = (xs / max(1, coarse.shape[2] - 1)) * 2 - 1
            grid = torch.stack(torch.meshgrid(gx, gy, indexing="xy"), -1)[None]
            smooth = torch.nn.functional.grid_sample(coarse[None], grid, mode="bilinear", padding_mode="border",
                                                     align_corners=True)[0]
        noise = torch.randint(-24, 25, (c, r1 - r0, w), generator=g, device=dev).float()
        out[r0:r1] = (smooth + noise).clamp(0, 255).to(torch.uint8).permute(1, 2, 0)
    return out


def encode_request(body: bytes, mosaics: Sequence[MosaicSpec], op: int, max_hw: Tuple[int, int], ts: int,
                   stride: int) -> np.ndarray:
    """JSON extent request -> the 64-byte payload record (int32 x 16) holding the window to return: the
    extent (classifybyextent) or the tile-aligned region of the grid's tiles that touch it (tilebyextent).
    400 on malformed / out-of-range extents, 413 when the window exceeds the endpoint's maximum."""
    try:
        d = json.loads(body or b"{}")
        names = [m.name for m in mosaics]
        name = d.get("mosaic", names[0] if len(names) == 1 else None)
        if name not in names:
            raise PayloadError(f"unknown mosaic {name!r}; registered: {names}")
        mi = names.index(name)
        m = mosaics[mi]
        e = d["extent"]
        xs, ys = (float(e["xmin"]), float(e["xmax"])), (float(e["ymin"]), float(e["ymax"]))
    except PayloadError:
        raise
    except (ValueError, KeyError, TypeError, AttributeError, IndexError) as err:  # (non-object bodies too)
        raise PayloadError(f"extent request must be JSON {{mosaic, extent: {{xmin, ymin, xmax, ymax}}, crs}}: {err}")
    if not all(math.isfinite(v) for v in xs + ys):  # json.loads accepts NaN / Infinity
        raise PayloadError("extent coordinates must be finite numbers")
    crs = str(d.get("crs", "pixel")).lower()
    try:
        if crs == "geo":
            corners = [m.geotransform.to_pixel(x, y) for x in xs for y in ys]
            c0, c1 = min(c for c, _ in corners), max(c for c, _ in corners)
            r0, r1 = min(r for _, r in corners), max(r for _, r in corners)
            x0, x1, y0, y1 = math.floor(c0), math.ceil(c1), math.floor(r0), math.ceil(r1)
        elif crs == "pixel":
            x0, x1, y0, y1 = int(xs[0]), int(xs[1]), int(ys[0]), int(ys[1])
        else:
            raise PayloadError(f"crs must be 'pixel' or 'geo', got {crs!r}")
    except (OverflowError, ValueError) as err:  # (a finite extent far outside any raster in geo units)
        raise PayloadError(f"extent out of range: {err}")
    x0, y0 = max(0, x0), max(0, y0)
    x1, y1 = min(m.width, x1), min(m.height, y1)
    if x1 <= x0 or y1 <= y0:
        raise PayloadError("extent does not intersect the mosaic")
    if op == OP_TILE:
        from ..ops.stitch import TileGrid

        g = TileGrid(m.height, m.width, ts, stride)
        ty0, ty1, tx0, tx1 = tile_window(g, x0, y0, x1, y1)
        x0, y0 = tx0 * g.stride, ty0 * g.stride
        x1, y1 = min(g.width, (tx1 - 1) * g.stride + g.ts), min(g.height, (ty1 - 1) * g.stride + g.ts)
    if y1 - y0 > max_hw[0] or x1 - x0 > max_hw[1]:
        raise PayloadError(f"extent {x1 - x0}x{y1 - y0} exceeds the endpoint's maximum {max_hw[1]}x{max_hw[0]}", 413)
    rec = np.zeros(RECORD_BYTES // 4, np.int32)
    rec[:7] = (_MAGIC, mi, x0, y0, x1, y1, op)
    return rec.view(np.uint8)


def request_decoder(mosaics: Sequence[MosaicSpec], op: int, max_hw: Tuple[int, int], ts: int, stride: int):
    """``ModelEndpoint(decode=...)`` for an extent endpoint (JSON bodies only)."""
    def decode(body: bytes, content_type: str) -> np.ndarray:
        ct = (content_type or "").split(";")[0].strip().lower()
        if ct not in ("application/json", "text/json", ""):
            raise PayloadError(f"extent requests are JSON, got {ct!r}", 415)
        return encode_request(body, mosaics, op, max_hw, ts, stride)
    return decode


def tile_window(grid, x0: int, y0: int, x1: int, y1: int) -> Tuple[int, int, int, int]:
    """[ty0, ty1, tx0, tx1) of the tiles of ``grid`` that touch pixel rows [y0, y1) and columns [x0, x1)."""
    ty0, ty1 = grid.tile_rows_for(y0, y1)
    tx0 = max(0, -(-(x0 - grid.ts + 1) // grid.stride))
    tx1 = min(grid.ntx, (x1 - 1) // grid.stride + 1)
    return ty0, ty1, tx0, tx1


class ExtentSegmenter:
    """Per-request window segmentation over resident mosaics (see module doc)."""

    def __init__(self, model_fn, mosaics: Sequence[MosaicSpec], ts: int, stride: int, n_out: int, device,
                 tile_batch: int = 16):
        from ..ops.stitch import TileGrid

        self.model_fn, self.n_out, self.device, self.tile_batch = model_fn, n_out, torch.device(device), tile_batch
        self.specs = list(mosaics)
        self.grids = [TileGrid(m.height, m.width, ts, stride) for m in self.specs]
        self.mosaics = [m.load(self.device) for m in self.specs]  # resident in HBM for the worker's lifetime

    def valid(self, rec: Sequence[int]) -> bool:
        _, mi, x0, y0, x1, y1 = (int(v) for v in rec[:6])
        return 0 <= mi < len(self.grids) and 0 <= x0 < x1 <= self.grids[mi].width and 0 <= y0 < y1 <= self.grids[mi].height

    def __call__(self, rec: Sequence[int]) -> Tuple[torch.Tensor, Tuple[int, int, int, int]]:
        """Class map of the record's window (the ingest already resolved the op to a window)."""
        from ..ops.stitch import TileGrid, tile_stitch

        _, mi, x0, y0, x1, y1 = (int(v) for v in rec[:6])
        if not (0 <= mi < len(self.grids)):
            raise ValueError(f"extent record names mosaic {mi}; {len(self.grids)} registered")
        if not (0 <= x0 < x1 <= self.grids[mi].width and 0 <= y0 < y1 <= self.grids[mi].height):
            raise ValueError(f"extent window ({x0}, {y0}, {x1}, {y1}) outside mosaic {self.specs[mi].name}")
        g, mosaic = self.grids[mi], self.mosaics[mi]
        ty0, ty1, tx0, tx1 = tile_window(g, x0, y0, x1, y1)
        oy, ox = ty0 * g.stride, tx0 * g.stride
        hs, ws = (ty1 - ty0 - 1) * g.stride + g.ts, (tx1 - tx0 - 1) * g.stride + g.ts
        region = torch.zeros(hs, ws, mosaic.shape[2], dtype=torch.uint8, device=self.device)  # zero past the edge
        hh, ww = min(hs, g.height - oy), min(ws, g.width - ox)
        region[:hh, :ww] = mosaic[oy:oy + hh, ox:ox + ww]
        sub = TileGrid(hs, ws, g.ts, g.stride)
        tiles = region.unfold(0, g.ts, g.stride).unfold(1, g.ts, g.stride).permute(0, 1, 3, 4, 2)  # [nty,ntx,ts,ts,c]
        nty, ntx = tiles.shape[:2]
        flat = tiles.reshape(nty * ntx, g.ts, g.ts, -1).contiguous()
        logits = torch.cat([self.model_fn(flat[i:i + self.tile_batch]) for i in range(0, flat.shape[0],
                                                                                      self.tile_batch)])
        logits = logits.reshape(nty, ntx, *logits.shape[1:])[..., : self.n_out]
        cls, _ = tile_stitch(logits, sub)
        return cls[y0 - oy:y1 - oy, x0 - ox:x1 - ox], (x0, y0, x1 - x0, y1 - y0)


class ExtentServable(Servable):
    """Worker side of ``/v2/landcover/{classify,tile}byextent``: payload = 64-byte extent records."""

    kind = "extent_segmenter"

    def __init__(self, seg: ExtentSegmenter, max_hw: Tuple[int, int], n_classes: int):
        self.seg, self.max_hw, self.n_classes = seg, tuple(max_hw), int(n_classes)
        self.outputs = [OutputField("class_map", "uint8", self.max_hw), OutputField("window", "int32", (4,)),
                        OutputField("histogram", "int64", (self.n_classes,))]

    def __call__(self, records_u8: torch.Tensor):
        recs = records_u8.reshape(records_u8.shape[0], -1).cpu().numpy().view(np.int32)
        b = recs.shape[0]
        canvas = torch.zeros(b, *self.max_hw, dtype=torch.uint8, device=records_u8.device)
        win = torch.zeros(b, 4, dtype=torch.int32)
        hist = torch.zeros(b, self.n_classes, dtype=torch.int64, device=records_u8.device)
        for i in range(b):
            if int(recs[i, 0]) != _MAGIC:  # (padding rows of a partial batch bucket)
                continue
            # a record that did not come through encode_request (e.g. raw bytes) fails on its own: window x = -1
            # marks it invalid (invalid_rows), the other requests of the batch are served
            if (int(recs[i, 4]) - int(recs[i, 2]) > self.max_hw[1] or int(recs[i, 5]) - int(recs[i, 3]) > self.max_hw[0]
                    or not self.seg.valid(recs[i])):
                win[i, 0] = -1
                continue
            cls, (x, y, w, h) = self.seg(recs[i])
            canvas[i, :h, :w] = cls
            win[i] = torch.tensor([x, y, w, h], dtype=torch.int32)
            hist[i] = torch.bincount(cls.reshape(-1).long(), minlength=self.n_classes)[: self.n_classes]
        return canvas, win.to(records_u8.device), hist

    @staticmethod
    def invalid_rows(outputs) -> np.ndarray:
        """Rows whose record was refused (worker: status IT_INVALID for those items only)."""
        win = outputs[1]
        win = win.numpy() if isinstance(win, torch.Tensor) else np.asarray(win)
        return win[:, 0] < 0

    @staticmethod
    def format(fields):
        x, y, w, h = (int(v) for v in fields["window"])
        enc, data = encode_class_map(np.ascontiguousarray(fields["class_map"][:h, :w]))
        return {"window": {"x0": x, "y0": y, "width": w, "height": h}, "shape": [h, w],
                "n_classes": int(fields["histogram"].shape[0]), "histogram": fields["histogram"].tolist(),
                "encoding": enc, "class_map": data}


def _register() -> None:
    from .servable import KINDS

    KINDS[ExtentServable.kind] = ExtentServable


_register()
