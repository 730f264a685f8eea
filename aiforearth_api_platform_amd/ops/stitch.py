"""Tile-stitch [K6]: blend overlapping tile logits into a mosaic and take the argmax."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import torch

from . import _ext


@dataclass(frozen=True)
class TileGrid:
    """Regular tiling of an H x W mosaic with tiles of ``ts`` pixels every ``stride`` pixels."""

    height: int
    width: int
    ts: int
    stride: int

    @property
    def overlap(self) -> int:
        return self.ts - self.stride

    @property
    def nty(self) -> int:
        return max(1, -(-(self.height - self.ts) // self.stride) + 1)

    @property
    def ntx(self) -> int:
        return max(1, -(-(self.width - self.ts) // self.stride) + 1)

    def origin(self, ty: int, tx: int) -> Tuple[int, int]:
        return ty * self.stride, tx * self.stride

    def padded_hw(self) -> Tuple[int, int]:
        return (self.nty - 1) * self.stride + self.ts, (self.ntx - 1) * self.stride + self.ts

    def tile_rows_for(self, row0: int, row1: int) -> Tuple[int, int]:
        """[ty0, ty1) of the tiles that touch mosaic rows [row0, row1)."""
        ty0 = max(0, -(-(row0 - self.ts + 1) // self.stride))
        ty1 = min(self.nty, (row1 - 1) // self.stride + 1)
        return ty0, ty1


def _ramp(ts: int, ov: int, device) -> torch.Tensor:
    i = torch.arange(ts, dtype=torch.float32, device=device)
    if ov <= 0:
        return torch.ones(ts, device=device)
    return torch.minimum(torch.ones_like(i), torch.minimum((i + 0.5) / ov, (ts - i - 0.5) / ov))


def stitch_reference(tiles: torch.Tensor, grid: TileGrid, row0: int = 0, rows: Optional[int] = None, ty0: int = 0,
                     with_prob: bool = False):
    """tiles [nty_local, ntx, ts, ts, C] -> (cls [rows, W] uint8, prob [rows, W, C] | None)."""
    rows = grid.height - row0 if rows is None else rows
    nty_l, ntx, ts, _, C = tiles.shape
    hp, wp = grid.padded_hw()
    acc = torch.zeros(hp, wp, C)
    wsum = torch.zeros(hp, wp)
    r = _ramp(ts, grid.overlap, "cpu")
    w2 = r[:, None] * r[None, :]
    for a in range(nty_l):
        for tx in range(ntx):
            y, x = grid.origin(ty0 + a, tx)
            acc[y:y + ts, x:x + ts] += w2[..., None] * tiles[a, tx].float().cpu()
            wsum[y:y + ts, x:x + ts] += w2
    acc = acc[row0:row0 + rows, :grid.width] / wsum[row0:row0 + rows, :grid.width, None].clamp(min=1e-12)
    cls = acc.argmax(-1).to(torch.uint8)
    return cls, (torch.softmax(acc, -1) if with_prob else None)


def tile_stitch(tiles: torch.Tensor, grid: TileGrid, row0: int = 0, rows: Optional[int] = None, ty0: int = 0,
                with_prob: bool = False):
    rows = grid.height - row0 if rows is None else rows
    if _ext.backend_for(tiles) == "hip":
        nty_l, ntx, ts, _, C = tiles.shape
        tiles = tiles.contiguous()
        cls = torch.empty(rows, grid.width, dtype=torch.uint8, device=tiles.device)
        prob = torch.empty(rows, grid.width, C, dtype=torch.bfloat16, device=tiles.device) if with_prob else None
        _ext.call("ai4e_tile_stitch", tiles.data_ptr(), cls.data_ptr(), _ext.ptr(prob), rows, grid.width, C, ts,
                  grid.stride, ntx, ty0, nty_l, grid.overlap, row0, _ext.stream_ptr(tiles.device))
        return cls, prob
    return stitch_reference(tiles, grid, row0, rows, ty0, with_prob)
