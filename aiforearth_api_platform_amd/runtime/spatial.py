"""Spatial-parallel tiled segmentation (BASELINE config #4): a large raster across GPUs over xGMI.

The reference's land-cover API only offers caller-side tiling (``classify`` / ``tile`` /
``tilebyextent`` ops, ``APIManagement/create_sync_api_management_api.sh:52-92``). Here one
4096x4096 (or larger) RGB+NIR mosaic is segmented by all ranks at once — the imagery analogue of
context parallelism (survey §5.7):

1. rank 0 owns the request; the mosaic is broadcast over RCCL (64 MiB for 4096^2 x 4 uint8);
2. the regular tile grid (``TileGrid``: tile ``ts``, ``stride``, overlap ``ts - stride``) is cut by
   whole tile rows, balanced over ranks; each rank runs the fused U-Net on its own tiles only
   (no redundant compute);
3. **halo exchange**: mosaic rows in the overlap band between two ranks need the neighbour's
   boundary tile row, so every rank ``isend``s its *last* tile row of logits to rank+1 (issued as
   soon as that row is computed, overlapped with the rest of its tiles) — one P2P transfer over
   one xGMI link per boundary;
4. each rank blends + argmaxes its own mosaic rows with the gather-form stitch kernel (K6);
5. the per-rank class bands are sent to rank 0 (P2P) and concatenated.

Works with any ``torch.distributed`` backend (``nccl`` = RCCL on the GPU node; ``gloo`` in the CPU
tests) and degenerates to a single-process path when world size is 1.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Tuple

import torch
import torch.distributed as dist

from ..ops.stitch import TileGrid, tile_stitch


def split_tile_rows(nty: int, world: int) -> List[Tuple[int, int]]:
    """Balanced contiguous [ty0, ty1) tile-row ranges per rank (first ranks get the extra rows)."""
    base, extra = divmod(nty, world)
    out, t = [], 0
    for r in range(world):
        n = base + (1 if r < extra else 0)
        out.append((t, t + n))
        t += n
    return out


def owned_rows(grid: TileGrid, ranges: List[Tuple[int, int]], r: int) -> Tuple[int, int]:
    """Mosaic rows [row0, row1) stitched by rank r: from its first tile's origin to the next rank's."""
    ty0, ty1 = ranges[r]
    row0 = 0 if r == 0 else ty0 * grid.stride
    row1 = grid.height if r == len(ranges) - 1 else ranges[r + 1][0] * grid.stride
    return min(row0, grid.height), min(row1, grid.height)


class SpatialSegmenter:
    def __init__(self, model_fn: Callable[[torch.Tensor], torch.Tensor], grid: TileGrid, n_out: int,
                 device: torch.device, tile_batch: int = 16, group=None, local: bool = False):
        """model_fn: uint8 tiles [b, ts, ts, C_in] -> logits NHWC [b, ts, ts, n_out].
        ``local``: one-GPU segmentation even inside an initialized process group (a pool worker)."""
        self.model_fn = model_fn
        self.grid = grid
        self.n_out = n_out
        self.device = device
        self.tile_batch = tile_batch
        self.group = group
        dist_on = dist.is_initialized() and not local
        self.rank = dist.get_rank(group) if dist_on else 0
        self.world = dist.get_world_size(group) if dist_on else 1
        self.bytes_sent = 0      # P2P / broadcast payload bytes over the group (xGMI on the GPU node)
        self.bytes_received = 0
        if grid.ts >= 2 * grid.stride:
            raise ValueError("tile overlap must be < 50% (a halo of one tile row per boundary)")
        if grid.nty < self.world:
            raise ValueError(f"{grid.nty} tile rows cannot be split over {self.world} ranks")

    def _tiles_for(self, mosaic: torch.Tensor, ty0: int, ty1: int) -> torch.Tensor:
        g = self.grid
        hp, wp = g.padded_hw()
        h, w, c = mosaic.shape
        if (hp, wp) != (h, w):
            pad = torch.zeros(hp, wp, c, dtype=mosaic.dtype, device=mosaic.device)
            pad[:h, :w] = mosaic
            mosaic = pad
        rows = []
        for ty in range(ty0, ty1):
            y = ty * g.stride
            band = mosaic[y:y + g.ts]                                   # [ts, wp, c]
            rows.append(band.unfold(1, g.ts, g.stride).permute(1, 0, 3, 2))  # [ntx, ts, ts, c]
        return torch.stack(rows) if rows else torch.zeros(0, g.ntx, g.ts, g.ts, c, dtype=mosaic.dtype,
                                                          device=mosaic.device)

    def _infer(self, tiles: torch.Tensor) -> torch.Tensor:
        """tiles [nrows, ntx, ts, ts, c] uint8 -> logits [nrows, ntx, ts, ts, n_out]."""
        nr, ntx = tiles.shape[:2]
        flat = tiles.reshape(nr * ntx, *tiles.shape[2:]).contiguous()
        outs = [self.model_fn(flat[i:i + self.tile_batch]) for i in range(0, flat.shape[0], self.tile_batch)]
        return torch.cat(outs).reshape(nr, ntx, *outs[0].shape[1:])[..., : self.n_out]

    def run(self, mosaic: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        """mosaic [H, W, C] uint8 on rank 0 (ignored elsewhere). Returns the class map on rank 0."""
        g = self.grid
        r, world = self.rank, self.world
        if world > 1:
            shape = torch.tensor(list(mosaic.shape) if r == 0 else [0, 0, 0], dtype=torch.int64, device=self.device)
            dist.broadcast(shape, 0, group=self.group)
            if int(shape[0]) < 0:  # the leader released the group (stop())
                return None
            if r != 0:
                mosaic = torch.empty(*shape.tolist(), dtype=torch.uint8, device=self.device)
            else:
                mosaic = mosaic.to(self.device)
            dist.broadcast(mosaic, 0, group=self.group)
        else:
            mosaic = mosaic.to(self.device)
        return self._segment(mosaic)

    def _segment(self, mosaic: torch.Tensor) -> Optional[torch.Tensor]:
        g = self.grid
        r, world = self.rank, self.world
        ranges = split_tile_rows(g.nty, world)
        ty0, ty1 = ranges[r]
        row0, row1 = owned_rows(g, ranges, r)
        tiles = self._tiles_for(mosaic, ty0, ty1)
        send_req = None
        # last tile row first, so the halo for rank+1 is on the wire while the rest computes
        if ty1 > ty0:
            last = self._infer(tiles[-1:])
            if r + 1 < world:
                send_req = dist.isend(last.contiguous(), r + 1, group=self.group)
                self.bytes_sent += last.numel() * last.element_size()
            rest = self._infer(tiles[:-1]) if ty1 - ty0 > 1 else last[:0]
            logits = torch.cat([rest, last])
        else:
            logits = torch.zeros(0, g.ntx, g.ts, g.ts, self.n_out, device=self.device, dtype=torch.bfloat16)
        lt0 = ty0
        if r > 0:  # halo: previous rank's last tile row
            halo = torch.empty(1, g.ntx, g.ts, g.ts, self.n_out, dtype=logits.dtype, device=self.device)
            dist.recv(halo, r - 1, group=self.group)
            self.bytes_received += halo.numel() * halo.element_size()
            logits = torch.cat([halo, logits])
            lt0 = ty0 - 1
        cls, _ = tile_stitch(logits, g, row0=row0, rows=row1 - row0, ty0=lt0)
        if send_req is not None:
            send_req.wait()
        if world == 1:
            return cls
        if r != 0:
            dist.send(cls.contiguous(), 0, group=self.group)
            self.bytes_sent += cls.numel()
            return None
        bands = [cls]
        for src in range(1, world):
            a, b = owned_rows(g, ranges, src)
            buf = torch.empty(b - a, g.width, dtype=torch.uint8, device=self.device)
            dist.recv(buf, src, group=self.group)
            self.bytes_received += buf.numel()
            bands.append(buf)
        return torch.cat(bands)

    # ------------------------------------------------------------ API worker group (leader + followers)
    def serve_follower(self) -> int:
        """Non-zero ranks of a land-cover worker group: segment every mosaic the leader broadcasts
        until it calls :meth:`stop`. Returns the number of mosaics served."""
        n = 0
        while True:
            shape = torch.zeros(3, dtype=torch.int64, device=self.device)
            dist.broadcast(shape, 0, group=self.group)
            if int(shape[0]) < 0:
                return n
            self._run_follower(tuple(int(v) for v in shape.tolist()))
            n += 1

    def _run_follower(self, shape) -> None:
        # same collective sequence as run() on a non-zero rank, after the shape broadcast
        mosaic = torch.empty(*shape, dtype=torch.uint8, device=self.device)
        dist.broadcast(mosaic, 0, group=self.group)
        self._segment(mosaic)

    def stop(self) -> None:
        if self.world > 1 and self.rank == 0:
            dist.broadcast(torch.full((3,), -1, dtype=torch.int64, device=self.device), 0, group=self.group)
