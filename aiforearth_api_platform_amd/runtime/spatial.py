"""Spatial-parallel tiled segmentation (BASELINE config #4): a large raster across GPUs over xGMI.

The reference's land-cover API only offers caller-side tiling (``classify`` / ``tile`` /
``tilebyextent`` ops, ``APIManagement/create_sync_api_management_api.sh:52-92``). Here one
4096x4096 (or larger) RGB+NIR mosaic is segmented by all ranks at once — the imagery analogue of
context parallelism (survey §5.7):

1. the regular tile grid (``TileGrid``: tile ``ts``, ``stride``, overlap ``ts - stride``) is split by
   TILES (row-major flat ranges, at most one tile apart between ranks); each rank runs the fused
   U-Net on its own tiles only (no redundant compute);
2. rank 0 owns the request and sends each rank only the mosaic rows its tiles cover (one P2P
   message per rank over its own xGMI link, instead of broadcasting the whole 64 MiB mosaic);
3. **halo exchange, overlapped with compute**: stitching is by tile rows (a rank blends the mosaic rows
   from its first tile row's origin to the next rank's), so a rank needs the logits of its tile rows plus
   the row above; the tiles of those rows computed elsewhere come over in one ``batch_isend_irecv`` —
   contiguous slices, mostly from the two neighbouring ranks. Each rank infers its BOUNDARY tiles (the
   ones other ranks stitch over) first and posts the whole exchange right after them, so the halo moves
   over xGMI while the interior tiles run (survey §7.5.5/§7.5.6);
4. each rank blends + argmaxes its own mosaic rows with the gather-form stitch kernel (K6);
5. the per-rank class bands go to rank 0 in one batched P2P exchange (every band's receive posted at
   once) and are concatenated.

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
                 device: torch.device, tile_batch: int = 16, group=None, local: bool = False,
                 tile_graphs: bool = False):
        """model_fn: uint8 tiles [b, ts, ts, C_in] -> logits NHWC [b, ts, ts, n_out].
        ``local``: one-GPU segmentation even inside an initialized process group (a pool worker).
        ``tile_graphs``: run each tile batch through a HIP graph captured per batch shape (the group form, whose
        P2P exchanges keep the whole servable out of the worker's graph; the one-GPU form is captured whole)."""
        self.model_fn = model_fn
        if tile_graphs and torch.device(device).type == "cuda":
            from .pipeline import _GraphRunner

            self.model_fn = _GraphRunner(model_fn, torch.device(device))
        self._graphed = self.model_fn is not model_fn
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
        self.events: List[tuple] = []  # ("tiles", lo, hi) per inferred batch, ("halo_posted", ...) (tests)
        if grid.ts >= 2 * grid.stride:
            raise ValueError("tile overlap must be < 50% (a halo of one tile row per boundary)")
        if grid.nty < self.world:
            raise ValueError(f"{grid.nty} tile rows cannot be split over {self.world} ranks")

    # ------------------------------------------------------------ plan (a pure function of grid and world)
    def _plan(self):
        """(computed flat tile ranges, stitched tile-row ranges, needed flat tile ranges, mosaic row bands).

        Compute is balanced by TILES (row-major flat index; ranks differ by at most one tile: 4096^2 with
        512/448 tiles is 81 tiles -> 10-11 per rank on 8 GPUs, where whole tile rows gave 2 to rank 0 and 1
        to the rest). Stitching stays by tile rows (a rank blends the mosaic rows from its first tile row's
        origin to the next rank's), so a rank needs the logits of its tile rows plus the row above — flat
        ranges too, so every logits transfer between two ranks is ONE contiguous slice."""
        g, world = self.grid, self.world
        comp = split_tile_rows(g.nty * g.ntx, world)
        own = split_tile_rows(g.nty, world)
        need = [(max(0, a - 1) * g.ntx, b * g.ntx) for a, b in own]
        bands = []
        for a, b in comp:  # padded-mosaic rows [y0, y1) that rank r's tiles cover
            bands.append((a // g.ntx * g.stride, (b - 1) // g.ntx * g.stride + g.ts) if b > a else (0, 0))
        return comp, own, need, bands

    def _tiles_range(self, band: torch.Tensor, y0: int, a: int, b: int) -> torch.Tensor:
        """Tiles with flat indices [a, b) cut from ``band`` (mosaic rows from padded row ``y0``; zero padding
        below / right of the mosaic) -> [b - a, ts, ts, c]."""
        g = self.grid
        hp, wp = g.padded_hw()
        rows, c = band.shape[0], band.shape[2]
        need_h = (b - 1) // g.ntx * g.stride + g.ts - y0
        if rows < need_h or band.shape[1] < wp:
            pad = torch.zeros(need_h, wp, c, dtype=band.dtype, device=band.device)
            pad[:rows, :band.shape[1]] = band[:need_h]
            band = pad
        out = []
        for ty in range(a // g.ntx, (b - 1) // g.ntx + 1):
            t0, t1 = max(a, ty * g.ntx) - ty * g.ntx, min(b, (ty + 1) * g.ntx) - ty * g.ntx
            y = ty * g.stride - y0
            row = band[y:y + g.ts, :wp].unfold(1, g.ts, g.stride).permute(1, 0, 3, 2)  # [ntx, ts, ts, c]
            out.append(row[t0:t1])
        return torch.cat(out)

    def _infer(self, tiles: torch.Tensor, order: Optional[List[Tuple[int, int]]] = None,
               after: Optional[Tuple[int, Callable[[torch.Tensor], None]]] = None) -> torch.Tensor:
        """tiles [n, ts, ts, c] uint8 -> logits [n, ts, ts, n_out]. ``order``: the tile ranges [lo, hi) to run, in
        that order (default: all, in index order); ``after`` = (k, fn): fn(logits) once the first k ranges are done
        (the halo exchange is posted there, before the remaining tiles run)."""
        flat = tiles.contiguous()
        out = None
        ranges = order if order is not None else [(0, flat.shape[0])]
        pending = after is not None
        for j, (lo, hi) in enumerate(ranges):
            for i in range(lo, hi, self.tile_batch):
                if pending and j >= after[0] and out is not None:  # (the first moment the logits buffer exists)
                    after[1](out)
                    pending = False
                # each batch's logits go straight into one preallocated buffer (a graph's output buffer is reused by
                # its next replay; one copy per batch instead of a clone plus a concatenation)
                y = self.model_fn(flat[i:min(hi, i + self.tile_batch)])[..., : self.n_out]
                if out is None:
                    out = torch.empty(flat.shape[0], *y.shape[1:], dtype=y.dtype, device=y.device)
                out[i:i + y.shape[0]].copy_(y)
                self.events.append(("tiles", i, i + y.shape[0]))
        if pending and out is not None:
            after[1](out)
        return out

    @staticmethod
    def _boundary_first(a: int, b: int, sends: List[Tuple[int, int]]) -> Tuple[List[Tuple[int, int]], int]:
        """Tile ranges of [a, b) (local indices) with every range another rank needs first; returns (ranges, number
        of leading boundary ranges)."""
        cover = sorted((lo - a, hi - a) for lo, hi in sends if hi > lo)
        merged: List[Tuple[int, int]] = []
        for lo, hi in cover:
            if merged and lo <= merged[-1][1]:
                merged[-1] = (merged[-1][0], max(merged[-1][1], hi))
            else:
                merged.append((lo, hi))
        rest, t = [], 0
        for lo, hi in merged:
            if lo > t:
                rest.append((t, lo))
            t = hi
        if t < b - a:
            rest.append((t, b - a))
        return merged + rest, len(merged)

    def run(self, mosaic: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        """mosaic [H, W, C] uint8 on rank 0 (ignored elsewhere). Returns the class map on rank 0."""
        if self.world == 1:
            return self._segment(mosaic.to(self.device), 0)
        shape = torch.tensor(list(mosaic.shape) if self.rank == 0 else [0, 0, 0], dtype=torch.int64,
                             device=self.device)
        dist.broadcast(shape, group_src=0, group=self.group)
        if int(shape[0]) < 0:  # the leader released the group (stop())
            return None
        return self._scatter_and_segment(mosaic, tuple(int(v) for v in shape.tolist()))

    def _scatter_and_segment(self, mosaic: Optional[torch.Tensor], shape) -> Optional[torch.Tensor]:
        """Rank 0 sends every rank only the mosaic rows its tiles cover (one P2P message per rank, ~1/world of
        the mosaic plus one tile overlap, instead of a 64 MiB broadcast to all)."""
        h, w, c = shape
        _, _, _, bands = self._plan()
        if self.rank == 0:
            mosaic = mosaic.to(self.device)
            ops = []
            for s in range(1, self.world):
                y0, y1 = bands[s]
                part = mosaic[min(y0, h):min(y1, h)].contiguous()
                if part.numel():
                    ops.append(dist.P2POp(dist.isend, part, group=self.group, group_peer=s))
                    self.bytes_sent += part.numel()
            for wk in dist.batch_isend_irecv(ops) if ops else []:
                wk.wait()
            return self._segment(mosaic[:bands[0][1]], bands[0][0])
        y0, y1 = bands[self.rank]
        band = torch.empty(max(0, min(y1, h) - min(y0, h)), w, c, dtype=torch.uint8, device=self.device)
        if band.numel():
            for wk in dist.batch_isend_irecv([dist.P2POp(dist.irecv, band, group=self.group, group_peer=0)]):
                wk.wait()
            self.bytes_received += band.numel()
        return self._segment(band, y0)

    def _segment(self, band: torch.Tensor, y0: int) -> Optional[torch.Tensor]:
        g = self.grid
        r, world = self.rank, self.world
        comp, own, need, _ = self._plan()
        a, b = comp[r]
        na, nb = need[r]
        tiles = self._tiles_range(band, y0, a, b)
        if world == 1:
            full = self._infer(tiles)                                      # [b - a, ts, ts, n_out]
        else:
            # halo exchange: each rank sends every other rank the slice of its computed tiles that rank stitches
            # over (contiguous flat ranges: typically the neighbours' boundary tiles), all in one batch. Those
            # boundary tiles run first; the exchange is posted as soon as they are done and completes over xGMI
            # while the interior tiles run (the receives land in `full`, which only the stitch reads)
            sends = [(s, max(a, need[s][0]), min(b, need[s][1])) for s in range(world) if s != r]
            order, nfirst = self._boundary_first(a, b, [(lo, hi) for _, lo, hi in sends])
            box = {}

            def post(logits: torch.Tensor) -> None:
                full = torch.empty(nb - na, *logits.shape[1:], dtype=logits.dtype, device=self.device)
                ops = []
                for s, lo, hi in sends:
                    if hi > lo:
                        t = logits[lo - a:hi - a]
                        ops.append(dist.P2POp(dist.isend, t, group=self.group, group_peer=s))
                        self.bytes_sent += t.numel() * t.element_size()
                    lo, hi = max(comp[s][0], na), min(comp[s][1], nb)
                    if hi > lo:
                        ops.append(dist.P2POp(dist.irecv, full[lo - na:hi - na], group=self.group, group_peer=s))
                        self.bytes_received += (hi - lo) * logits[0].numel() * logits.element_size()
                box["full"], box["works"] = full, (dist.batch_isend_irecv(ops) if ops else [])
                self.events.append(("halo_posted", len(ops)))

            logits = self._infer(tiles, order=order, after=(nfirst, post))
            full = box["full"]
            lo, hi = max(a, na), min(b, nb)
            if hi > lo:
                full[lo - na:hi - na] = logits[lo - a:hi - a]
            for wk in box["works"]:
                wk.wait()
        ty0, ty1 = own[r]
        row0, row1 = owned_rows(g, own, r)
        cls, _ = tile_stitch(full.reshape(-1, g.ntx, *full.shape[1:]), g, row0=row0, rows=row1 - row0,
                             ty0=na // g.ntx)
        if world == 1:
            return cls
        if r != 0:
            for wk in dist.batch_isend_irecv([dist.P2POp(dist.isend, cls.contiguous(), group=self.group,
                                                         group_peer=0)]):
                wk.wait()
            self.bytes_sent += cls.numel()
            return None
        # the class bands: every rank's receive posted at once straight into its rows of the output (no sequential
        # blocking receives, no concatenation copy)
        out = torch.empty(g.height, g.width, dtype=torch.uint8, device=self.device)
        r0, r1 = owned_rows(g, own, 0)
        out[r0:r1] = cls
        ops = []
        for src in range(1, world):
            lo, hi = owned_rows(g, own, src)
            if hi > lo:
                ops.append(dist.P2POp(dist.irecv, out[lo:hi], group=self.group, group_peer=src))
                self.bytes_received += (hi - lo) * g.width
        for wk in dist.batch_isend_irecv(ops) if ops else []:
            wk.wait()
        return out

    # ------------------------------------------------------------ API worker group (leader + followers)
    def serve_follower(self) -> int:
        """Non-zero ranks of a land-cover worker group: segment every mosaic the leader broadcasts
        until it calls :meth:`stop`. Returns the number of mosaics served."""
        n = 0
        while True:
            shape = torch.zeros(3, dtype=torch.int64, device=self.device)
            dist.broadcast(shape, group_src=0, group=self.group)
            if int(shape[0]) < 0:
                return n
            self._run_follower(tuple(int(v) for v in shape.tolist()))
            n += 1

    def _run_follower(self, shape) -> None:
        # same P2P sequence as run() on a non-zero rank, after the shape broadcast
        self._scatter_and_segment(None, shape)

    def stop(self) -> None:
        if self.world > 1 and self.rank == 0:
            dist.broadcast(torch.full((3,), -1, dtype=torch.int64, device=self.device), group_src=0, group=self.group)
