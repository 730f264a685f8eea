"""Spatial-parallel segmentation over gloo (2, 3 and 8 CPU ranks) == single-process result; the tile split is
balanced to one tile and every rank receives only its band of the mosaic."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from aiforearth_api_platform_amd.ops.stitch import TileGrid
from aiforearth_api_platform_amd.runtime.spatial import SpatialSegmenter, owned_rows, split_tile_rows


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    from aiforearth_api_platform_amd.models.unet import FusedUNet, unet_landcover
    f = FusedUNet(unet_landcover(n_classes=5, seed=1, width=32))
    return lambda t: f(t).float()


GRID = TileGrid(120, 100, 32, 24)
GRID9 = TileGrid(216, 100, 32, 24)  # 9 tile rows x 4: the 4096^2 / 512 / 448 row count, at world 8


def _worker(rank, world, port, mosaic, q, grid=GRID):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    seg = SpatialSegmenter(_model(), grid, 5, torch.device("cpu"), tile_batch=8)
    out = seg.run(mosaic if rank == 0 else None)
    q.put((rank, out, seg.bytes_received))
    dist.barrier()
    dist.destroy_process_group()


def test_split_and_ownership():
    r = split_tile_rows(9, 8)
    assert r[0] == (0, 2) and r[-1] == (8, 9) and sum(b - a for a, b in r) == 9
    g = TileGrid(4096, 4096, 512, 448)
    rows = [owned_rows(g, split_tile_rows(g.nty, 8), i) for i in range(8)]
    assert rows[0][0] == 0 and rows[-1][1] == 4096
    assert all(rows[i][1] == rows[i + 1][0] for i in range(7))
    # compute is split by tiles: 81 tiles over 8 ranks -> 10 or 11 each (whole rows gave 2:1)
    seg = SpatialSegmenter(lambda t: t, g, 7, torch.device("cpu"))
    seg.world = 8
    comp, own, need, bands = seg._plan()
    sizes = [b - a for a, b in comp]
    assert sum(sizes) == 81 and max(sizes) - min(sizes) <= 1
    assert all(comp[i][1] == comp[i + 1][0] for i in range(7))
    # each rank's mosaic band covers its tiles and is far smaller than the mosaic
    for (a, b), (y0, y1) in zip(comp, bands):
        assert y0 == a // g.ntx * g.stride and y1 == (b - 1) // g.ntx * g.stride + g.ts
        assert y1 - y0 <= 2 * g.stride + g.ts - g.stride + g.ts


@pytest.mark.parametrize("world", [2, 3, 8])
def test_spatial_matches_single_process(world):
    grid = GRID9 if world == 8 else GRID
    torch.manual_seed(0)
    mosaic = torch.randint(0, 256, (grid.height, grid.width, 4), dtype=torch.uint8)
    single = SpatialSegmenter(_model(), grid, 5, torch.device("cpu"), tile_batch=8).run(mosaic)
    assert single.shape == (grid.height, grid.width)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mosaic, q, grid)) for r in range(world)]
    [p.start() for p in procs]
    res = {}
    for _ in range(world):
        r, out, nbytes = q.get(timeout=240)
        res[r] = (out, nbytes)
    [p.join(60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    assert torch.equal(res[0][0], single)
    # followers got a band of the mosaic + halo logits, not the whole mosaic
    mosaic_bytes = mosaic.numel()
    for r in range(1, world):
        assert res[r][0] is None
    if world == 8:
        ts_bytes = grid.ts * grid.ts * 5 * 4  # one fp32 logits tile
        for r in range(1, world):
            band_bytes = res[r][1] - (res[r][1] // ts_bytes) * ts_bytes
            assert band_bytes < mosaic_bytes // 2, (r, band_bytes, mosaic_bytes)
