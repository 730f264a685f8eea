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
    q.put((rank, None if out is None else out.numpy().copy(), seg.bytes_received))
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
        res[r] = (None if out is None else torch.from_numpy(out), nbytes)
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


def _delayed_worker(rank, world, port, mosaic, q, grid, delay_rank):
    """A rank whose tiles run slowly (the delayed peer); every rank records its event order."""
    import time as _t

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    base = _model()

    def slow(t):
        if rank == delay_rank:
            _t.sleep(0.15)
        return base(t)

    seg = SpatialSegmenter(slow, grid, 5, torch.device("cpu"), tile_batch=2)
    out = seg.run(mosaic if rank == 0 else None)
    q.put((rank, None if out is None else out.numpy().copy(), list(seg.events)))
    dist.barrier()
    dist.destroy_process_group()


def test_halo_posted_before_interior_tiles_finish():
    """Boundary tiles run first and the halo exchange is posted right after them: on every rank the post precedes the
    last interior tile batch (with a delayed peer the exchange is in flight while the interior tiles still run), and
    the result still equals the single-process class map."""
    grid = GRID9
    torch.manual_seed(0)
    mosaic = torch.randint(0, 256, (grid.height, grid.width, 4), dtype=torch.uint8)
    single = SpatialSegmenter(_model(), grid, 5, torch.device("cpu"), tile_batch=8).run(mosaic)
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_delayed_worker, args=(r, world, port, mosaic, q, grid, 1)) for r in range(world)]
    [p.start() for p in procs]
    res = {}
    for _ in range(world):
        r, out, ev = q.get(timeout=240)
        res[r] = (None if out is None else torch.from_numpy(out), ev)
    [p.join(60) for p in procs]
    assert torch.equal(res[0][0], single)
    for r, (_, ev) in res.items():
        kinds = [e[0] for e in ev]
        assert kinds.count("halo_posted") == 1, ev
        post = kinds.index("halo_posted")
        assert 0 < post < len(ev) - 1, (r, ev)  # boundary tiles before it, interior tiles after it
