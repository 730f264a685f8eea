"""Spatial-parallel segmentation over gloo (2 and 3 CPU ranks) == single-process result."""
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


def _worker(rank, world, port, mosaic, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    seg = SpatialSegmenter(_model(), GRID, 5, torch.device("cpu"), tile_batch=8)
    out = seg.run(mosaic if rank == 0 else None)
    if rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


def test_split_and_ownership():
    r = split_tile_rows(9, 8)
    assert r[0] == (0, 2) and r[-1] == (8, 9) and sum(b - a for a, b in r) == 9
    g = TileGrid(4096, 4096, 512, 448)
    rows = [owned_rows(g, split_tile_rows(g.nty, 8), i) for i in range(8)]
    assert rows[0][0] == 0 and rows[-1][1] == 4096
    assert all(rows[i][1] == rows[i + 1][0] for i in range(7))


@pytest.mark.parametrize("world", [2, 3])
def test_spatial_matches_single_process(world):
    torch.manual_seed(0)
    mosaic = torch.randint(0, 256, (120, 100, 4), dtype=torch.uint8)
    single = SpatialSegmenter(_model(), GRID, 5, torch.device("cpu"), tile_batch=8).run(mosaic)
    assert single.shape == (120, 100)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mosaic, q)) for r in range(world)]
    [p.start() for p in procs]
    out = q.get(timeout=120)
    [p.join(60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    assert torch.equal(out, single)
