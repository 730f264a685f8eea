"""BASELINE config #4: land-cover U-Net on a tiled 4096x4096 RGB+NIR mosaic, spatial-parallel over GPUs.

All ranks segment ONE mosaic together (tile rows split across ranks, halo exchange of boundary tile
logits over RCCL P2P, per-rank stitch, bands gathered on rank 0). Reports mosaics/s, Mpx/s, tiles/s.

    python bench/landcover_bench.py [--size 4096 --tile 512 --stride 448 --tile-batch 16]
"""
import argparse

import torch

from common import Dist, build_once, timed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--tile", type=int, default=512)
    ap.add_argument("--stride", type=int, default=448)
    ap.add_argument("--tile-batch", type=int, default=16)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    d = Dist()
    build_once(d)
    from aiforearth_api_platform_amd.models.unet import FusedUNet, unet_landcover
    from aiforearth_api_platform_amd.ops.stitch import TileGrid
    from aiforearth_api_platform_amd.runtime.spatial import SpatialSegmenter
    f = FusedUNet(unet_landcover(seed=0), device=d.device)
    grid = TileGrid(a.size, a.size, a.tile, a.stride)
    seg = SpatialSegmenter(f.forward_u8, grid, f.n_classes, d.device, tile_batch=a.tile_batch)
    mosaic = torch.randint(0, 256, (a.size, a.size, 4), dtype=torch.uint8, device=d.device) if d.rank == 0 else None
    dt = timed(lambda: seg.run(mosaic), a.steps, a.warmup, d.sync)
    (dt,) = d.max(dt)
    per = dt / a.steps
    ntiles = grid.nty * grid.ntx
    d.emit({"metric": "land-cover mosaics/sec (whole node)", "value": round(1 / per, 4), "unit": "mosaics/s",
            "n_gpus": d.world, "ms_per_mosaic": round(per * 1e3, 2), "mpx_per_s": round(a.size * a.size / per / 1e6, 2),
            "tiles_per_s": round(ntiles / per, 2), "dtype": "bf16", "data": "synthetic uint8 RGB+NIR, random-init",
            "config": {"model": "unet_landcover", "mosaic": a.size, "tile": a.tile, "stride": a.stride,
                       "tiles": ntiles, "parallelism": f"spatial{d.world}"}}, a.json_out)
    d.close()


if __name__ == "__main__":
    main()
