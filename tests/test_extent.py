"""Land-cover extent operations (runtime/extent.py): classifybyextent / tilebyextent over a registered mosaic
equal the matching window of the full-mosaic classify (same tile grid), on CPU — directly and through the
worker pool + gateway (a sync route, JSON extents in pixel and geo coordinates)."""
import asyncio
import base64
import io
import json

import numpy as np
import pytest
import torch
from PIL import Image

from aiforearth_api_platform_amd.models import zoo
from aiforearth_api_platform_amd.runtime.decode import PayloadError
from aiforearth_api_platform_amd.runtime.extent import (OP_CLASSIFY, OP_TILE, ExtentSegmenter, GeoTransform, MosaicSpec,
                                                        encode_request, synthetic_mosaic, tile_window)
from aiforearth_api_platform_amd.ops.stitch import TileGrid

H, W, TS, ST, NC = 200, 180, 64, 56, 5
GT = [500000.0, 2.0, 0.0, 4200000.0, 0.0, -2.0]  # 2 m pixels, north-up (dy < 0)
MOSAICS = {"tileA": {"height": H, "width": W, "seed": 3, "geotransform": GT}}
KW = dict(tile=TS, stride=ST, n_classes=NC, unet_width=32, tile_batch=8)


@pytest.fixture(scope="module")
def full_map():
    seg = zoo.landcover("cpu", height=H, width=W, **KW)
    mosaic = synthetic_mosaic(H, W, 4, 3, "cpu")
    cls, _ = seg(mosaic[None])
    return cls[0].numpy()


def _rec(body, op=OP_CLASSIFY, max_hw=(256, 256)):
    return encode_request(json.dumps(body).encode(), MosaicSpec.parse(MOSAICS), op, max_hw, TS, ST).view(np.int32)


def test_geotransform_and_records():
    gt = GeoTransform.of(GT)
    assert gt.to_pixel(500000.0 + 2 * 10, 4200000.0 - 2 * 7) == (10.0, 7.0)
    r = _rec({"extent": {"xmin": 10, "ymin": 20, "xmax": 70, "ymax": 41}})
    assert tuple(r[1:6]) == (0, 10, 20, 70, 41)
    g = _rec({"mosaic": "tileA", "crs": "geo", "extent": {"xmin": GT[0] + 20, "xmax": GT[0] + 140,
                                                          "ymin": GT[3] - 82, "ymax": GT[3] - 40}})
    assert tuple(g[2:6]) == (10, 20, 70, 41)
    t = _rec({"extent": {"xmin": 10, "ymin": 20, "xmax": 70, "ymax": 41}}, op=OP_TILE)
    grid = TileGrid(H, W, TS, ST)
    ty0, ty1, tx0, tx1 = tile_window(grid, 10, 20, 70, 41)
    assert tuple(t[2:6]) == (tx0 * ST, ty0 * ST, min(W, (tx1 - 1) * ST + TS), min(H, (ty1 - 1) * ST + TS))
    assert t[2] % ST == 0 and t[3] % ST == 0
    with pytest.raises(PayloadError):
        _rec({"mosaic": "nope", "extent": {"xmin": 0, "ymin": 0, "xmax": 5, "ymax": 5}})
    with pytest.raises(PayloadError):
        _rec({"extent": {"xmin": 500, "ymin": 0, "xmax": 600, "ymax": 5}})  # outside the mosaic
    with pytest.raises(PayloadError) as e:
        _rec({"extent": {"xmin": 0, "ymin": 0, "xmax": 150, "ymax": 150}}, max_hw=(100, 100))
    assert e.value.status == 413


@pytest.mark.parametrize("box", [(0, 0, 180, 200), (10, 20, 70, 41), (55, 50, 130, 170), (150, 160, 180, 200),
                                 (0, 111, 57, 113)])
def test_extent_equals_window_of_full_classify(full_map, box):
    from aiforearth_api_platform_amd.models.unet import FusedUNet, unet_landcover

    f = FusedUNet(unet_landcover(n_classes=NC, seed=0, width=32), device="cpu")
    seg = ExtentSegmenter(f.forward_u8, MosaicSpec.parse(MOSAICS), TS, ST, f.n_classes, "cpu", tile_batch=8)
    x0, y0, x1, y1 = box
    cls, win = seg(np.array([0, 0, x0, y0, x1, y1], np.int32))
    assert win == (x0, y0, x1 - x0, y1 - y0)
    assert np.array_equal(cls.numpy(), full_map[y0:y1, x0:x1])


def _png(b64):
    return np.asarray(Image.open(io.BytesIO(base64.b64decode(b64))))


def test_extent_routes_through_pool_and_gateway(full_map):
    from aiohttp.test_utils import TestClient, TestServer

    from aiforearth_api_platform_amd.config import Config
    from aiforearth_api_platform_amd.gateway.control import ControlPlane
    from aiforearth_api_platform_amd.gateway.server import Gateway, Route, RouteTable
    from aiforearth_api_platform_amd.runtime.extent import request_decoder
    from aiforearth_api_platform_amd.runtime.model_endpoint import ModelEndpoint
    from aiforearth_api_platform_amd.runtime.worker_pool import ModelSpec, WorkerPool

    cp = ControlPlane(Config.load(env={}))
    specs = MosaicSpec.parse(MOSAICS)
    kwargs = dict(KW, mosaics=MOSAICS, max_extent=(256, 256))
    eps, pools = {}, []
    table = RouteTable()
    for name, op in (("classifybyextent", OP_CLASSIFY), ("tilebyextent", OP_TILE)):
        path = f"/v2/landcover/{name}"
        spec = ModelSpec("aiforearth_api_platform_amd.models.zoo:landcover_extent", (64,), 2, 5, kwargs, False)
        pool = WorkerPool(cp, "http://127.0.0.1" + path, spec, ["cpu"], heartbeat_interval_s=0.2,
                          max_delay_s=0.01).start(wait_ready_s=300)
        pools.append(pool)
        ep = ModelEndpoint(cp, path, worker=pool, decode=request_decoder(specs, op, (256, 256), TS, ST))
        table.add(Route(path, "sync", ep))
        table.add(Route(path + "-async", "async", ep))
    gw = Gateway(cp, table)

    async def go():
        c = TestClient(TestServer(gw.app))
        await c.start_server()
        try:
            out = {}
            body = {"mosaic": "tileA", "extent": {"xmin": 33, "ymin": 61, "xmax": 120, "ymax": 150}}
            r = await c.post("/v2/landcover/classifybyextent", json=body)
            assert r.status == 200, await r.text()
            out["classify"] = await r.json()
            geo = {"mosaic": "tileA", "crs": "geo",
                   "extent": {"xmin": GT[0] + 2 * 33, "xmax": GT[0] + 2 * 120, "ymin": GT[3] - 2 * 150,
                              "ymax": GT[3] - 2 * 61}}
            r = await c.post("/v2/landcover/classifybyextent", json=geo)
            out["geo"] = await r.json()
            r = await c.post("/v2/landcover/tilebyextent", json=body)
            out["tile"] = await r.json()
            r = await c.post("/v2/landcover/classifybyextent", json={"extent": {"xmin": 0, "ymin": 0}})
            out["bad"] = r.status
            r = await c.post("/v2/landcover/classifybyextent", data=b"\x00" * 64,
                             headers={"Content-Type": "image/png"})
            out["badtype"] = r.status
            # NaN / Infinity (json.loads accepts them), a non-object body, a geo extent past float range: 400
            hj = {"Content-Type": "application/json"}
            out["odd"] = [(await c.post("/v2/landcover/classifybyextent", data=b, headers=hj)).status for b in (
                b'{"extent": {"xmin": NaN, "ymin": 0, "xmax": 5, "ymax": 5}}',
                b'{"extent": {"xmin": 0, "ymin": -Infinity, "xmax": 5, "ymax": 5}}',
                b'[1, 2, 3]', b'"text"',
                b'{"crs": "geo", "extent": {"xmin": 1e308, "ymin": 0, "xmax": 1.7e308, "ymax": 5}}')]
            # raw 64-byte records must not reach the workers: binary batch ingest is refused
            r = await c.post("/v2/landcover/classifybyextent-async", data=b"\x00" * 128,
                             headers={"Content-Type": "application/x-ai4e-batch"})
            out["batch"] = r.status
            return out
        finally:
            await c.close()

    try:
        out = asyncio.new_event_loop().run_until_complete(go())
    finally:
        for p in pools:
            p.stop()
        cp.close()
    cl = out["classify"]
    assert cl["window"] == {"x0": 33, "y0": 61, "width": 87, "height": 89}
    assert np.array_equal(_png(cl["class_map"]), full_map[61:150, 33:120])
    assert cl["histogram"] == np.bincount(full_map[61:150, 33:120].reshape(-1), minlength=NC)[:NC].tolist()
    assert out["geo"]["window"] == cl["window"] and out["geo"]["class_map"] == cl["class_map"]
    tw = out["tile"]["window"]
    assert tw["x0"] % ST == 0 and tw["y0"] % ST == 0 and tw["x0"] <= 33 and tw["y0"] <= 61
    assert tw["x0"] + tw["width"] >= 120 and tw["y0"] + tw["height"] >= 150
    assert np.array_equal(_png(out["tile"]["class_map"]),
                          full_map[tw["y0"]:tw["y0"] + tw["height"], tw["x0"]:tw["x0"] + tw["width"]])
    assert out["bad"] == 400 and out["badtype"] == 415
    assert out["odd"] == [400] * 5, out["odd"]
    assert out["batch"] == 415


def test_extent_servable_refuses_bad_records_per_item():
    """A record that did not come through encode_request (bad window / mosaic index) is marked invalid on its own
    (invalid_rows -> IT_INVALID in the worker); the other requests of the batch are served."""
    from aiforearth_api_platform_amd.models.unet import FusedUNet, unet_landcover
    from aiforearth_api_platform_amd.runtime.extent import _MAGIC, ExtentServable

    f = FusedUNet(unet_landcover(n_classes=NC, seed=0, width=32), device="cpu")
    seg = ExtentSegmenter(f.forward_u8, MosaicSpec.parse(MOSAICS), TS, ST, f.n_classes, "cpu", tile_batch=8)
    sv = ExtentServable(seg, (64, 64), NC)
    good = _rec({"extent": {"xmin": 10, "ymin": 20, "xmax": 40, "ymax": 41}}, max_hw=(64, 64))
    recs = np.stack([good, good.copy(), good.copy(), np.zeros(16, np.int32)])
    recs[1, 4] = W + 500                     # window past the mosaic
    recs[2, 1] = 7                           # no such mosaic
    canvas, win, hist = sv(torch.from_numpy(recs.view(np.uint8)))
    bad = ExtentServable.invalid_rows([canvas, win, hist])
    assert bad.tolist() == [False, True, True, False]  # (row 3: padding without the magic)
    assert int(recs[0, 0]) == _MAGIC and tuple(win[0].tolist()) == (10, 20, 30, 21)
