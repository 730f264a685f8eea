"""Land-cover extent operations on the GPU: the HIP U-Net + K6 stitch over a resident mosaic; the window's class
map equals the same window of the full-mosaic classify (same tile grid, same kernels)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from aiforearth_api_platform_amd.models import zoo
from aiforearth_api_platform_amd.runtime.extent import ExtentSegmenter, MosaicSpec, synthetic_mosaic

H, W, TS, ST, NC = 1000, 900, 256, 224, 7
MOSAICS = {"m": {"height": H, "width": W, "seed": 5}}


@pytest.fixture(scope="module")
def setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from aiforearth_api_platform_amd.ops import _ext
    from aiforearth_api_platform_amd.models.unet import FusedUNet, unet_landcover

    _ext.lib()
    full = zoo.landcover("cuda", height=H, width=W, tile=TS, stride=ST, n_classes=NC, tile_batch=8)
    cls, _ = full(synthetic_mosaic(H, W, 4, 5, "cuda")[None])
    f = FusedUNet(unet_landcover(n_classes=NC, seed=0), device="cuda")
    seg = ExtentSegmenter(f.forward_u8, MosaicSpec.parse(MOSAICS), TS, ST, f.n_classes, "cuda", tile_batch=8)
    return cls[0].cpu().numpy(), seg


@pytest.mark.parametrize("box", [(0, 0, 900, 1000), (100, 200, 400, 451), (640, 700, 900, 1000), (223, 223, 226, 226)])
def test_extent_equals_full_window_gpu(setup, box):
    full, seg = setup
    x0, y0, x1, y1 = box
    cls, win = seg(np.array([0, 0, x0, y0, x1, y1], np.int32))
    torch.cuda.synchronize()
    assert win == (x0, y0, x1 - x0, y1 - y0)
    assert np.array_equal(cls.cpu().numpy(), full[y0:y1, x0:x1])
