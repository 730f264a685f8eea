"""HIP-graph capture of whole servables that used to run eagerly: the land-cover segmenter (tiling, U-Net tile
batches, stitch, histogram — no host sync left) replayed from a graph equals its eager run."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, scope="module")
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from aiforearth_api_platform_amd import _build
    from aiforearth_api_platform_amd.ops import _ext
    _build.build_kernels()
    _ext.lib()


def test_landcover_servable_graph_replay_matches_eager():
    from aiforearth_api_platform_amd.models import zoo
    s = zoo.landcover("cuda", height=1000, width=900, tile=256, stride=224, tile_batch=8)
    x = torch.randint(0, 256, (1, 1000, 900, 4), dtype=torch.uint8, device="cuda")
    ref_cls, ref_hist = (t.clone() for t in s(x))
    static_in = x.clone()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        s(static_in)
    torch.cuda.current_stream().wait_stream(st)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cls, hist = s(static_in)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(cls, ref_cls) and torch.equal(hist, ref_hist)
    assert int(hist.sum()) == 1000 * 900
    y = torch.randint(0, 256, (1, 1000, 900, 4), dtype=torch.uint8, device="cuda")
    static_in.copy_(y)
    g.replay()
    want_cls, want_hist = s(y)
    torch.cuda.synchronize()
    assert torch.equal(cls, want_cls) and torch.equal(hist, want_hist)


def test_spatial_tile_graphs_match_eager():
    """The spatial group form runs each U-Net tile batch through a per-shape HIP graph (full batches and the
    ragged last one): the class map equals the eager segmenter's."""
    from aiforearth_api_platform_amd.models.unet import FusedUNet, unet_landcover
    from aiforearth_api_platform_amd.ops.stitch import TileGrid
    from aiforearth_api_platform_amd.runtime.spatial import SpatialSegmenter
    f = FusedUNet(unet_landcover(seed=2), device="cuda")
    grid = TileGrid(700, 600, 256, 224)  # 3 x 3 tiles: batches of 4 + a ragged 1
    eager = SpatialSegmenter(f.forward_u8, grid, 7, torch.device("cuda"), tile_batch=4)
    graphed = SpatialSegmenter(f.forward_u8, grid, 7, torch.device("cuda"), tile_batch=4, tile_graphs=True)
    assert graphed._graphed
    for seed in (0, 1):
        m = torch.randint(0, 256, (700, 600, 4), dtype=torch.uint8, generator=torch.Generator().manual_seed(seed))
        a = eager.run(m)
        b = graphed.run(m)
        torch.cuda.synchronize()
        assert torch.equal(a, b)
