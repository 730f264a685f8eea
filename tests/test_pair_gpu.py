"""K1p fused 1x1 pair (csrc/kernels/conv_pair.hip): block i's c3 + residual + ReLU and block i+1's c1 in
one launch, vs a PyTorch fp32 reference of the two convs (GPU box only). Y is rounded to bf16 before the
chained 1x1, where the kernel rounds it (the Y chunk in LDS)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from aiforearth_api_platform_amd.ops import _ext
from aiforearth_api_platform_amd.ops.conv import conv_pair, pack_conv, pair_supported

DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _ext.lib()


def _w(pc):
    return pc.w_packed[:pc.cout, :pc.cin_pad].float()


CASES = [
    # n, h, w, mid, tile[, midn]
    (2, 14, 14, 256, 0),      # layer3 shape, M = 392 (partial last tile)
    (2, 14, 14, 256, 0, 512),  # last layer3 block -> layer4's 512-wide c1
    (1, 5, 7, 256, 64, 512),
    (2, 28, 28, 128, 0, 256),  # last layer2 block -> layer3's first c1
    (1, 5, 9, 128, 64, 256),
    (2, 14, 14, 256, 64),
    (1, 5, 7, 256, 0),        # M = 35 < one tile
    (8, 14, 14, 256, 96),     # M = 1568: 17 tiles
    (8, 14, 14, 256, 98),     # loads + stores spread over the C phase
    (1, 5, 7, 256, 98),       # ... with a partial tile
    (2, 7, 7, 512, 0),        # layer4 shape
    (1, 3, 5, 512, 32),
    (2, 14, 14, 256, 98, 512),  # spread variant of the other shapes
    (1, 5, 7, 256, 98, 512),
    (2, 28, 28, 128, 98, 256),
    (1, 5, 9, 128, 98, 256),
    (2, 7, 7, 512, 98),
    (1, 3, 5, 512, 98),
    (8, 14, 14, 256, 99),     # 16-B Y writes (fragment pairs swapped with v_permlane16_swap)
    (1, 5, 7, 256, 99),       # ... with a partial tile
]


def test_conv_pair_yw_bit_identical():
    """bm_cfg 99 (16-B Y writes, the default) computes the same bits as the 8-B-write schedule (98)."""
    torch.manual_seed(12)
    c3 = pack_conv(torch.randn(1024, 256, 1, 1) / 16, torch.randn(1024) * 0.1).to(DEV)
    c1n = pack_conv(torch.randn(256, 1024, 1, 1) / 32, torch.randn(256) * 0.1).to(DEV)
    t2 = torch.randn(9, 14, 14, 256, device=DEV).relu().to(torch.bfloat16)
    res = torch.randn(9, 14, 14, 1024, device=DEV).to(torch.bfloat16)
    a = conv_pair(t2, c3, res, c1n, tile_cfg=98)
    b = conv_pair(t2, c3, res, c1n, tile_cfg=99)
    torch.cuda.synchronize()
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("case", CASES)
def test_conv_pair(case):
    n, h, w, mid, tile = case[:5]
    midn = case[5] if len(case) > 5 else mid
    c4 = 4 * mid
    assert pair_supported(mid, c4, midn)
    torch.manual_seed(11)
    c3 = pack_conv(torch.randn(c4, mid, 1, 1) / mid ** 0.5, torch.randn(c4) * 0.1).to(DEV)
    c1n = pack_conv(torch.randn(midn, c4, 1, 1) / c4 ** 0.5, torch.randn(midn) * 0.1).to(DEV)
    t2 = torch.randn(n, h, w, mid, device=DEV).relu().to(torch.bfloat16)
    res = torch.randn(n, h, w, c4, device=DEV).to(torch.bfloat16)
    y, t1n = conv_pair(t2, c3, res, c1n, tile_cfg=tile)
    torch.cuda.synchronize()
    y_ref = (t2.float().reshape(-1, mid) @ _w(c3).t() + c3.b_ref.to(DEV) + res.float().reshape(-1, c4)).relu()
    t_ref = (y_ref.to(torch.bfloat16).float() @ _w(c1n).t() + c1n.b_ref.to(DEV)).relu()
    y_err = (y.float().reshape(-1, c4) - y_ref).abs().max().item()
    t_err = (t1n.float().reshape(-1, midn) - t_ref).abs().max().item()
    assert y_err <= 0.02 * y_ref.abs().max().item() + 1e-2, y_err
    assert t_err <= 0.02 * t_ref.abs().max().item() + 1e-2, t_err


def test_conv_pair_in_resnet_layer3_matches_unfused(monkeypatch):
    """The fused forward with K1p in layer3 equals the same forward with the pair split into two K1 convs."""
    from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50
    from aiforearth_api_platform_amd.ops import conv as convmod

    torch.manual_seed(0)
    fused = FusedResNet(resnet50(), device=DEV)
    x = torch.randint(0, 256, (4, 224, 224, 3), dtype=torch.uint8, device=DEV)
    with torch.no_grad():
        monkeypatch.setattr(convmod, "PAIR", True)
        a = fused.forward_u8(x)
        monkeypatch.setattr(convmod, "PAIR", False)
        b = fused.forward_u8(x)
    torch.cuda.synchronize()
    assert (a - b).abs().max().item() <= 0.05 * b.abs().max().item() + 1e-2


def test_side_stream_downsample_matches_serial():
    """Stage-entry downsample forked onto a side stream (captured in a HIP graph) == the serial forward."""
    from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50

    torch.manual_seed(0)
    fused = FusedResNet(resnet50(), device=DEV)
    x = torch.randint(0, 256, (8, 224, 224, 3), dtype=torch.uint8, device=DEV)
    with torch.no_grad():
        fused.par_down = False
        ref = fused.forward_u8(x)
        fused.par_down = True
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fused.forward_u8(x)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                out = fused.forward_u8(x)
        g.replay()
        torch.cuda.synchronize()
    assert torch.equal(out, ref)


