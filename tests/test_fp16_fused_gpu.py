"""fp16 instantiations of the fused kernels (f16 MFMA, fp32 accumulation) — the ensemble's crop classifier runs
the same fused graph as the bf16 headline model (BASELINE config 5): K1c bottleneck chains
(``ai4e_conv_chain_f16_fwd``), the K1p layer3 pair (``ai4e_conv_pair_f16_fwd``) and K1s with the fused first c1
(``ai4e_stem_pool_c1_f16_fwd``), each against a plain fp32 PyTorch reference of the same ops with the
intermediates rounded to fp16 where the kernel rounds them. fp16 keeps 10 mantissa bits: the bound is 8x
tighter than the bf16 tests' 0.02."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
TOL = 0.0025


@pytest.fixture(autouse=True, scope="module")
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from aiforearth_api_platform_amd.ops import _ext
    _ext.lib()


def _wq(pc, k):
    return pc.w_packed[:pc.cout, :k * k * pc.cin_pad].float().reshape(pc.cout, k, k, pc.cin_pad).permute(0, 3, 1, 2)


def _conv(x, w, b, stride=1, pad=0):
    return F.conv2d(x.float().permute(0, 3, 1, 2), w, b, stride=stride, padding=pad).permute(0, 2, 3, 1)


def _close(got, ref):
    err = (got.float() - ref).abs().max().item()
    assert err <= TOL * ref.abs().max().item() + TOL, err


CHAIN_CASES = [
    # n, h, w, mid, stride, next (True = same width, or the chained 1x1's output width)
    (2, 56, 56, 64, 1, True),
    (2, 56, 56, 64, 1, 128),     # layer1 -> layer2
    (2, 56, 56, 64, 1, False),
    (1, 15, 13, 64, 1, True),    # partial tile
    (2, 28, 28, 128, 1, True),
    (2, 28, 28, 128, 1, False),
    (2, 56, 56, 128, 2, True),   # strided c2: the LDS-DMA ring phase A
    (3, 12, 4, 128, 1, True),    # patch mode, tiles straddle images
]


@pytest.mark.parametrize("case", CHAIN_CASES)
def test_conv_chain_f16(case):
    from aiforearth_api_platform_amd.ops import _ext
    from aiforearth_api_platform_amd.ops.conv import conv_chain, pack_conv

    n, h, w, mid, s, nxt = case
    midn = 0 if not nxt else (mid if nxt is True else nxt)
    torch.manual_seed(7)
    c2 = pack_conv(torch.randn(mid, mid, 3, 3) / (9 * mid) ** 0.5, torch.randn(mid) * 0.1, stride=s, pad=1).to(DEV)
    c3 = pack_conv(torch.randn(4 * mid, mid, 1, 1) / mid ** 0.5, torch.randn(4 * mid) * 0.1).to(DEV)
    c1n = pack_conv(torch.randn(midn, 4 * mid, 1, 1) / (4 * mid) ** 0.5, torch.randn(midn) * 0.1).to(DEV) if nxt else None
    c2, c3 = c2.cast(torch.float16), c3.cast(torch.float16)
    c1n = c1n.cast(torch.float16) if c1n is not None else None
    t1 = torch.randn(n, h, w, mid, device=DEV).relu().half()
    oh, ow = c2.out_hw(h, w)
    res = torch.randn(n, oh, ow, 4 * mid, device=DEV).half()
    calls = []
    orig = _ext.call
    try:
        _ext.call = lambda name, *a: (calls.append(name), orig(name, *a))[1]
        y, t1n = conv_chain(t1, c2, c3, res, c1n=c1n)
    finally:
        _ext.call = orig
    torch.cuda.synchronize()
    assert calls == ["ai4e_conv_chain_f16_fwd"] and y.dtype == torch.float16
    t2 = F.relu(_conv(t1, _wq(c2, 3), c2.bias[:mid], s, 1)).half()
    yr = F.relu(_conv(t2, _wq(c3, 1), c3.bias[:4 * mid]) + res.float())
    _close(y, yr)
    if nxt:
        _close(t1n, F.relu(_conv(y, _wq(c1n, 1), c1n.bias[:midn])))


def test_conv_chain_down_f16():
    from aiforearth_api_platform_amd.ops.conv import conv_chain, pack_conv

    n, h, w, mid = 2, 56, 56, 64
    torch.manual_seed(9)
    c2 = pack_conv(torch.randn(mid, mid, 3, 3) / (9 * mid) ** 0.5, torch.randn(mid) * 0.1, pad=1).to(DEV).cast(torch.float16)
    c3 = pack_conv(torch.randn(4 * mid, mid, 1, 1) / mid ** 0.5, torch.randn(4 * mid) * 0.1).to(DEV).cast(torch.float16)
    dn = pack_conv(torch.randn(4 * mid, 64, 1, 1) / 8, torch.randn(4 * mid) * 0.1).to(DEV).cast(torch.float16)
    c1n = pack_conv(torch.randn(mid, 4 * mid, 1, 1) / (4 * mid) ** 0.5, torch.randn(mid) * 0.1).to(DEV).cast(torch.float16)
    t1 = torch.randn(n, h, w, mid, device=DEV).relu().half()
    x0 = torch.randn(n, h, w, 64, device=DEV).relu().half()
    y, t1n = conv_chain(t1, c2, c3, None, c1n=c1n, down=dn, x0=x0)
    torch.cuda.synchronize()
    t2 = F.relu(_conv(t1, _wq(c2, 3), c2.bias[:mid], 1, 1)).half()
    yr = F.relu(_conv(t2, _wq(c3, 1), c3.bias[:4 * mid]) + _conv(x0, _wq(dn, 1), dn.bias[:4 * mid]))
    _close(y, yr)
    _close(t1n, F.relu(_conv(y, _wq(c1n, 1), c1n.bias[:mid])))


@pytest.mark.parametrize("n,h,w", [(4, 14, 14), (3, 13, 11)])
def test_conv_pair_f16(n, h, w):
    from aiforearth_api_platform_amd.ops.conv import conv_pair, pack_conv

    torch.manual_seed(3)
    mid, c4, midn = 256, 1024, 256
    c3 = pack_conv(torch.randn(c4, mid, 1, 1) / mid ** 0.5, torch.randn(c4) * 0.1).to(DEV).cast(torch.float16)
    c1n = pack_conv(torch.randn(midn, c4, 1, 1) / c4 ** 0.5, torch.randn(midn) * 0.1).to(DEV).cast(torch.float16)
    t2 = torch.randn(n, h, w, mid, device=DEV).relu().half()
    res = torch.randn(n, h, w, c4, device=DEV).half()
    y, t1n = conv_pair(t2, c3, res, c1n)
    torch.cuda.synchronize()
    yr = F.relu(_conv(t2, _wq(c3, 1), c3.bias[:c4]) + res.float())
    _close(y, yr)
    _close(t1n, F.relu(_conv(y, _wq(c1n, 1), c1n.bias[:midn])))


@pytest.mark.parametrize("shape", [(3, 112, 112), (2, 31, 25)])
def test_stem_pool_c1_f16(shape):
    from aiforearth_api_platform_amd.ops.conv import pack_conv, pack_stem_s2d, stem_pool_c1

    n, h, w = shape
    torch.manual_seed(8)
    pc = pack_stem_s2d(torch.randn(64, 3, 7, 7) / 12, torch.randn(64) * 0.1).to(DEV).cast(torch.float16)
    c1 = pack_conv(torch.randn(64, 64, 1, 1) / 8, torch.randn(64) * 0.1).to(DEV).cast(torch.float16)
    x = torch.randn(n, h, w, 16, device=DEV).half()
    y, t1 = stem_pool_c1(x, pc, c1)
    torch.cuda.synchronize()
    assert y.dtype == torch.float16 and t1.dtype == torch.float16
    xp = F.pad(x.float().permute(0, 3, 1, 2), (1, 2, 1, 2))
    conv = F.relu(F.conv2d(xp, _wq(pc, 4), pc.bias[:64])).half().float()
    yr = F.max_pool2d(conv, 3, 2, 1).permute(0, 2, 3, 1)
    _close(y, yr)
    _close(t1, F.relu(_conv(y, _wq(c1, 1), c1.bias[:64])))


def test_resnet50_fp16_runs_the_fused_kernels():
    """The fp16 crop classifier's forward dispatches K1s + c1, the K1c chains and the K1p pairs in their f16 forms."""
    from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50
    from aiforearth_api_platform_amd.ops import _ext

    m = FusedResNet(resnet50(num_classes=200, seed=4), device=DEV, dtype=torch.float16)
    img = torch.randint(0, 256, (8, 224, 224, 3), dtype=torch.uint8, device=DEV)
    calls = []
    orig = _ext.call
    try:
        _ext.call = lambda name, *a: (calls.append(name), orig(name, *a))[1]
        out = m.forward_u8(img)
    finally:
        _ext.call = orig
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    assert calls.count("ai4e_stem_pool_c1_f16_fwd") == 1
    assert calls.count("ai4e_conv_chain_f16_fwd") == 7   # layer1 (3) + layer2 (4)
    assert calls.count("ai4e_conv_pair_f16_fwd") == 5    # the layer3 c3 + residual + next c1 pairs
    assert "ai4e_conv_chain_fwd" not in calls and "ai4e_conv_pair_fwd" not in calls
