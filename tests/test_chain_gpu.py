"""K1c fused bottleneck chain (csrc/kernels/conv_chain.hip) vs a PyTorch fp32 reference of the same
three convs (GPU box only). Intermediates are rounded to bf16 where the kernel rounds them (T2 in LDS,
Y before the chained 1x1)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from aiforearth_api_platform_amd.ops import _ext
from aiforearth_api_platform_amd.ops.conv import chain_kernel_builds, conv_chain, pack_conv

DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _ext.lib()


def _wq(pc, k):
    return pc.w_packed[:pc.cout, :k * k * pc.cin_pad].float().reshape(pc.cout, k, k, pc.cin_pad).permute(0, 3, 1, 2)


def _conv(x, w, b, stride=1, pad=0):
    return F.conv2d(x.float().permute(0, 3, 1, 2), w, b, stride=stride, padding=pad).permute(0, 2, 3, 1)


CASES = [
    # n, h, w, mid, stride, next (True = same width, or the chained 1x1's output width)
    (2, 56, 56, 64, 1, True),
    (2, 56, 56, 64, 1, 128),      # layer1 -> layer2 boundary
    (1, 15, 13, 64, 1, 128),
    (2, 56, 56, 64, 1, False),
    (1, 15, 13, 64, 1, True),     # M = 195: one partial tile
    (3, 9, 11, 64, 2, True),      # strided 3x3, ragged
    (2, 28, 28, 128, 1, True),
    (2, 28, 28, 128, 1, False),
    (2, 56, 56, 128, 2, True),    # layer2 block 0: strided c2 chained into block 1's c1
    (1, 9, 13, 128, 1, True),     # M = 117 < one 128-pixel tile
    (3, 12, 8, 64, 1, True),      # patch mode: tiles straddle image boundaries (96-pixel images)
    (3, 12, 4, 128, 1, True),     # patch mode, MID 128: 35-row patch, tiles straddle images
    (5, 7, 8, 64, 1, 128),        # patch mode, ragged last tile
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("tile", [0, 3])
def test_conv_chain(case, tile):
    """tile 3 = phase A from the LDS input patch (stride 1 and a patch that fits; other shapes fall back to the
    ring, which the same comparison then covers); tile 0 = the LDS-DMA ring everywhere."""
    n, h, w, mid, s, nxt = case
    midn = 0 if not nxt else (mid if nxt is True else nxt)
    assert chain_kernel_builds(mid, midn)
    torch.manual_seed(7)
    c2 = pack_conv(torch.randn(mid, mid, 3, 3) / (9 * mid) ** 0.5, torch.randn(mid) * 0.1, stride=s, pad=1).to(DEV)
    c3 = pack_conv(torch.randn(4 * mid, mid, 1, 1) / mid ** 0.5, torch.randn(4 * mid) * 0.1).to(DEV)
    c1n = pack_conv(torch.randn(midn, 4 * mid, 1, 1) / (4 * mid) ** 0.5, torch.randn(midn) * 0.1).to(DEV) if nxt else None
    t1 = torch.randn(n, h, w, mid, device=DEV).relu().to(torch.bfloat16)
    oh, ow = c2.out_hw(h, w)
    res = torch.randn(n, oh, ow, 4 * mid, device=DEV).to(torch.bfloat16)
    y, t1n = conv_chain(t1, c2, c3, res, c1n=c1n, force=True, tile_cfg=tile)
    torch.cuda.synchronize()

    t2 = F.relu(_conv(t1, _wq(c2, 3), c2.bias[:mid], s, 1)).to(torch.bfloat16)
    yr = F.relu(_conv(t2, _wq(c3, 1), c3.bias[:4 * mid]) + res.float())
    err = (y.float() - yr).abs().max().item()
    assert err <= 0.02 * yr.abs().max().item() + 0.03, err
    if nxt:
        tr = F.relu(_conv(y, _wq(c1n, 1), c1n.bias[:midn]))
        err = (t1n.float() - tr).abs().max().item()
        assert err <= 0.02 * tr.abs().max().item() + 0.03, err
    else:
        assert t1n is None


def test_resnet_chain_matches_unfused(monkeypatch):
    """FusedResNet with K1c chains == the per-conv K1 graph (same weights, same input)."""
    from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50

    torch.manual_seed(0)
    m = FusedResNet(resnet50(seed=1), device=DEV)
    img = torch.randint(0, 256, (4, 224, 224, 3), dtype=torch.uint8, device=DEV)
    m.chain = True
    a = m.forward_u8(img)
    m.chain = False
    b = m.forward_u8(img)
    torch.cuda.synchronize()
    assert (a - b).abs().max().item() <= 0.05 * b.abs().max().item() + 1e-3
    assert (a.argmax(1) == b.argmax(1)).float().mean().item() >= 0.75


@pytest.mark.parametrize("shape", [(2, 112, 112), (3, 30, 26), (1, 17, 9), (600, 16, 16)])
@pytest.mark.parametrize("variant", [0, 1])
def test_stem_pool(shape, variant):
    """K1s fused s2d stem conv + ReLU + 3x3/2 max-pool vs PyTorch fp32 (conv output rounded to bf16)."""
    from aiforearth_api_platform_amd.ops.conv import pack_stem_s2d, stem_pool

    n, h, w = shape
    torch.manual_seed(5)
    pc = pack_stem_s2d(torch.randn(64, 3, 7, 7) / 12, torch.randn(64) * 0.1).to(DEV)
    x = torch.randn(n, h, w, 16, device=DEV).to(torch.bfloat16)
    y = stem_pool(x, pc, variant=variant)
    torch.cuda.synchronize()
    xp = F.pad(x.float().permute(0, 3, 1, 2), (1, 2, 1, 2))
    conv = F.relu(F.conv2d(xp, _wq(pc, 4), pc.bias[:64])).to(torch.bfloat16).float()
    ref = F.max_pool2d(conv, 3, 2, 1).permute(0, 2, 3, 1)
    assert y.shape == ref.shape
    err = (y.float() - ref).abs().max().item()
    assert err <= 0.02 * ref.abs().max().item() + 0.02, err


@pytest.mark.parametrize("shape", [(256, 1000, 5), (3, 1000, 1), (7, 10, 10), (2, 2048, 5), (5, 1500, 3)])
def test_softmax_topk(shape):
    """Fused softmax + top-k head kernel vs torch.softmax + torch.topk on the same bf16 logits."""
    from aiforearth_api_platform_amd.ops.head import softmax_topk

    n, c, k = shape
    torch.manual_seed(11)
    logits = (torch.randn(n, c, device=DEV) * 3).to(torch.bfloat16)
    idx, prob = softmax_topk(logits, k)
    torch.cuda.synchronize()
    rp, ri = torch.topk(torch.softmax(logits.float(), 1), k, 1)
    assert idx.dtype == torch.int32 and prob.dtype == torch.float32
    assert torch.allclose(prob, rp, rtol=1e-4, atol=1e-6)
    # bf16 logits tie often: compare the probability of the chosen class, not the index
    chosen = torch.softmax(logits.float(), 1).gather(1, idx.long())
    assert torch.allclose(chosen, rp, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("shape", [(2, 56, 56), (1, 15, 13), (3, 12, 8)])
@pytest.mark.parametrize("tile", [-1, 3, 19])
def test_conv_chain_down(shape, tile):
    """K1c DOWN mode: the residual is the 1x1 projection of the block input, folded into c3's K."""
    n, h, w = shape
    mid = 64
    torch.manual_seed(9)
    c2 = pack_conv(torch.randn(mid, mid, 3, 3) / (9 * mid) ** 0.5, torch.randn(mid) * 0.1, pad=1).to(DEV)
    c3 = pack_conv(torch.randn(4 * mid, mid, 1, 1) / mid ** 0.5, torch.randn(4 * mid) * 0.1).to(DEV)
    dn = pack_conv(torch.randn(4 * mid, 64, 1, 1) / 8, torch.randn(4 * mid) * 0.1).to(DEV)
    c1n = pack_conv(torch.randn(mid, 4 * mid, 1, 1) / (4 * mid) ** 0.5, torch.randn(mid) * 0.1).to(DEV)
    t1 = torch.randn(n, h, w, mid, device=DEV).relu().to(torch.bfloat16)
    x0 = torch.randn(n, h, w, 64, device=DEV).relu().to(torch.bfloat16)
    y, t1n = conv_chain(t1, c2, c3, None, c1n=c1n, down=dn, x0=x0, tile_cfg=tile)
    torch.cuda.synchronize()
    t2 = F.relu(_conv(t1, _wq(c2, 3), c2.bias[:mid], 1, 1)).to(torch.bfloat16)
    res = _conv(x0, _wq(dn, 1), dn.bias[:4 * mid])
    yr = F.relu(_conv(t2, _wq(c3, 1), c3.bias[:4 * mid]) + res)
    err = (y.float() - yr).abs().max().item()
    assert err <= 0.02 * yr.abs().max().item() + 0.03, err
    tr = F.relu(_conv(y, _wq(c1n, 1), c1n.bias[:mid]))
    err = (t1n.float() - tr).abs().max().item()
    assert err <= 0.02 * tr.abs().max().item() + 0.03, err


@pytest.mark.parametrize("shape", [(3, 112, 112), (2, 31, 25), (1, 17, 9)])
def test_stem_pool_fused_c1(shape):
    """K1s with the first bottleneck's 1x1 fused (t1 from the pooled tile in LDS) == K1s + a K1 conv."""
    from aiforearth_api_platform_amd.ops.conv import conv2d_nhwc, pack_stem_s2d, stem_pool, stem_pool_c1

    n, h, w = shape
    torch.manual_seed(8)
    pc = pack_stem_s2d(torch.randn(64, 3, 7, 7) / 12, torch.randn(64) * 0.1).to(DEV)
    c1 = pack_conv(torch.randn(64, 64, 1, 1) / 8, torch.randn(64) * 0.1).to(DEV)
    x = torch.randn(n, h, w, 16, device=DEV).to(torch.bfloat16)
    y, t1 = stem_pool_c1(x, pc, c1)
    yr = stem_pool(x, pc)
    tr = conv2d_nhwc(yr, c1, relu=True)
    torch.cuda.synchronize()
    assert torch.equal(y, yr)
    assert (t1.float() - tr.float()).abs().max().item() <= 0.02 * tr.float().abs().max().item() + 0.02
