"""ResNet-50 folding/packing on CPU: fused NHWC graph == nn.Module reference; packed layout == im2col GEMM."""
import torch
import torch.nn.functional as F

from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50
from aiforearth_api_platform_amd.ops.conv import conv2d_nhwc, pack_conv
from aiforearth_api_platform_amd.ops.pool import preprocess_u8


def emulate_packed_conv(x_nhwc, pc):
    """Exactly the K1 kernel's math on CPU: gather (kh,kw,c)-ordered K, GEMM with the packed rows."""
    n, h, w, c = x_nhwc.shape
    oh, ow = pc.out_hw(h, w)
    xp = F.pad(x_nhwc.float(), (0, 0, pc.pad, pc.pad, pc.pad, pc.pad))
    cols = []
    for kh in range(pc.kh):
        for kw in range(pc.kw):
            cols.append(xp[:, kh:kh + pc.stride * (oh - 1) + 1:pc.stride, kw:kw + pc.stride * (ow - 1) + 1:pc.stride, :])
    a = torch.cat(cols, dim=-1).reshape(n * oh * ow, -1)
    a = F.pad(a, (0, pc.kpad - a.shape[1]))
    y = a @ pc.w_packed[:pc.cout].float().t() + pc.bias[:pc.cout]
    return y.reshape(n, oh, ow, pc.cout)


def test_packed_layout_matches_reference_conv():
    torch.manual_seed(0)
    for (cin, cout, k, s, p) in [(3, 64, 7, 2, 3), (64, 64, 3, 1, 1), (128, 128, 3, 2, 1), (256, 512, 1, 2, 0)]:
        w = torch.randn(cout, cin, k, k) * 0.1
        b = torch.randn(cout)
        pc = pack_conv(w, b, stride=s, pad=p)
        x = torch.randn(2, 13, 11, pc.cin_pad)
        x[..., cin:] = 0
        ref = F.conv2d(x[..., :cin].permute(0, 3, 1, 2), w, b, stride=s, padding=p).permute(0, 2, 3, 1)
        emu = emulate_packed_conv(x.to(torch.bfloat16).float(), pc)
        assert torch.allclose(emu, ref, atol=0.05 * ref.abs().max().item() + 1e-3), (cin, cout, k, s)


def test_fused_resnet_matches_module():
    torch.manual_seed(0)
    m = resnet50(num_classes=100, seed=1)
    fused = FusedResNet(m)
    img = torch.randint(0, 256, (2, 64, 64, 3), dtype=torch.uint8)
    logits = fused(img)
    x = preprocess_u8(img)[..., :3].permute(0, 3, 1, 2).float()
    with torch.no_grad():
        ref = m(x)
    assert logits.shape == (2, 100)
    assert torch.allclose(logits, ref, rtol=1e-3, atol=1e-3 * ref.abs().max().item())


def test_conv_writes_channel_slice_of_concat_buffer():
    w = torch.randn(16, 8, 3, 3)
    pc = pack_conv(w, None, pad=1)
    x = torch.randn(1, 5, 5, 8)
    out = torch.zeros(1, 5, 5, 40)
    conv2d_nhwc(x, pc, out=out, out_coff=24)
    assert out[..., :24].abs().sum() == 0 and out[..., 24:].abs().sum() > 0


def test_flops_resnet50():
    fused = FusedResNet(resnet50())
    gf = fused.flops(1) / 1e9
    assert 8.0 < gf < 8.4  # ~4.1 GMAC / image


def test_chunked_prefix_matches_full_batch():
    """Cache-resident micro-batching of the high-resolution stages does not change the result."""
    m = resnet50(seed=5)
    img = torch.randint(0, 256, (6, 64, 64, 3), dtype=torch.uint8)
    ref = FusedResNet(m, chunk=None).forward_u8(img)
    for chunk in [(4, 3), (2, 7), (5, 16)]:
        out = FusedResNet(m, chunk=chunk).forward_u8(img)
        assert out.shape == ref.shape
        assert (out - ref).abs().max().item() < 1e-2, chunk


def test_pair_route_defaults():
    from aiforearth_api_platform_amd.ops import conv as convmod

    assert convmod.pair_route(256, 1024, 256)          # layer3 pairs: K1p by default
    assert not convmod.pair_route(128, 512, 256)       # layer2 -> layer3: the K1c chain
    assert not convmod.pair_route(256, 1024, 512)      # layer3 -> layer4: opt-in (AI4E_PAIR_X)
    assert not convmod.pair_route(512, 2048, 512)      # layer4: opt-in (AI4E_PAIR_L4)
    assert not convmod.pair_route(64, 256, 64)         # not a K1p shape
