"""K1t (csrc/kernels/conv_tile3x3.hip): the 64 -> 64 3x3 conv from an LDS input patch, against fp32 PyTorch
references of the same op — plain, with the fused GroupNorm + ReLU input prologue, on a channel-sliced input — its
GroupNorm statistics against the statistics of the stored output, and the U-Net forward with and without it."""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(autouse=True)
def _k1t_on(monkeypatch):
    monkeypatch.setenv("AI4E_CONV_TILE64", "1")


def _conv_ref(xin: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    y = F.conv2d(xin.permute(0, 3, 1, 2).float(), w.float(), b.float(), padding=1)
    return y.permute(0, 2, 3, 1)


def _case(n, h, w, seed, cin=64, cout=64):
    from aiforearth_api_platform_amd.ops.conv import pack_conv
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, h, w, cin, generator=g).to(torch.bfloat16)
    wt = (torch.randn(cout, cin, 3, 3, generator=g) * 0.05).to(torch.bfloat16).float()
    b = torch.randn(cout, generator=g) * 0.1
    return x, wt, b, pack_conv(wt, b, pad=1).to(DEV)


# the last two: 768 tiles > the persistent grid (2 x 256 CUs), so workgroups walk several tiles (next-tile prefetch)
@pytest.mark.parametrize("n,h,w,cin,cout", [(2, 16, 64, 64, 64), (1, 64, 32, 64, 64), (3, 8, 96, 64, 64),
                                            (2, 16, 64, 128, 64), (1, 8, 32, 128, 64), (3, 128, 512, 64, 64),
                                            (3, 128, 512, 128, 64)])
def test_conv3x3_tile64_matches_fp32(n, h, w, cin, cout):
    from aiforearth_api_platform_amd.ops.conv import conv3x3_tile64
    x, wt, b, pc = _case(n, h, w, n * 100 + h, cin, cout)
    y, st = conv3x3_tile64(x.to(DEV), pc)
    assert st is None
    ref = _conv_ref(x, wt, b)
    rel = ((y.float().cpu() - ref).norm() / ref.norm()).item()
    assert rel < 6e-3, rel


@pytest.mark.parametrize("cin,cout", [(64, 64), (128, 64)])
def test_conv3x3_tile64_prologue_and_sliced_input(cin, cout):
    """The prologue affine is per image (and per k-slice for 128 / 256 channels): 3 images of 256 / 512 tiles, so
    persistent workgroups cross images."""
    from aiforearth_api_platform_amd.ops.conv import conv3x3_tile64
    n, h, w = 3, 128, 512
    x, wt, b, pc = _case(n, h, w, 7, cin, cout)
    g = torch.Generator().manual_seed(8)
    aff = torch.stack([0.5 + torch.rand(n, cin, generator=g), torch.randn(n, cin, generator=g) * 0.5], -1)
    wide = torch.zeros(n, h, w, cin + 64, dtype=torch.bfloat16)
    wide[..., 64:] = x
    y, _ = conv3x3_tile64(wide.to(DEV)[..., 64:], pc, pro=aff.to(DEV).contiguous(), pro_relu=True)
    xin = torch.relu(x.float() * aff[:, None, None, :, 0] + aff[:, None, None, :, 1]).to(torch.bfloat16)
    ref = _conv_ref(xin, wt, b)
    rel = ((y.float().cpu() - ref).norm() / ref.norm()).item()
    assert rel < 6e-3, rel


@pytest.mark.parametrize("groups,cin,n,h,w,cout", [(32, 64, 2, 32, 64, 64), (16, 64, 2, 32, 64, 64),
                                                   (32, 128, 2, 32, 64, 64), (32, 64, 3, 128, 512, 64),
                                                   (32, 128, 3, 128, 512, 64)])
def test_conv3x3_tile64_groupnorm_statistics(groups, cin, n, h, w, cout):
    """The epilogue's shifted per-tile sums, finalized (ops.norm.group_norm_affine), equal the GroupNorm affine of
    the stored output computed directly in fp64 (the last case: several tiles per persistent workgroup)."""
    from aiforearth_api_platform_amd.ops.conv import conv3x3_tile64
    from aiforearth_api_platform_amd.ops.norm import group_norm_affine
    x, wt, b, pc = _case(n, h, w, 21, cin, cout)
    y, st = conv3x3_tile64(x.to(DEV), pc, gn_groups=groups)
    gamma = torch.linspace(0.5, 1.5, cout)
    beta = torch.linspace(-0.2, 0.2, cout)
    ss = group_norm_affine(st, gamma, beta, n=n, hw=h * w, c=cout, groups=groups).cpu()
    yd = y.double().cpu().reshape(n, h * w, groups, cout // groups)
    mean = yd.mean(dim=(1, 3))
    var = yd.var(dim=(1, 3), unbiased=False)
    rstd = (var + 1e-5).rsqrt()
    a = (gamma.double().reshape(groups, -1)[None] * rstd[..., None]).reshape(n, cout)
    bb = beta.double()[None] - (mean[..., None] * a.reshape(n, groups, -1)).reshape(n, cout)
    assert torch.allclose(ss[..., 0].double(), a, rtol=1e-4, atol=1e-5)
    assert torch.allclose(ss[..., 1].double(), bb, rtol=1e-4, atol=1e-4)


def test_unet_forward_with_and_without_k1t():
    """The land-cover U-Net (its full-resolution DoubleConvs take K1t with the fused GroupNorm prologue) equals the
    K1 path (AI4E_CONV_TILE64=0) and stays within the fp32 reference's tolerance."""
    from aiforearth_api_platform_amd.models.unet import FusedUNet, unet_landcover
    m = unet_landcover(seed=3)
    f = FusedUNet(m, device=DEV)
    img = torch.randint(0, 256, (2, 256, 256, 4), dtype=torch.uint8, generator=torch.Generator().manual_seed(3))
    y_tile = f.forward_u8(img.to(DEV)).float()
    os.environ["AI4E_CONV_TILE64"] = "0"  # (the fixture restores it)
    y_k1 = f.forward_u8(img.to(DEV)).float()
    k = f.n_classes
    rel = ((y_tile[..., :k] - y_k1[..., :k]).norm() / y_k1[..., :k].norm()).item()
    assert rel < 2e-2, rel
    agree = (y_tile[..., :k].argmax(-1) == y_k1[..., :k].argmax(-1)).float().mean().item()
    assert agree > 0.97, agree


@pytest.mark.parametrize("n,h,w,slice_", [(2, 32, 64, False), (3, 64, 96, True)])
def test_gn_relu_head8_matches_fp32(n, h, w, slice_):
    """The fused U-Net head (csrc/kernels/norm_resample.hip gn_relu_head8_kernel): conv1x1(relu(z * a + b)) + bias,
    64 -> 8, against fp32 PyTorch of the same op (normalized values rounded to bf16 as the apply pass stores them)."""
    from aiforearth_api_platform_amd.ops.conv import pack_conv
    from aiforearth_api_platform_amd.ops.norm import gn_relu_head8
    g = torch.Generator().manual_seed(n * 7 + h)
    z = torch.randn(n, h, w, 64, generator=g).to(torch.bfloat16)
    ss = torch.stack([0.5 + torch.rand(n, 64, generator=g), torch.randn(n, 64, generator=g) * 0.3], -1)
    wt = (torch.randn(8, 64, 1, 1, generator=g) * 0.1).to(torch.bfloat16).float()
    b = torch.randn(8, generator=g) * 0.1
    pc = pack_conv(wt, b).to(DEV)
    zin = z
    if slice_:  # a channel slice of a wider buffer
        wide = torch.zeros(n, h, w, 128, dtype=torch.bfloat16)
        wide[..., 64:] = z
        zin = wide.to(DEV)[..., 64:]
    y = gn_relu_head8(zin.to(DEV), ss.to(DEV).contiguous(), pc).float().cpu()
    xn = torch.relu((z.float() * ss[:, None, None, :, 0] + ss[:, None, None, :, 1]).to(torch.bfloat16).float())
    ref = xn @ wt.reshape(8, 64).t() + b
    rel = ((y - ref).norm() / ref.norm()).item()
    assert rel < 6e-3, rel


def test_unet_fused_head_equals_apply_then_conv():
    """The U-Net forward with the fused head equals AI4E_UNET_FUSED_HEAD=0 (GroupNorm apply, then the 1x1 head)."""
    from aiforearth_api_platform_amd.models.unet import FusedUNet, unet_landcover
    m = unet_landcover(seed=5)
    img = torch.randint(0, 256, (2, 256, 256, 4), dtype=torch.uint8, generator=torch.Generator().manual_seed(5))
    y_f = FusedUNet(m, device=DEV).forward_u8(img.to(DEV)).float()
    os.environ["AI4E_UNET_FUSED_HEAD"] = "0"
    try:
        y_u = FusedUNet(m, device=DEV).forward_u8(img.to(DEV)).float()
    finally:
        del os.environ["AI4E_UNET_FUSED_HEAD"]
    k = m.n_classes
    rel = ((y_f[..., :k] - y_u[..., :k]).norm() / y_u[..., :k].norm()).item()
    assert rel < 1e-2, rel
    assert (y_f[..., :k].argmax(-1) == y_u[..., :k].argmax(-1)).float().mean().item() > 0.99
