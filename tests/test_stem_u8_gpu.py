"""The uint8-input stem (K1s building its input footprint from the RGB images: preprocess fused into the stem launch)
against the two-launch path it replaces (preprocess_s2d_u8 + stem_pool_c1), and the stem against an fp32 PyTorch
reference of conv 7x7/2 + ReLU + max-pool 3x3/2 + the fused 1x1 (GPU box only)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from aiforearth_api_platform_amd.ops import _ext
from aiforearth_api_platform_amd.ops.conv import pack_conv, pack_stem_s2d, stem_pool_c1, stem_pool_c1_u8, stem_u8_supported
from aiforearth_api_platform_amd.ops.pool import IMAGENET_MEAN, IMAGENET_STD, preprocess_s2d_u8

DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from aiforearth_api_platform_amd import _build
    _build.build_kernels()
    _ext.lib()


def _stem(seed=0):
    g = torch.Generator().manual_seed(seed)
    w7 = torch.randn(64, 3, 7, 7, generator=g) / 12
    b = torch.randn(64, generator=g) * 0.1
    w1 = torch.randn(64, 64, 1, 1, generator=g) / 8
    b1 = torch.randn(64, generator=g) * 0.1
    return w7, b, pack_stem_s2d(w7, b).to(DEV), w1, b1, pack_conv(w1, b1).to(DEV)


@pytest.mark.parametrize("shape", [(250, 224, 224), (3, 64, 96), (2, 30, 46), (1, 226, 222)])
def test_stem_u8_matches_two_launch_path(shape):
    n, h, w = shape
    _, _, pc, _, _, c1 = _stem()
    img = torch.randint(0, 256, (n, h, w, 3), dtype=torch.uint8, device=DEV)
    assert stem_u8_supported(img, pc, c1)
    y, t1 = stem_pool_c1_u8(img, pc, c1)
    y_ref, t1_ref = stem_pool_c1(preprocess_s2d_u8(img), pc, c1)
    torch.cuda.synchronize()
    # the same normalization arithmetic, the same footprint values: bit-identical except the last pooled rows and
    # columns (one, or two for odd H/2), where the two-launch path's [N, H/2, W/2, 16] s2d tensor leaves the image's
    # last row / column out (the fp32 test below checks the edge against the 7x7/2 conv)
    assert torch.equal(y[:, :-2, :-2], y_ref[:, :-2, :-2])
    assert torch.equal(t1[:, :-2, :-2], t1_ref[:, :-2, :-2])


@pytest.mark.parametrize("shape", [(2, 64, 96), (3, 224, 224), (1, 30, 46)])
def test_stem_u8_vs_fp32_reference(shape):
    w7, b, pc, w1, b1, c1 = _stem(1)
    img = torch.randint(0, 256, (*shape, 3), dtype=torch.uint8, device=DEV)
    y, t1 = stem_pool_c1_u8(img, pc, c1)
    x = (img.float() / 255 - torch.tensor(IMAGENET_MEAN, device=DEV)) / torch.tensor(IMAGENET_STD, device=DEV)
    xq = x.to(torch.bfloat16).float().permute(0, 3, 1, 2)
    wq = w7.to(torch.bfloat16).float().to(DEV)
    ref = F.max_pool2d(F.relu(F.conv2d(xq, wq, b.to(DEV), stride=2, padding=3)), 3, 2, 1)
    ref = ref.permute(0, 2, 3, 1)
    # every output, the bottom / right edge included (the exact 7x7/2, pad 3 conv): the edge is no worse than the
    # interior (the two-launch path's s2d tensor leaves the image's last row / column out there)
    err = (y.float() - ref).abs()
    assert err.max().item() <= 0.02 * ref.abs().max().item() + 0.02
    edge = torch.cat([err[:, -1].flatten(), err[:, :, -1].flatten()]).max().item()
    assert edge <= max(2 * err[:, :-1, :-1].max().item(), 0.05), edge
    # the fused 1x1 on the pooled tile == the 1x1 of the stored pooled values
    ref1 = F.relu(F.conv2d(y.float().permute(0, 3, 1, 2), w1.to(torch.bfloat16).float().to(DEV), b1.to(DEV)))
    ref1 = ref1.permute(0, 2, 3, 1)
    assert (t1.float() - ref1).abs().max().item() <= 0.01 * ref1.abs().max().item() + 0.02
