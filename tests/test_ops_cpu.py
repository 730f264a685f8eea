"""CPU reference ops (used as the numerics oracle for the HIP kernels)."""
import math

import torch
import torch.nn.functional as F

from aiforearth_api_platform_amd.ops.detection import (batched_nms, box_iou, crop_resize_reference, decode_boxes,
                                                       map_levels, nms_batched_sorted, nms_reference,
                                                       roi_align_reference)
from aiforearth_api_platform_amd.ops.norm import group_norm_nhwc, upsample2x_nhwc
from aiforearth_api_platform_amd.ops.stitch import TileGrid, stitch_reference, tile_stitch


def rand_boxes(n, g=None, size=100.0):
    xy = torch.rand(n, 2, generator=g) * size
    wh = torch.rand(n, 2, generator=g) * size / 3 + 1
    return torch.cat([xy, xy + wh], 1)


def test_nms_reference_properties():
    g = torch.Generator().manual_seed(0)
    b = rand_boxes(200, g)
    s = torch.rand(200, generator=g)
    keep = nms_reference(b, s, 0.5)
    kb = b[keep]
    iou = box_iou(kb, kb)
    iou.fill_diagonal_(0)
    assert iou.max() <= 0.5
    assert torch.all(s[keep][:-1] >= s[keep][1:])
    # every removed box overlaps some kept higher-scoring box
    rem = torch.tensor([i for i in range(200) if i not in set(keep.tolist())])
    ov = box_iou(b[rem], kb)
    assert torch.all((ov > 0.5).any(1))


def test_batched_nms_separates_classes():
    b = torch.tensor([[0, 0, 10, 10], [0, 0, 10, 10.]])
    s = torch.tensor([0.9, 0.8])
    assert batched_nms(b, s, torch.tensor([0, 0]), 0.5).tolist() == [0]
    assert sorted(batched_nms(b, s, torch.tensor([0, 1]), 0.5).tolist()) == [0, 1]


def test_nms_sorted_batched_cpu_matches_reference():
    g = torch.Generator().manual_seed(1)
    B, N = 3, 300
    boxes = torch.stack([rand_boxes(N, g) for _ in range(B)])
    keep, cnt = nms_batched_sorted(boxes, 0.6, 100)
    for i in range(B):
        ref = nms_reference(boxes[i], torch.arange(N, 0, -1).float(), 0.6)[:100]
        assert keep[i, :cnt[i]].long().tolist() == ref.tolist()


def test_decode_boxes_identity_and_levels():
    a = torch.tensor([[10., 20., 30., 60.]])
    assert torch.allclose(decode_boxes(a, torch.zeros(1, 4)), a)
    d = decode_boxes(a, torch.tensor([[0.1, 0.0, math.log(2), 0.0]]))
    assert torch.allclose(d, torch.tensor([[2.0, 20.0, 42.0, 60.0]]))
    rois = torch.tensor([[0, 0, 0, 224, 224.], [0, 0, 0, 20, 20], [0, 0, 0, 900, 900]])
    assert map_levels(rois).tolist() == [2, 0, 3]


def test_roi_align_reference_constant_and_linear():
    # on a linear ramp feature map, bilinear RoIAlign is exact for the bin centres
    H = W = 16
    f = torch.arange(W, dtype=torch.float32)[None, None, :, None].expand(1, H, W, 8).contiguous()
    rois = torch.tensor([[0, 2.0, 2.0, 10.0, 10.0]])
    out = roi_align_reference(f, rois, (4, 4), 1.0, sampling=2, aligned=True)
    # aligned: x spans [1.5, 9.5) -> bin centres at 1.5 + (pw + 0.5) * 2
    exp = torch.tensor([1.5 + (pw + 0.5) * 2 for pw in range(4)])
    assert torch.allclose(out[0, 0, :, 0], exp, atol=1e-5)


def test_crop_resize_reference_full_image_identity():
    img = torch.randint(0, 256, (1, 8, 8, 3), dtype=torch.uint8)
    out = crop_resize_reference(img, torch.tensor([[0, 0, 0, 8, 8.]]), (8, 8), mean=(0, 0, 0), std=(1, 1, 1))
    assert torch.allclose(out[0, ..., :3], img[0].float() / 255, atol=1e-6)


def test_groupnorm_upsample_torch_path():
    x = torch.randn(2, 6, 5, 64)
    g, b = torch.rand(64) + 0.5, torch.randn(64)
    y = group_norm_nhwc(x, g, b, 32, relu=True)
    ref = F.relu(F.group_norm(x.permute(0, 3, 1, 2), 32, g, b)).permute(0, 2, 3, 1)
    assert torch.allclose(y, ref, atol=1e-5)
    buf = torch.zeros(2, 12, 10, 80)
    upsample2x_nhwc(x, out=buf, out_coff=16)
    ref = F.interpolate(x.permute(0, 3, 1, 2), scale_factor=2, mode="bilinear").permute(0, 2, 3, 1)
    assert torch.allclose(buf[..., 16:], ref, atol=1e-5) and buf[..., :16].abs().sum() == 0


def test_tile_grid_and_stitch_reference():
    grid = TileGrid(100, 90, 32, 24)
    assert grid.nty == 4 and grid.ntx == 4 and grid.padded_hw() == (104, 104)
    # a constant per-class logit field must stitch back exactly
    C = 4
    field = torch.randn(*grid.padded_hw(), C)
    tiles = torch.stack([torch.stack([field[y:y + 32, x:x + 32] for x in range(0, 4 * 24, 24)])
                         for y in range(0, 4 * 24, 24)])
    cls, prob = stitch_reference(tiles, grid, with_prob=True)
    assert torch.equal(cls, field[:100, :90].argmax(-1).to(torch.uint8))
    # sharded rows: a shard only needs its tile rows
    ty0, ty1 = grid.tile_rows_for(40, 70)
    cls2, _ = tile_stitch(tiles[ty0:ty1], grid, row0=40, rows=30, ty0=ty0)
    assert torch.equal(cls2, cls[40:70])


def test_pack_mfma_frags_layout():
    """K1p weight packing: fragment (rb, ks), lane l holds row 16 rb + (l & 15), K 32 ks + 8 (l >> 4) .. +8."""
    from aiforearth_api_platform_amd.ops.conv import pack_mfma_frags

    w = torch.arange(64 * 96, dtype=torch.float32).reshape(64, 96)
    p = pack_mfma_frags(w)
    assert p.shape == (4, 3, 64, 8)
    for rb in range(4):
        for ks in range(3):
            for lane in (0, 5, 16, 37, 63):
                r, k0 = 16 * rb + (lane & 15), 32 * ks + 8 * (lane >> 4)
                assert torch.equal(p[rb, ks, lane], w[r, k0:k0 + 8])


def test_conv_pair_cpu_fallback_matches_two_convs():
    from aiforearth_api_platform_amd.ops.conv import conv2d_nhwc, conv_pair, pack_conv

    torch.manual_seed(3)
    c3 = pack_conv(torch.randn(1024, 256, 1, 1) / 16, torch.randn(1024) * 0.1)
    c1n = pack_conv(torch.randn(256, 1024, 1, 1) / 32, torch.randn(256) * 0.1)
    t2 = torch.randn(1, 3, 4, 256).relu()
    res = torch.randn(1, 3, 4, 1024)
    y, t1n = conv_pair(t2, c3, res, c1n)
    y_ref = conv2d_nhwc(t2, c3, residual=res, relu=True)
    assert torch.allclose(y, y_ref)
    assert torch.allclose(t1n, conv2d_nhwc(y_ref, c1n, relu=True))


def test_gpu_telemetry_fail_soft_and_summary():
    from aiforearth_api_platform_amd.utils.gpu_telemetry import GpuTelemetry, summarize

    t = GpuTelemetry(0)  # no GPU driver in the CPU container: empty, never raises
    t.start(0.01)
    s = t.stop()
    assert isinstance(s, dict)
    out = summarize([{"gfx_mhz": 2000.0, "power_w": 900.0}, {"gfx_mhz": 2400.0}])
    assert out["gfx_mhz"] == {"min": 2000.0, "mean": 2200.0, "max": 2400.0, "n": 2}
    assert out["power_w"]["n"] == 1


def test_conv_head_cpu_fallback_matches_two_convs():
    """``conv2d_head_nhwc`` (the RPN conv with its 16-channel head fused on the GPU's 256-wide tiles) falls back to the
    two convs off the HIP backend; the result is the head of the ReLU'd conv, [N, H, W, 16]."""
    from aiforearth_api_platform_amd.ops.conv import conv2d_head_nhwc, conv2d_nhwc, pack_conv

    g = torch.Generator().manual_seed(3)
    pc = pack_conv(torch.randn(256, 256, 3, 3, generator=g) * 0.02, torch.randn(256, generator=g) * 0.1, pad=1)
    head = pack_conv(torch.randn(16, 256, 1, 1, generator=g) * 0.05, torch.randn(16, generator=g) * 0.1)
    x = torch.randn(1, 6, 5, 256, generator=g)
    y = conv2d_head_nhwc(x, pc, head, tile_cfg=6)
    ref = conv2d_nhwc(conv2d_nhwc(x, pc, relu=True), head)
    assert y.shape == (1, 6, 5, 16)
    assert torch.equal(y, ref)


def test_split_cfg_decoding_and_cpu_conv():
    """Tile-table entries ``cfg | ks << 4`` select split-K on the 256-wide configs only; the CPU path ignores them."""
    from aiforearth_api_platform_amd.ops.conv import conv2d_nhwc, pack_conv, split_cfg

    assert split_cfg(9) == (1, 9) and split_cfg(0) == (1, 0)
    assert split_cfg(9 | 2 << 4) == (2, 9) and split_cfg(6 | 4 << 4) == (4, 6) and split_cfg(10 | 3 << 4) == (3, 10)
    assert split_cfg(4 | 2 << 4) == (1, 4)  # not a 256-wide config: the plain tile
    torch.manual_seed(0)
    pc = pack_conv(torch.randn(32, 16, 3, 3) / 12, torch.zeros(32), pad=1)
    x = torch.randn(2, 5, 5, pc.cin_pad).bfloat16()
    a = conv2d_nhwc(x, pc, relu=True, tile_cfg=9 | 2 << 4)
    b = conv2d_nhwc(x, pc, relu=True, tile_cfg=9)
    assert torch.equal(a, b)
