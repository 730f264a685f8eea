"""HIP kernels K2-K6 vs the PyTorch references (GPU box only)."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from aiforearth_api_platform_amd.ops import _ext
from aiforearth_api_platform_amd.ops.detection import (crop_resize_nhwc, crop_resize_reference, nms_batched_sorted,
                                                       nms_reference, roi_align_nhwc, roi_align_reference)
from aiforearth_api_platform_amd.ops.norm import group_norm_nhwc, upsample2x_nhwc
from aiforearth_api_platform_amd.ops.stitch import TileGrid, stitch_reference, tile_stitch

DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from aiforearth_api_platform_amd import _build
    _build.build_kernels()
    _ext.lib()


@pytest.mark.parametrize("shape,groups", [((2, 33, 17, 64), 32), ((1, 64, 64, 256), 32), ((3, 9, 9, 32), 8),
                                          ((2, 40, 40, 512), 32)])
@pytest.mark.parametrize("relu", [False, True])
def test_groupnorm(shape, groups, relu):
    torch.manual_seed(0)
    x = (torch.randn(*shape) * 2 + 0.5).to(DEV).bfloat16()
    g, b = torch.rand(shape[-1]) + 0.5, torch.randn(shape[-1])
    y = group_norm_nhwc(x, g, b, groups, relu=relu)
    ref = F.group_norm(x.float().permute(0, 3, 1, 2), groups, g.to(DEV), b.to(DEV))
    ref = (F.relu(ref) if relu else ref).permute(0, 2, 3, 1)
    assert (y.float() - ref).abs().max().item() < 0.05


@pytest.mark.parametrize("shape,groups", [((2, 64, 64, 64), 32), ((1, 40, 40, 512), 32), ((3, 9, 9, 32), 8)])
def test_groupnorm_bitwise_reproducible(shape, groups):
    """The statistics reduction has a fixed order (no float atomics): repeated runs give identical bits."""
    torch.manual_seed(5)
    x = (torch.randn(*shape) * 3 + 1.0).to(DEV).bfloat16()
    g, b = torch.rand(shape[-1]) + 0.5, torch.randn(shape[-1])
    first = group_norm_nhwc(x, g, b, groups, relu=True)
    for _ in range(5):
        assert torch.equal(group_norm_nhwc(x, g, b, groups, relu=True), first)


@pytest.mark.parametrize("dc,std", [(50.0, 0.5), (300.0, 2.0)])
def test_groupnorm_large_dc_offset(dc, std):
    """A group whose mean is far from 0 relative to its spread: the shifted chunk sums keep E[x^2] - mean^2
    from cancelling (reference: torch fp32 GroupNorm of the same bf16 input)."""
    torch.manual_seed(3)
    x = (dc + std * torch.randn(2, 48, 64, 64)).to(DEV).bfloat16()  # 3072 pixels: 3 chunks per image
    g, b = torch.rand(64) + 0.5, torch.randn(64)
    y = group_norm_nhwc(x, g, b, 32)
    ref = F.group_norm(x.float().permute(0, 3, 1, 2), 32, g.to(DEV), b.to(DEV)).permute(0, 2, 3, 1)
    assert (y.float() - ref).abs().max().item() < 0.03


def test_conv_fused_groupnorm_stats_dc_offset(monkeypatch):
    """Conv-epilogue GroupNorm statistics on an output with a large DC offset (bias 40): same as the fp32
    reference GroupNorm of the stored conv output."""
    from aiforearth_api_platform_amd.ops import conv as convmod
    from aiforearth_api_platform_amd.ops.conv import conv2d_gn_nhwc, pack_conv

    monkeypatch.setattr(convmod, "tuned_tile", lambda *a: 1)
    torch.manual_seed(9)
    pc = pack_conv(torch.randn(64, 64, 3, 3) / (9 * 64) ** 0.5 * 0.2, torch.full((64,), 40.0), pad=1).to(DEV)
    x = torch.randn(2, 32, 32, 64, device=DEV).to(torch.bfloat16)
    y, st = conv2d_gn_nhwc(x, pc, 32)
    assert st is not None
    gamma, beta = torch.rand(64, device=DEV) + 0.5, torch.randn(64, device=DEV) * 0.1
    a = group_norm_nhwc(y, gamma, beta, groups=32, stats=st)
    ref = F.group_norm(y.float().permute(0, 3, 1, 2), 32, gamma, beta).permute(0, 2, 3, 1)
    assert (a.float() - ref).abs().max().item() < 0.03


def test_groupnorm_concat_slices():
    x_big = torch.randn(1, 16, 16, 96, device=DEV).bfloat16()
    x = x_big[..., 32:96]
    out = torch.zeros(1, 16, 16, 128, device=DEV, dtype=torch.bfloat16)
    g, b = torch.ones(64), torch.zeros(64)
    group_norm_nhwc(x, g, b, 32, out=out[..., 64:])
    ref = F.group_norm(x.float().permute(0, 3, 1, 2), 32).permute(0, 2, 3, 1)
    assert out[..., :64].abs().max() == 0
    assert (out[..., 64:].float() - ref).abs().max().item() < 0.05


@pytest.mark.parametrize("shape", [(2, 16, 16, 64), (1, 7, 9, 32), (1, 64, 64, 128), (1, 1, 1, 8), (2, 1, 5, 16), (1, 3, 1, 8)])
def test_upsample_into_concat(shape):
    x = torch.randn(*shape, device=DEV).bfloat16()
    n, h, w, c = shape
    buf = torch.zeros(n, 2 * h, 2 * w, c + 16, device=DEV, dtype=torch.bfloat16)
    upsample2x_nhwc(x, out=buf, out_coff=16)
    ref = F.interpolate(x.float().permute(0, 3, 1, 2), scale_factor=2, mode="bilinear",
                        align_corners=False).permute(0, 2, 3, 1)
    assert (buf[..., 16:].float() - ref).abs().max().item() < 0.02
    assert buf[..., :16].abs().max() == 0


@pytest.mark.parametrize("N,thr", [(100, 0.5), (2000, 0.7), (777, 0.3)])
def test_nms_matches_reference(N, thr):
    """Parity unpinned against torchvision.ops.nms (not installed in this image): the kernel is compared with the
    greedy reference ``ops.detection.nms_reference``, whose semantics are pinned by a hand-computed case in
    tests/test_detector_cpu.py::test_nms_reference_hand_computed."""
    g = torch.Generator().manual_seed(N)
    B = 3
    xy = torch.rand(B, N, 2, generator=g) * 500
    wh = torch.rand(B, N, 2, generator=g) * 120 + 2
    boxes = torch.cat([xy, xy + wh], -1)
    valid = torch.tensor([N, N - 7, N // 2], dtype=torch.int32)
    keep, cnt = nms_batched_sorted(boxes.to(DEV), thr, 1000, valid.to(DEV))
    keep, cnt = keep.cpu(), cnt.cpu()
    for b in range(B):
        n = int(valid[b])
        ref = nms_reference(boxes[b, :n], torch.arange(n, 0, -1).float(), thr)[:1000]
        assert keep[b, :cnt[b]].long().tolist() == ref.tolist()


@pytest.mark.parametrize("N,thr,max_out,dense", [(4352, 0.7, 1000, False), (8192, 0.5, 300, False),
                                                  (130, 0.9, 1000, False), (3000, 0.3, 1000, True)])
def test_nms_multiwave_scan_matches_reference(N, thr, max_out, dense):
    """The RPN-sized scans (4352 proposals, max_out truncation, the 8192 limit, a dense cluster where most boxes are
    suppressed) through the default multi-wave reduce (csrc/kernels/detection.hip nms_reduce_mw_kernel) == the greedy
    reference."""
    g = torch.Generator().manual_seed(N + int(dense))
    B = 2
    xy = torch.rand(B, N, 2, generator=g) * (60 if dense else 600)
    wh = torch.rand(B, N, 2, generator=g) * 120 + 2
    boxes = torch.cat([xy, xy + wh], -1)
    valid = torch.tensor([N, N - 37], dtype=torch.int32)
    keep, cnt = nms_batched_sorted(boxes.to(DEV), thr, max_out, valid.to(DEV))
    keep, cnt = keep.cpu(), cnt.cpu()
    for b in range(B):
        n = int(valid[b])
        ref = nms_reference(boxes[b, :n], torch.arange(n, 0, -1).float(), thr)[:max_out]
        assert int(cnt[b]) == len(ref)
        assert keep[b, :cnt[b]].long().tolist() == ref.tolist()
        assert (keep[b, cnt[b]:] == -1).all()  # padded by the scan itself (no fill launch)


@pytest.mark.parametrize("aligned", [False, True])
def test_roi_align(aligned):
    g = torch.Generator().manual_seed(0)
    feat = torch.randn(2, 25, 38, 64, generator=g)
    R = 40
    x1 = torch.rand(R, generator=g) * 500
    y1 = torch.rand(R, generator=g) * 350
    rois = torch.stack([torch.randint(0, 2, (R,), generator=g).float(), x1, y1,
                        x1 + torch.rand(R, generator=g) * 200 + 1, y1 + torch.rand(R, generator=g) * 150 + 1], 1)
    ref = roi_align_reference(feat.bfloat16().float(), rois, (7, 7), 1 / 16, 2, aligned)
    out = roi_align_nhwc(feat.to(DEV).bfloat16(), rois.to(DEV), (7, 7), 1 / 16, 2, aligned)
    assert (out.float().cpu() - ref).abs().max().item() < 0.03


@pytest.mark.parametrize("C", [256, 64, 24])
def test_roi_align_fpn_matches_per_level_reference(C):
    """In-kernel FPN level assignment (one workgroup per RoI row) == map_levels + per-level reference RoIAlign."""
    from aiforearth_api_platform_amd.ops.detection import multiscale_roi_align, roi_align_fpn
    g = torch.Generator().manual_seed(1)
    feats = [torch.randn(2, 160 // s, 160 // s, C, generator=g).bfloat16() for s in (1, 2, 4, 8)]
    scales = [1 / 4, 1 / 8, 1 / 16, 1 / 32]
    R = 300
    x1 = torch.rand(R, generator=g) * 600
    y1 = torch.rand(R, generator=g) * 600
    wh = torch.rand(R, 2, generator=g) ** 2 * 600 + 1  # small boxes (P2) through large ones (P5)
    rois = torch.stack([torch.randint(0, 2, (R,), generator=g).float(), x1, y1, x1 + wh[:, 0], y1 + wh[:, 1]], 1)
    ref = multiscale_roi_align([f.float() for f in feats], scales, rois, (7, 7), 2)
    out = roi_align_fpn([f.to(DEV) for f in feats], scales, rois.to(DEV), (7, 7), 2)
    assert out.shape == (R, 7, 7, C)
    assert (out.float().cpu() - ref).abs().max().item() < 0.03


def test_crop_resize():
    img = torch.randint(0, 256, (2, 300, 400, 3), dtype=torch.uint8)
    boxes = torch.tensor([[0, 10.5, 20, 200, 220], [1, 0, 0, 400, 300], [1, 350, 250, 399, 299]])
    ref = crop_resize_reference(img, boxes, (224, 224))
    out = crop_resize_nhwc(img.to(DEV), boxes.to(DEV), (224, 224))
    assert (out.float().cpu() - ref).abs().max().item() < 0.03


@pytest.mark.parametrize("with_prob", [False, True])
def test_tile_stitch(with_prob):
    grid = TileGrid(300, 260, 64, 48)
    C = 7
    g = torch.Generator().manual_seed(3)
    tiles = torch.randn(grid.nty, grid.ntx, 64, 64, C, generator=g).bfloat16()
    cls_ref, prob_ref = stitch_reference(tiles.float(), grid, with_prob=with_prob)
    cls, prob = tile_stitch(tiles.to(DEV), grid, with_prob=with_prob)
    agree = (cls.cpu() == cls_ref).float().mean().item()
    assert agree > 0.995, agree  # ties / bf16 rounding at near-equal logits may flip a few pixels
    if with_prob:
        assert (prob.float().cpu() - prob_ref).abs().max().item() < 0.02
    ty0, ty1 = grid.tile_rows_for(100, 180)
    cls2, _ = tile_stitch(tiles[ty0:ty1].to(DEV), grid, row0=100, rows=80, ty0=ty0)
    assert torch.equal(cls2.cpu(), cls.cpu()[100:180])


@pytest.mark.parametrize("B,h,w,k", [(2, 40, 40, 1000), (3, 10, 10, 300), (1, 5, 7, 105)])
def test_rpn_decode_matches_reference(B, h, w, k):
    """Fused RPN decode (gather + decode + clip + sigmoid + min-size mask into the all-level buffers) vs the
    PyTorch formulation of the same op on the CPU."""
    from aiforearth_api_platform_amd.ops.detection import rpn_decode_into

    A = 3
    torch.manual_seed(3)
    head = (torch.randn(B, h, w, 16) * 2).to(torch.bfloat16)
    head[..., A + 2: 5 * A: 4] *= 3  # some dw beyond the clip
    anchors = torch.rand(h * w * A, 4) * 300
    anchors[:, 2:] += anchors[:, :2] + torch.rand(h * w * A, 2) * 5  # includes tiny boxes
    idx = head[..., :A].float().reshape(B, -1).topk(min(k, h * w * A), dim=1)[1]
    k = idx.shape[1]
    KT, off = k + 17, 9
    outs = []
    for dev in ("cpu", DEV):
        hd = head.to(dev) if dev != "cpu" else head.float()
        bx = torch.full((B, KT, 4), 7.0, device=dev)
        sc = torch.full((B, KT), 7.0, device=dev)
        lv = torch.full((B, KT), 7.0, device=dev)
        rpn_decode_into(hd, idx.to(dev), anchors.to(dev), A, bx, sc, lv, off, 2, (320, 300), 1.0)
        outs.append((bx.cpu(), sc.cpu(), lv.cpu()))
    (b0, s0, l0), (b1, s1, l1) = outs
    assert torch.allclose(b0, b1, rtol=1e-4, atol=1e-2)
    assert torch.allclose(s0, s1, rtol=1e-4, atol=1e-5)
    assert torch.equal(l0, l1)
    assert (b1[:, :off] == 7.0).all() and (b1[:, off + k:] == 7.0).all()


@pytest.mark.parametrize("B,h,w,k,ties", [(2, 160, 160, 1000, False), (3, 40, 40, 1000, True), (1, 5, 7, 105, False),
                                           (2, 20, 20, 1, True)])
def test_rpn_topk_selects_the_k_largest(B, h, w, k, ties):
    """Graph-safe RPN top-k (radix select, one workgroup per image) vs torch.topk on the fp32 CPU copy: the same
    multiset of selected values (exact; unique even with ties), distinct in-range indices, every unselected value
    <= every selected one; and a deterministic output (two calls bitwise equal)."""
    from aiforearth_api_platform_amd.ops.detection import rpn_topk

    A = 3
    torch.manual_seed(11)
    head = torch.randn(B, h, w, 16) * 3
    if ties:
        head = head.round()  # a handful of distinct values: many ties at the k-th
    head[0, 0, 0, 0] = float("-inf")
    head = head.to(torch.bfloat16)
    idx = rpn_topk(head.to(DEV), A, k)
    assert torch.equal(idx, rpn_topk(head.to(DEV), A, k))
    idx = idx.cpu()
    logits = head[..., :A].float().reshape(B, -1)
    ref = logits.topk(k, dim=1)[0]
    assert idx.shape == (B, k) and int(idx.min()) >= 0 and int(idx.max()) < h * w * A
    for b in range(B):
        assert idx[b].unique().numel() == k
        got = logits[b, idx[b]]
        assert torch.equal(got.sort(descending=True)[0], ref[b])
        rest = torch.ones(h * w * A, dtype=torch.bool)
        rest[idx[b]] = False
        if rest.any():
            assert logits[b, rest].max() <= got.min()


@pytest.mark.parametrize("B,h,w,k", [(2, 40, 40, 1000), (1, 20, 20, 7)])
def test_rpn_topk_tied_logits_same_set_as_cpu(B, h, w, k):
    """Deliberately tied logits (a few distinct values): the HIP selection is the SET of the k largest by
    (value desc, index asc) — the CPU path's stable-sort set — so proposals (and NMS winners among equal scores)
    do not depend on the backend."""
    from aiforearth_api_platform_amd.ops.detection import rpn_topk

    A = 3
    torch.manual_seed(3)
    head = (torch.randn(B, h, w, 16) * 1.5).round().to(torch.bfloat16)
    got = rpn_topk(head.to(DEV), A, k).cpu()
    ref = rpn_topk(head, A, k)  # CPU: stable descending sort, first k
    for b in range(B):
        assert set(got[b].tolist()) == set(ref[b].tolist())
        # output order: the keys above the k-th value, then the taken ties, each in index order
        vals = head[b, ..., :A].float().reshape(-1)[got[b]]
        kth = vals.min()
        above, tie = got[b][vals > kth], got[b][vals == kth]
        assert torch.equal(above, above.sort()[0]) and torch.equal(tie, tie.sort()[0])


@pytest.mark.parametrize("B,N,groups", [(32, 4300, "lvl"), (2, 3000, "label"), (3, 1, "lvl"), (2, 8192, "label")])
def test_sort_select_matches_reference(B, N, groups):
    """One-launch NMS-stage sort + select (sort_select_kernel) vs the PyTorch form: sorted scores exact (ties in index
    order), gathered boxes / offset boxes / groups / labels exact, valid counts exact."""
    from aiforearth_api_platform_amd.ops.detection import sort_select

    torch.manual_seed(9)
    sc = torch.rand(B, N)
    sc[:, ::7] = -1.0
    sc[:, 1::11] = 0.25
    bx = torch.rand(B, N, 4) * 600
    scale = 641.0
    if groups == "lvl":
        lvl = torch.randint(0, 5, (B, N)).float()
        got = sort_select(sc.to(DEV), bx.to(DEV), scale, groups=lvl.to(DEV))
        ref = sort_select(sc, bx, scale, groups=lvl)
    else:
        got = sort_select(sc.to(DEV), bx.to(DEV), scale, group_mod=3, want_labels=True)
        ref = sort_select(sc, bx, scale, group_mod=3, want_labels=True)
    for g, r in zip(got, ref):
        assert torch.equal(g.cpu(), r), (g.cpu(), r)


def test_gather_keep_matches_reference():
    from aiforearth_api_platform_amd.ops.detection import gather_keep

    torch.manual_seed(2)
    B, N, K = 3, 500, 100
    bx, sc, lb = torch.rand(B, N, 4), torch.rand(B, N), torch.randint(1, 4, (B, N))
    keep = torch.randint(0, N, (B, K), dtype=torch.int32)
    keep[:, 60:] = -1
    got = gather_keep(keep.to(DEV), bx.to(DEV), sc.to(DEV), lb.to(DEV), rois=True)
    ref = gather_keep(keep, bx, sc, lb, rois=True)
    for g, r in zip(got, ref):
        assert torch.equal(g.cpu(), r)
    assert (got[0][:, 60:] == 0).all()
    # the RoIAlign rows: (image, box) per kept row, from the same launch
    assert got[3].shape == (B * K, 5) and torch.equal(got[3][:, 0].cpu(), torch.arange(B).repeat_interleave(K).float())


@pytest.mark.parametrize("B,N", [(32, 4300), (2, 8192), (3, 1), (4, 3000)])
def test_argsort_desc_rows_matches_sort(B, N):
    """Graph-safe row sort (bitonic in LDS) vs torch.sort on the CPU: the gathered scores equal the descending sorted
    values exactly, the order is a permutation, and ties (-1 padding scores, repeated values) come in index order."""
    from aiforearth_api_platform_amd.ops.detection import argsort_desc_rows

    torch.manual_seed(5)
    sc = torch.rand(B, N)
    sc[:, ::7] = -1.0                       # invalid proposals
    sc[:, 1::11] = 0.5                      # ties
    order = argsort_desc_rows(sc.to(DEV)).cpu()
    assert order.shape == (B, N) and order.dtype == torch.long
    for b in range(B):
        assert torch.equal(order[b].sort()[0], torch.arange(N))
        got = sc[b, order[b]]
        assert torch.equal(got, sc[b].sort(descending=True)[0])
        same = got[1:] == got[:-1]
        assert bool((order[b, 1:][same] > order[b, :-1][same]).all())


@pytest.mark.parametrize("B,R,nc", [(2, 1000, 4), (3, 37, 7)])
def test_det_decode_matches_reference(B, R, nc):
    """Fused box-head postprocess (softmax + per-class decode + clip + validity mask) vs its PyTorch form."""
    from aiforearth_api_platform_amd.ops.detection import det_decode

    torch.manual_seed(4)
    ldp = (5 * nc + 3) // 4 * 4
    pred = torch.randn(B, R, ldp) * 2
    pred[..., nc:] *= 0.5
    props = torch.rand(B, R, 4) * 200
    props[..., 2:] += props[..., :2] + torch.rand(B, R, 2) * 100
    count = torch.randint(R // 2, R + 1, (B,), dtype=torch.int32)
    wts = (10.0, 10.0, 5.0, 5.0)
    ref = det_decode(pred, props, count, nc, wts, (320, 300), 0.05)
    got = det_decode(pred.to(DEV).bfloat16().float(), props.to(DEV), count.to(DEV), nc, wts, (320, 300), 0.05)
    ref2 = det_decode(pred.bfloat16().float(), props, count, nc, wts, (320, 300), 0.05)
    b0, s0, l0 = ref2
    b1, s1, l1 = [t.cpu() for t in got]
    assert torch.allclose(b0, b1, rtol=1e-4, atol=1e-2)
    assert torch.allclose(s0, s1, rtol=1e-4, atol=1e-5)
    assert torch.equal(l0, l1)
    assert ref[0].shape == b1.shape


@pytest.mark.parametrize("cfg", [1, 2, 4, 5, 7, 8])
@pytest.mark.parametrize("shape", [(2, 32, 32, 64, 64, 32), (3, 16, 16, 64, 128, 32), (1, 16, 32, 128, 256, 16)])
def test_conv_fused_groupnorm_stats(cfg, shape, monkeypatch):
    """GroupNorm statistics from the conv epilogue (conv2d_gn_nhwc -> group_norm_nhwc(stats=...)) == the
    norm's own statistics pass over the stored conv output."""
    from aiforearth_api_platform_amd.ops import conv as convmod
    from aiforearth_api_platform_amd.ops.conv import conv2d_gn_nhwc, pack_conv

    n, h, w, cin, cout, g = shape
    monkeypatch.setattr(convmod, "tuned_tile", lambda *a: cfg)
    torch.manual_seed(5)
    pc = pack_conv(torch.randn(cout, cin, 3, 3) / (9 * cin) ** 0.5, torch.randn(cout) * 0.3, pad=1).to(DEV)
    x = torch.randn(n, h, w, cin, device=DEV).to(torch.bfloat16)
    gamma, beta = torch.rand(cout, device=DEV) + 0.5, torch.randn(cout, device=DEV) * 0.1
    y, st = conv2d_gn_nhwc(x, pc, g)
    assert st is not None
    a = group_norm_nhwc(y, gamma, beta, groups=g, relu=True, stats=st)
    b = group_norm_nhwc(y, gamma, beta, groups=g, relu=True)
    torch.cuda.synchronize()
    assert (a.float() - b.float()).abs().max().item() <= 0.02


@pytest.mark.parametrize("cfg", [6, 9])
@pytest.mark.parametrize("shape", [(2, 24, 32, 64, 256, 32), (1, 48, 16, 128, 512, 32), (3, 16, 48, 256, 256, 64),
                                   (2, 24, 32, 64, 384, 48)])
def test_conv256_fused_groupnorm_stats(cfg, shape, monkeypatch):
    """The 256-wide ping-pong configs (6: 256-pixel, 9: 192-pixel tiles) emit the GroupNorm statistics from their
    epilogue too: normalizing with them == the norm's own statistics pass over the stored output, and both == an fp32
    PyTorch GroupNorm of it; the last shape has a 128-channel tail tile (Kout 384)."""
    from aiforearth_api_platform_amd.ops import conv as convmod
    from aiforearth_api_platform_amd.ops.conv import conv2d_gn_nhwc, pack_conv

    n, h, w, cin, cout, g = shape
    monkeypatch.setattr(convmod, "tuned_tile", lambda *a: cfg)
    torch.manual_seed(6)
    pc = pack_conv(torch.randn(cout, cin, 3, 3) / (9 * cin) ** 0.5, torch.randn(cout) * 0.3 + 2.0, pad=1).to(DEV)
    x = torch.randn(n, h, w, cin, device=DEV).to(torch.bfloat16)
    gamma, beta = torch.rand(cout, device=DEV) + 0.5, torch.randn(cout, device=DEV) * 0.1
    y, st = conv2d_gn_nhwc(x, pc, g)
    assert st is not None
    # the finalized affine (a, b) from the epilogue statistics == the fp32 GroupNorm of the stored output (any C)
    from aiforearth_api_platform_amd.ops.norm import group_norm_affine

    ab = group_norm_affine(st, gamma, beta, n, h * w, cout, g).clone()
    ref = F.group_norm(y.float().permute(0, 3, 1, 2), g, gamma, beta).permute(0, 2, 3, 1)
    got = y.float() * ab[:, None, None, :, 0] + ab[:, None, None, :, 1]
    torch.cuda.synchronize()
    assert (got - ref).abs().max().item() <= 0.03
    if (cout // 8) <= 256 and 256 % (cout // 8) == 0:  # (the apply kernel's channel limit)
        a = group_norm_nhwc(y, gamma, beta, groups=g, relu=True, stats=st)
        b = group_norm_nhwc(y, gamma, beta, groups=g, relu=True)
        torch.cuda.synchronize()
        assert (a.float() - b.float()).abs().max().item() <= 0.02
        assert (a.float() - F.relu(ref)).abs().max().item() <= 0.03


@pytest.mark.parametrize("shape", [(2, 32, 32, 64, 64, 32), (1, 16, 24, 128, 256, 16)])
def test_groupnorm_apply_fused_maxpool(shape, monkeypatch):
    """GN apply + ReLU that also writes the 2x2/2 max-pool (the U-Net encoder's skip + next input) == GN then
    max-pool, with the GN output in a channel slice of a wider concat buffer."""
    from aiforearth_api_platform_amd.ops import conv as convmod
    from aiforearth_api_platform_amd.ops.conv import conv2d_gn_nhwc, pack_conv

    n, h, w, cin, cout, g = shape
    monkeypatch.setattr(convmod, "tuned_tile", lambda *a: 1)
    torch.manual_seed(6)
    pc = pack_conv(torch.randn(cout, cin, 3, 3) / (9 * cin) ** 0.5, torch.randn(cout) * 0.3, pad=1).to(DEV)
    x = torch.randn(n, h, w, cin, device=DEV).to(torch.bfloat16)
    gamma, beta = torch.rand(cout, device=DEV) + 0.5, torch.randn(cout, device=DEV) * 0.3
    y, st = conv2d_gn_nhwc(x, pc, g)
    assert st is not None
    cat = torch.full((n, h, w, cout + 64), 7.0, device=DEV, dtype=torch.bfloat16)
    pooled = torch.empty(n, h // 2, w // 2, cout, device=DEV, dtype=torch.bfloat16)
    a = group_norm_nhwc(y, gamma, beta, groups=g, relu=True, stats=st, out=cat[..., :cout], pool_out=pooled)
    b = group_norm_nhwc(y, gamma, beta, groups=g, relu=True, stats=st)
    ref_pool = F.max_pool2d(b.permute(0, 3, 1, 2).float(), 2, 2).permute(0, 2, 3, 1)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert (cat[..., cout:] == 7.0).all()
    assert torch.equal(pooled.float(), ref_pool)


def test_crop_resize_u8_and_gpu_resize_match_fp32_reference():
    """K5/K7 uint8 crop-resize (ensemble wire format) and whole-frame GPU resize vs the fp32 reference."""
    from aiforearth_api_platform_amd.ops.detection import crop_resize_u8, crop_resize_u8_reference, resize_u8
    torch.manual_seed(3)
    img = torch.randint(0, 256, (2, 150, 190, 3), dtype=torch.uint8)
    boxes = torch.tensor([[0, 10.0, 5.0, 120.0, 140.0], [1, 0.0, 0.0, 190.0, 150.0], [0, 50.5, 60.2, 51.0, 61.0]])
    ref = crop_resize_u8_reference(img, boxes, (64, 48))
    out = crop_resize_u8(img.to(DEV), boxes.to(DEV), (64, 48)).cpu()
    assert out.shape == ref.shape and (out.int() - ref.int()).abs().max().item() <= 1
    frames = torch.randint(0, 256, (3, 480, 640, 3), dtype=torch.uint8)
    full = torch.tensor([[i, 0.0, 0.0, 640.0, 480.0] for i in range(3)])
    r = resize_u8(frames.to(DEV), (224, 224)).cpu()
    assert (r.int() - crop_resize_u8_reference(frames, full, (224, 224)).int()).abs().max().item() <= 1


def test_resizing_servable_scales_boxes_to_frame_coordinates():
    from aiforearth_api_platform_amd.models import zoo
    frames = torch.randint(0, 256, (2, 480, 640, 3), dtype=torch.uint8, device=DEV)
    s = zoo.megadetector(DEV, model_hw=(256, 256), box_score_thresh=0.0)
    boxes, scores, labels, count = s(frames)
    plain = zoo.megadetector(DEV, box_score_thresh=0.0)
    from aiforearth_api_platform_amd.ops.detection import resize_u8
    b2, _, _, c2 = plain(resize_u8(frames, (256, 256)))
    assert torch.equal(count, c2)
    k = int(count[0, 0])
    assert torch.allclose(boxes[0, :k], b2[0, :k] * torch.tensor([2.5, 1.875, 2.5, 1.875], device=DEV), atol=1e-3)


@pytest.mark.parametrize("cfg,shape", [(6, (2, 32, 32)), (9, (3, 24, 16)), (10, (1, 40, 20)), (6, (1, 10, 10))])
def test_conv_fused_rpn_head_matches_two_convs(cfg, shape):
    """The 16-channel 1x1 head run in the 256-wide conv's epilogue (``conv2d_head_nhwc``, the RPN conv + head) against
    the two separate convs (same bf16 intermediate; only the head's fp32 summation order differs) and against fp32
    PyTorch of the same bf16 weights. The last shape has a partial pixel tile (M % BM != 0)."""
    from aiforearth_api_platform_amd.ops.conv import conv2d_head_nhwc, conv2d_nhwc, pack_conv

    n, h, w = shape
    g = torch.Generator().manual_seed(11)
    pc = pack_conv(torch.randn(256, 256, 3, 3, generator=g) * 0.02, torch.randn(256, generator=g) * 0.1, pad=1).to(DEV)
    hw = torch.zeros(16, 256, 1, 1)
    hw[:15] = torch.randn(15, 256, 1, 1, generator=g) * 0.05
    hb = torch.zeros(16)
    hb[:15] = torch.randn(15, generator=g) * 0.1
    head = pack_conv(hw, hb).to(DEV)
    x = (torch.randn(n, h, w, 256, generator=g)).to(DEV, torch.bfloat16)
    fused = conv2d_head_nhwc(x, pc, head, tile_cfg=cfg)
    t = conv2d_nhwc(x, pc, relu=True, tile_cfg=cfg)
    two = conv2d_nhwc(t, head)
    torch.cuda.synchronize()
    assert fused.shape == (n, h, w, 16)
    err = (fused.float() - two.float()).abs().max().item()
    assert err <= 1e-2 * two.float().abs().max().item() + 1e-3, err
    # fp32 reference of the same (bf16-rounded) weights
    w1 = pc.w_packed[:256, :2304].float().reshape(256, 3, 3, 256).permute(0, 3, 1, 2)
    ref_t = F.relu(F.conv2d(x.float().permute(0, 3, 1, 2), w1, pc.bias[:256], padding=1))
    ref = F.conv2d(ref_t, head.w_packed[:16, :256].float()[:, :, None, None], head.bias[:16])
    ref = ref.permute(0, 2, 3, 1)
    err = (fused.float() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item() + 1e-2, err

