"""HIP kernel numerics vs PyTorch fp32 references (GPU box only)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from aiforearth_api_platform_amd.ops import _ext
from aiforearth_api_platform_amd.ops.conv import conv2d_nhwc, pack_conv
from aiforearth_api_platform_amd.ops.pool import global_avgpool_nhwc, maxpool2d_nhwc, preprocess_u8

DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from aiforearth_api_platform_amd import _build
    _build.build_kernels()
    _ext.lib()


def ref_conv(x, w, b, stride, pad, res=None, relu=False):
    y = F.conv2d(x.float().permute(0, 3, 1, 2), w.float(), b.float(), stride=stride, padding=pad).permute(0, 2, 3, 1)
    if res is not None:
        y = y + res.float()
    return F.relu(y) if relu else y


CASES = [
    # n, h, w, cin, cout, k, stride, pad
    (2, 56, 56, 64, 64, 1, 1, 0),
    (2, 56, 56, 64, 64, 3, 1, 1),
    (2, 56, 56, 64, 256, 1, 1, 0),
    (2, 56, 56, 128, 128, 3, 2, 1),
    (3, 28, 28, 256, 512, 1, 2, 0),
    (2, 7, 7, 512, 2048, 1, 1, 0),
    (2, 112, 112, 3, 64, 7, 2, 3),      # stem (C padded to 8)
    (5, 1, 1, 2048, 1000, 1, 1, 0),     # classifier, M tiny, Kout % 64 != 0
    (1, 33, 17, 40, 96, 3, 1, 1),       # ragged M / C=40 (not multiple of 32)
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("epi", ["plain", "relu", "res_relu"])
def test_conv_igemm(case, epi):
    n, h, w, cin, cout, k, s, p = case
    torch.manual_seed(0)
    wt = torch.randn(cout, cin, k, k) / (cin * k * k) ** 0.5
    b = torch.randn(cout) * 0.1
    pc = pack_conv(wt, b, stride=s, pad=p).to(DEV)
    x = torch.randn(n, h, w, pc.cin_pad, device=DEV).to(torch.bfloat16)
    x[..., cin:] = 0
    oh, ow = pc.out_hw(h, w)
    res = torch.randn(n, oh, ow, cout, device=DEV).to(torch.bfloat16) if epi == "res_relu" else None
    y = conv2d_nhwc(x, pc, residual=res, relu=epi != "plain")
    torch.cuda.synchronize()
    wq = pc.w_packed[:cout, :k * k * pc.cin_pad].float().reshape(cout, k, k, pc.cin_pad).permute(0, 3, 1, 2)
    ref = ref_conv(x, wq, b.to(DEV), s, p, res, epi != "plain")
    err = (y.float() - ref).abs().max().item()
    assert err <= 0.02 * ref.abs().max().item() + 0.02, err


@pytest.mark.parametrize("tile", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10])
def test_conv_tile_configs(tile):
    torch.manual_seed(1)
    wt = torch.randn(256, 64, 3, 3) / 24
    pc = pack_conv(wt, torch.zeros(256), pad=1).to(DEV)
    x = torch.randn(2, 20, 20, 64, device=DEV).to(torch.bfloat16)
    y = conv2d_nhwc(x, pc, tile_cfg=tile)
    ref = ref_conv(x, pc.w_packed[:256, :576].float().reshape(256, 3, 3, 64).permute(0, 3, 1, 2), torch.zeros(256, device=DEV), 1, 1)
    assert (y.float() - ref).abs().max().item() < 0.02 * ref.abs().max().item() + 0.02


@pytest.mark.parametrize("tile", [7, 8])
@pytest.mark.parametrize("shape", [(3, 14, 14, 256, 256, 3, 1, 1), (2, 7, 7, 512, 512, 3, 1, 1),
                                   (5, 14, 14, 256, 1024, 1, 1, 0), (1, 9, 11, 64, 136, 1, 1, 0)])
def test_conv_occupancy3_configs_residual(tile, shape):
    """3-stage ring (two-pass LDS epilogue, residual loaded per pass): ragged M, residual + ReLU."""
    n, h, w, cin, cout, k, st, pd = shape
    torch.manual_seed(7)
    wt = torch.randn(cout, cin, k, k) / (cin * k * k) ** 0.5
    b = torch.randn(cout) * 0.1
    pc = pack_conv(wt, b, stride=st, pad=pd).to(DEV)
    x = torch.randn(n, h, w, cin, device=DEV).to(torch.bfloat16)
    oh, ow = pc.out_hw(h, w)
    res = torch.randn(n, oh, ow, cout, device=DEV).to(torch.bfloat16)
    y = conv2d_nhwc(x, pc, residual=res, relu=True, tile_cfg=tile)
    wq = pc.w_packed[:cout, :k * k * cin].float().reshape(cout, k, k, cin).permute(0, 3, 1, 2)
    ref = ref_conv(x, wq, b.to(DEV), st, pd, res, True)
    assert (y.float() - ref).abs().max().item() <= 0.02 * ref.abs().max().item() + 0.02


CASES_256 = [
    # n, h, w, cin, cout, k, stride, pad  (256x256 ping-pong tile: C % 64 == 0, Cout % 8 == 0)
    (2, 56, 56, 64, 256, 1, 1, 0),      # one K tile (nk = 1)
    (3, 28, 28, 256, 512, 1, 2, 0),     # strided pointwise
    (2, 14, 14, 256, 256, 3, 1, 1),     # 3x3, 36 K tiles
    (2, 28, 28, 128, 128, 3, 2, 1),     # Cout < 256: half the channel tile masked
    (2, 7, 7, 512, 2048, 1, 1, 0),      # M = 98 < 256
    (1, 33, 17, 64, 264, 3, 1, 1),      # ragged M, Cout = 256 + 8
    (2, 14, 14, 128, 256, 1, 1, 0),     # nk = 2: only the checked tail
    (2, 14, 14, 192, 256, 1, 1, 0),     # nk = 3: one unchecked tile, then the tail
]


@pytest.mark.parametrize("tile", [6, 9, 10])  # 9: the same schedule with 192-pixel tiles; 10: its 3-phase form
@pytest.mark.parametrize("case", CASES_256)
@pytest.mark.parametrize("epi", ["plain", "res_relu"])
def test_conv_tile256(case, epi, tile):
    n, h, w, cin, cout, k, s, p = case
    torch.manual_seed(3)
    wt = torch.randn(cout, cin, k, k) / (cin * k * k) ** 0.5
    b = torch.randn(cout) * 0.1
    pc = pack_conv(wt, b, stride=s, pad=p).to(DEV)
    x = torch.randn(n, h, w, pc.cin_pad, device=DEV).to(torch.bfloat16)
    oh, ow = pc.out_hw(h, w)
    res = torch.randn(n, oh, ow, cout, device=DEV).to(torch.bfloat16) if epi == "res_relu" else None
    y = conv2d_nhwc(x, pc, residual=res, relu=epi != "plain", tile_cfg=tile)
    torch.cuda.synchronize()
    wq = pc.w_packed[:cout, :k * k * pc.cin_pad].float().reshape(cout, k, k, pc.cin_pad).permute(0, 3, 1, 2)
    ref = ref_conv(x, wq, b.to(DEV), s, p, res, epi != "plain")
    err = (y.float() - ref).abs().max().item()
    assert err <= 0.02 * ref.abs().max().item() + 0.02, err


SPLITK_CASES = [
    # n, h, w, cin, cout, k, stride, pad (K tiles of 64: 72, 36, 8, 4, 36)
    (250, 7, 7, 512, 512, 3, 1, 1),     # ResNet-50 layer4 3x3 at the serving batch
    (3, 14, 14, 512, 512, 3, 2, 1),     # layer4's strided 3x3
    (2, 7, 7, 512, 2048, 1, 1, 0),      # pointwise, M < BM
    (3, 28, 28, 256, 512, 1, 2, 0),     # strided pointwise
    (1, 33, 17, 256, 264, 3, 1, 1),     # ragged M, Cout = 256 + 8 (masked second channel tile)
]


@pytest.mark.parametrize("ks", [2])
@pytest.mark.parametrize("tile", [6, 9, 10])
@pytest.mark.parametrize("case", SPLITK_CASES)
def test_conv_splitk(case, tile, ks):
    """Split-K over two workgroups per output tile (arrival-ordered hand-off through the fp32 park) vs fp32, and
    bit-identical on a second launch (the counters were left zero; either split may arrive last)."""
    n, h, w, cin, cout, k, s, p = case
    torch.manual_seed(11)
    wt = torch.randn(cout, cin, k, k) / (cin * k * k) ** 0.5
    b = torch.randn(cout) * 0.1
    pc = pack_conv(wt, b, stride=s, pad=p).to(DEV)
    x = torch.randn(n, h, w, pc.cin_pad, device=DEV).to(torch.bfloat16)
    oh, ow = pc.out_hw(h, w)
    res = torch.randn(n, oh, ow, cout, device=DEV).to(torch.bfloat16)
    y = conv2d_nhwc(x, pc, residual=res, relu=True, tile_cfg=tile | ks << 4)
    y2 = conv2d_nhwc(x, pc, residual=res, relu=True, tile_cfg=tile | ks << 4)  # counters were left zero
    torch.cuda.synchronize()
    wq = pc.w_packed[:cout, :k * k * pc.cin_pad].float().reshape(cout, k, k, pc.cin_pad).permute(0, 3, 1, 2)
    ref = ref_conv(x, wq, b.to(DEV), s, p, res, True)
    err = (y.float() - ref).abs().max().item()
    assert err <= 0.02 * ref.abs().max().item() + 0.02, err
    assert torch.equal(y, y2)


def test_conv_splitk_streams_and_graph():
    """Concurrent split-K launches on two streams (separate workspaces) and a captured graph's replays."""
    torch.manual_seed(12)
    wt = torch.randn(512, 512, 3, 3) / (512 * 9) ** 0.5
    pc = pack_conv(wt, torch.randn(512) * 0.1, pad=1).to(DEV)
    xs = [torch.randn(64, 7, 7, 512, device=DEV).to(torch.bfloat16) for _ in range(2)]
    refs = [conv2d_nhwc(x, pc, relu=True, tile_cfg=9) for x in xs]
    streams = [torch.cuda.Stream() for _ in range(2)]
    outs = [[], []]
    torch.cuda.synchronize()
    for _ in range(8):
        for i in range(2):
            with torch.cuda.stream(streams[i]):
                outs[i].append(conv2d_nhwc(xs[i], pc, relu=True, tile_cfg=9 | 2 << 4))
    torch.cuda.synchronize()
    for i in range(2):
        for y in outs[i]:
            assert (y.float() - refs[i].float()).abs().max().item() <= 0.02 * refs[i].float().abs().max().item()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        conv2d_nhwc(xs[0], pc, relu=True, tile_cfg=9 | 2 << 4)
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        yg = conv2d_nhwc(xs[0], pc, relu=True, tile_cfg=9 | 2 << 4)
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        assert (yg.float() - refs[0].float()).abs().max().item() <= 0.02 * refs[0].float().abs().max().item()


def test_conv_channel_slices():
    """Write into a channel slice of a concat buffer and read from a channel slice."""
    torch.manual_seed(2)
    pc = pack_conv(torch.randn(32, 16, 3, 3) / 12, torch.randn(32), pad=1).to(DEV)
    big = torch.randn(1, 9, 9, 48, device=DEV).to(torch.bfloat16)
    xin = big[..., 16:32]
    out = torch.zeros(1, 9, 9, 64, device=DEV, dtype=torch.bfloat16)
    conv2d_nhwc(xin, pc, out=out, out_coff=32)
    ref = ref_conv(xin.contiguous(), pc.w_packed[:32, :144].float().reshape(32, 3, 3, 16).permute(0, 3, 1, 2),
                   pc.bias[:32], 1, 1)
    assert out[..., :32].abs().max().item() == 0
    assert (out[..., 32:].float() - ref).abs().max().item() < 0.05


def test_preprocess_maxpool_avgpool():
    img = torch.randint(0, 256, (3, 31, 29, 3), dtype=torch.uint8, device=DEV)
    y = preprocess_u8(img)
    import os
    os.environ["AI4E_KERNEL_BACKEND"] = "torch"
    try:
        ref = preprocess_u8(img.cpu())
    finally:
        os.environ["AI4E_KERNEL_BACKEND"] = "auto"
    assert (y.float().cpu() - ref).abs().max().item() < 0.02
    x = torch.randn(2, 57, 55, 64, device=DEV).to(torch.bfloat16)
    mp = maxpool2d_nhwc(x)
    mref = F.max_pool2d(x.float().permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    assert torch.equal(mp.float(), mref)
    ap = global_avgpool_nhwc(x)
    aref = x.float().mean(dim=(1, 2), keepdim=True)
    assert (ap.float() - aref).abs().max().item() < 0.01


def test_resnet50_fused_matches_reference():
    from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50
    torch.manual_seed(0)
    m = resnet50(seed=3)
    fused = FusedResNet(m, device=DEV)
    img = torch.randint(0, 256, (4, 224, 224, 3), dtype=torch.uint8)
    logits = fused(img.to(DEV)).cpu()
    x = preprocess_u8(img)[..., :3].permute(0, 3, 1, 2).float()
    with torch.no_grad():
        ref = m(x)
    rel = (logits - ref).norm() / ref.norm()
    assert rel < 0.05, rel.item()
    # top-1 agreement on most images
    assert (logits.argmax(1) == ref.argmax(1)).float().mean() >= 0.75


def test_resnet50_serving_batch_matches_reference():
    """At the serving batch (250) the forward takes the batch-250 tile-table entries, the whole-wave K1c chain
    grids and the 256x256 K1 tile: all of it against the fp32 PyTorch model on the same GPU."""
    from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50
    m = resnet50(seed=5)
    fused = FusedResNet(m, device=DEV)
    img = torch.randint(0, 256, (250, 224, 224, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(5))
    logits = fused(img.to(DEV)).float()
    x = preprocess_u8(img)[..., :3].permute(0, 3, 1, 2).float().to(DEV)
    with torch.no_grad():
        ref = m.to(DEV).float()(x)
    rel = (logits - ref).norm() / ref.norm()
    assert rel < 0.05, rel.item()
    assert (logits.argmax(1) == ref.argmax(1)).float().mean() >= 0.75


def test_engine_graph_replay_matches_eager():
    from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50
    from aiforearth_api_platform_amd.runtime.engine import InferenceEngine
    fused = FusedResNet(resnet50(seed=4), device=DEV)
    eng = InferenceEngine(fused.forward_u8, (64, 64, 3), 8, device=torch.device(DEV), use_graphs=True, buckets=[4, 8])
    eng.warmup()
    img = torch.randint(0, 256, (6, 64, 64, 3), dtype=torch.uint8)
    i_g, p_g = eng.run_sync(img)
    logits = fused(img.to(DEV))
    p, i = torch.topk(torch.softmax(logits.float(), 1), 5, 1)
    assert torch.equal(i_g[:, 0], i[:, 0].int().cpu())
    assert torch.allclose(p_g, p.cpu(), atol=1e-3)


def test_preprocess_s2d_matches_torch():
    from aiforearth_api_platform_amd.ops.pool import preprocess_s2d_u8, space_to_depth_shifted, IMAGENET_MEAN, IMAGENET_STD
    img = torch.randint(0, 256, (2, 36, 44, 3), dtype=torch.uint8)
    y = preprocess_s2d_u8(img.to(DEV)).float().cpu()
    x = (img.float() / 255 - torch.tensor(IMAGENET_MEAN)) / torch.tensor(IMAGENET_STD)
    ref = space_to_depth_shifted(x)
    assert y.shape == (2, 18, 22, 16)
    assert (y - ref).abs().max().item() < 0.02


def test_resnet_chunked_prefix_matches_full_batch_gpu():
    from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50
    m = resnet50(seed=6)
    img = torch.randint(0, 256, (12, 96, 96, 3), dtype=torch.uint8).to(DEV)
    ref = FusedResNet(m, device=DEV, chunk=None).forward_u8(img)
    for chunk in [(4, 3), (8, 7)]:
        out = FusedResNet(m, device=DEV, chunk=chunk).forward_u8(img)
        assert (out - ref).abs().max().item() < 2e-2, chunk


@pytest.mark.parametrize("shape,tile", [(s, t) for s in [(2, 40, 40, 256, 256), (3, 10, 14, 512, 256), (1, 6, 2, 64, 68)]
                                        for t in (1, 2, 4, 6) if t != 6 or s[4] % 8 == 0])  # (tile 6: Cout % 8 == 0)
def test_conv_residual_upsampled2x(tile, shape):
    """FPN top-down merge fused into the lateral 1x1: the epilogue reads the residual from the half-resolution
    map at (oh/2, ow/2) (nearest 2x upsample) == conv + explicitly upsampled residual."""
    n, h, w, cin, cout = shape
    torch.manual_seed(2)
    pc = pack_conv(torch.randn(cout, cin, 1, 1) / cin ** 0.5, torch.randn(cout) * 0.1).to(DEV)
    x = torch.randn(n, h, w, cin, device=DEV).to(torch.bfloat16)
    coarse = torch.randn(n, h // 2, w // 2, cout, device=DEV).to(torch.bfloat16)
    y = conv2d_nhwc(x, pc, residual=coarse, residual_up2=True, tile_cfg=tile)
    up = coarse.repeat_interleave(2, dim=1).repeat_interleave(2, dim=2).contiguous()
    ref = conv2d_nhwc(x, pc, residual=up, tile_cfg=tile)
    torch.cuda.synchronize()
    assert torch.equal(y, ref)
