"""The fp16 element type of the K1 conv (f16 MFMA, ``ai4e_conv2d_f16_fwd``), the fp16 pool / s2d preprocess
kernels and the fp16 ResNet-50 built from them (the stage graph's crop classifier, ``zoo.crop_classifier``),
each against a plain fp32 PyTorch reference of the same op; and the N:M stage graph's detector -> classifier
path (HIP graphs for both stages) against the same stages run eagerly."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from aiforearth_api_platform_amd import _build
    from aiforearth_api_platform_amd.ops import _ext
    _build.build_kernels()
    _ext.lib()


def _ref(x, wq, b, s, p, res=None, relu=False):
    y = F.conv2d(x.float().permute(0, 3, 1, 2), wq, b.float(), stride=s, padding=p).permute(0, 2, 3, 1)
    if res is not None:
        y = y + res.float()
    return F.relu(y) if relu else y


CASES = [
    (2, 56, 56, 64, 64, 1, 1, 0),
    (2, 28, 28, 128, 128, 3, 1, 1),
    (3, 28, 28, 256, 512, 1, 2, 0),
    (2, 7, 7, 512, 2048, 1, 1, 0),
    (2, 112, 112, 16, 64, 4, 1, 1),     # s2d stem shape (4x4 over 16 channels)
    (1, 33, 17, 40, 96, 3, 1, 1),       # ragged M, C = 40
]


# (the 256-wide configs 6 / 9 need Cin % 64 == 0 and Cout % 8 == 0: those combinations are not generated)
@pytest.mark.parametrize("case,tile", [(c, t) for c in CASES for t in (-1, 1, 3, 6, 8, 9)
                                       if t not in (6, 9) or (c[3] % 64 == 0 and c[4] % 8 == 0)])
def test_conv_f16_matches_fp32(case, tile):
    from aiforearth_api_platform_amd.ops.conv import conv2d_nhwc, pack_conv
    n, h, w, cin, cout, k, s, p = case
    torch.manual_seed(11)
    wt = torch.randn(cout, cin, k, k) / (cin * k * k) ** 0.5
    b = torch.randn(cout) * 0.1
    pc = pack_conv(wt, b, stride=s, pad=p).to(DEV).cast(torch.float16)
    assert pc.w_packed.dtype == torch.float16
    x = torch.randn(n, h, w, pc.cin_pad, device=DEV).half()
    x[..., cin:] = 0
    oh, ow = pc.out_hw(h, w)
    res = torch.randn(n, oh, ow, cout, device=DEV).half()
    y = conv2d_nhwc(x, pc, residual=res, relu=True, tile_cfg=tile)
    assert y.dtype == torch.float16
    wq = pc.w_packed[:cout, :k * k * pc.cin_pad].float().reshape(cout, k, k, pc.cin_pad).permute(0, 3, 1, 2)
    ref = _ref(x, wq, pc.bias[:cout], s, p, res, True)
    err = (y.float() - ref).abs().max().item()
    # fp16 keeps 3 more mantissa bits than bf16: the bound is 8x tighter than the bf16 tests' 0.02
    assert err <= 0.0025 * ref.abs().max().item() + 0.0025, err


def test_conv_dtype_mismatch_is_refused():
    from aiforearth_api_platform_amd.ops.conv import conv2d_nhwc, pack_conv
    pc = pack_conv(torch.randn(64, 64, 1, 1), torch.zeros(64)).to(DEV)
    with pytest.raises(TypeError):
        conv2d_nhwc(torch.randn(1, 8, 8, 64, device=DEV).half(), pc)  # bf16 weights, fp16 activations


def test_pools_and_preprocess_f16():
    from aiforearth_api_platform_amd.ops.pool import global_avgpool_nhwc, maxpool2d_nhwc, preprocess_s2d_u8
    img = torch.randint(0, 256, (3, 64, 48, 3), dtype=torch.uint8, device=DEV)
    a = preprocess_s2d_u8(img, dtype=torch.float16)
    b = preprocess_s2d_u8(img.cpu())  # fp32 torch path
    assert a.dtype == torch.float16
    assert (a.float().cpu() - b).abs().max().item() < 2e-3
    x = torch.randn(2, 57, 55, 64, device=DEV).half()
    mp = maxpool2d_nhwc(x)
    assert mp.dtype == torch.float16
    assert torch.equal(mp.float(), F.max_pool2d(x.float().permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1))
    ap = global_avgpool_nhwc(x)
    assert (ap.float() - x.float().mean(dim=(1, 2), keepdim=True)).abs().max().item() < 2e-3


def test_resnet50_fp16_beats_bf16_against_fp32():
    from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50
    from aiforearth_api_platform_amd.ops.pool import preprocess_u8
    m = resnet50(num_classes=200, seed=4)
    img = torch.randint(0, 256, (16, 224, 224, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(4))
    x = preprocess_u8(img)[..., :3].permute(0, 3, 1, 2).float().to(DEV)
    with torch.no_grad():
        ref = m.to(DEV).float()(x)
    m = m.cpu()
    f16 = FusedResNet(m, device=DEV, dtype=torch.float16)
    bf16 = FusedResNet(m, device=DEV)
    o16 = f16.forward_u8(img.to(DEV))
    o_bf = bf16.forward_u8(img.to(DEV))
    assert o16.dtype == torch.float32 and torch.isfinite(o16).all()
    rel16 = ((o16 - ref).norm() / ref.norm()).item()
    relbf = ((o_bf - ref).norm() / ref.norm()).item()
    assert rel16 < 0.02, rel16
    assert rel16 < relbf, (rel16, relbf)
    assert (o16.argmax(1) == ref.argmax(1)).float().mean() >= 0.9


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_stage_graph_graphs_match_eager(dtype):
    """StageGraphPipeline, single process: detection + crop selection + crop-resize + compaction in one HIP
    graph, the crop classifier in per-bucket graphs — equal to the same callables run eagerly."""
    from aiforearth_api_platform_amd.models import zoo
    from aiforearth_api_platform_amd.models.faster_rcnn import DetectorConfig, FasterRCNN
    from aiforearth_api_platform_amd.runtime.pipeline import PipelineConfig, StageGraphPipeline
    det = FasterRCNN(DetectorConfig(box_score_thresh=0.0, detections_per_img=20), seed=0, device=DEV)
    cls = zoo.crop_classifier(DEV, 30, 1, dtype)
    cfg = PipelineConfig(score_thresh=0.0, class_id=None, max_crops_per_image=3)
    p = StageGraphPipeline(det.forward_u8, cls, torch.device(DEV), cfg)
    imgs = [torch.randint(0, 256, (4, 256, 256, 3), dtype=torch.uint8, device=DEV) for _ in range(2)]
    got = p.run_batches(imgs)
    for im, (boxes, scores, valid, res) in zip(imgs, got):
        _, b2, s2, v2, crops, count = p._detect_crop_compact(im)
        n = int(count)
        assert torch.equal(valid, v2) and torch.allclose(boxes, b2) and torch.allclose(scores, s2)
        assert res.shape == (n, 2) and n == int(valid.sum())
        bucket = next(b for b in p.BUCKETS if b >= n)  # the graph ran the bucket-padded batch
        pad = torch.zeros(bucket, *crops.shape[1:], dtype=crops.dtype, device=crops.device)
        pad[:n] = crops[:n]
        eager = p._classify_static(pad)[:n]
        assert torch.equal(res[:, 0], eager[:, 0])
        assert torch.allclose(res[:, 1], eager[:, 1], atol=1e-3)
