"""Model-level checks on the GPU: U-Net, Faster-RCNN, detector->classifier, spatial segmentation."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda")


@pytest.fixture(autouse=True, scope="module")
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from aiforearth_api_platform_amd import _build
    from aiforearth_api_platform_amd.ops import _ext
    _build.build_kernels()
    _ext.lib()


def test_unet_gpu_matches_reference():
    from aiforearth_api_platform_amd.models.unet import LANDCOVER_MEAN, LANDCOVER_STD, FusedUNet, unet_landcover
    from aiforearth_api_platform_amd.ops.pool import preprocess_u8
    m = unet_landcover(seed=0)
    f = FusedUNet(m, device=DEV)
    img = torch.randint(0, 256, (2, 256, 256, 4), dtype=torch.uint8)
    out = f(img.to(DEV))[..., :7].float().cpu()
    x = preprocess_u8(img, LANDCOVER_MEAN, LANDCOVER_STD)[..., :4].permute(0, 3, 1, 2)
    with torch.no_grad():
        ref = m(x).permute(0, 2, 3, 1)
    rel = ((out - ref).norm() / ref.norm()).item()
    assert rel < 0.05, rel
    assert (out.argmax(-1) == ref.argmax(-1)).float().mean() > 0.9


def test_detector_gpu_invariants_and_features():
    from aiforearth_api_platform_amd.models.faster_rcnn import DetectorConfig, FasterRCNN
    from aiforearth_api_platform_amd.ops.detection import box_iou
    from aiforearth_api_platform_amd.ops.pool import preprocess_u8
    cfg = DetectorConfig(box_score_thresh=0.0)
    det_gpu = FasterRCNN(cfg, seed=0, device=DEV)
    det_cpu = FasterRCNN(cfg, seed=0, device="cpu")
    img = torch.randint(0, 256, (2, 256, 320, 3), dtype=torch.uint8)
    # backbone + FPN features agree with the fp32 CPU reference
    Pg = det_gpu.fpn(det_gpu.backbone_stages(preprocess_u8(img.to(DEV))))
    Pc = det_cpu.fpn(det_cpu.backbone_stages(preprocess_u8(img)))
    for a, b in zip(Pg, Pc):
        rel = ((a.float().cpu() - b).norm() / b.norm()).item()
        assert rel < 0.05, rel
    boxes, scores, labels, n = det_gpu(img.to(DEV))
    torch.cuda.synchronize()
    assert n.min().item() > 0
    for b in range(2):
        k = int(n[b])
        bb, ss, ll = boxes[b, :k].cpu(), scores[b, :k].cpu(), labels[b, :k].cpu()
        assert torch.all(ss[:-1] >= ss[1:])
        for c in range(1, 4):
            m = ll == c
            if m.sum() > 1:
                iou = box_iou(bb[m], bb[m])
                iou.fill_diagonal_(0)
                assert iou.max() <= cfg.box_nms_thresh + 1e-4


def test_detector_hip_graph_capture():
    from aiforearth_api_platform_amd.models.faster_rcnn import DetectorConfig, FasterRCNN
    det = FasterRCNN(DetectorConfig(), seed=0, device=DEV)
    x = torch.randint(0, 256, (2, 256, 256, 3), dtype=torch.uint8, device=DEV)
    ref = det(x)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        det(x)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        out = det(x)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out[3], ref[3]) and torch.allclose(out[1], ref[1])


def test_pipeline_and_spatial_single_gpu():
    from aiforearth_api_platform_amd.models.faster_rcnn import DetectorConfig, FasterRCNN
    from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50
    from aiforearth_api_platform_amd.models.unet import FusedUNet, unet_landcover
    from aiforearth_api_platform_amd.ops.stitch import TileGrid
    from aiforearth_api_platform_amd.runtime.pipeline import PipelineConfig, StageGraphPipeline
    from aiforearth_api_platform_amd.runtime.spatial import SpatialSegmenter
    det = FasterRCNN(DetectorConfig(box_score_thresh=0.0), seed=0, device=DEV)
    cls = FusedResNet(resnet50(num_classes=20, seed=1), device=DEV)
    p = StageGraphPipeline(det.forward_u8, cls.forward_u8, torch.device(DEV),
                           PipelineConfig(score_thresh=0.0, class_id=None))
    out = p.run_batches([torch.randint(0, 256, (2, 256, 256, 3), dtype=torch.uint8, device=DEV)])
    boxes, scores, valid, res = out[0]
    assert int(valid.sum()) == res.shape[0] > 0 and torch.all((res[:, 0] >= 0) & (res[:, 0] < 20))
    f = FusedUNet(unet_landcover(seed=0), device=DEV)
    seg = SpatialSegmenter(f.forward_u8, TileGrid(700, 600, 256, 224), 7, DEV, tile_batch=8)
    cls_map = seg.run(torch.randint(0, 256, (700, 600, 4), dtype=torch.uint8))
    assert cls_map.shape == (700, 600) and cls_map.max() < 7


def test_engine_buckets_resnet_fused_head():
    """Engine with batch buckets + the fused softmax/top-k head: a 5-image batch runs the 8-bucket graph and
    matches the eager FusedResNet logits' top-5."""
    from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50
    from aiforearth_api_platform_amd.runtime.engine import InferenceEngine

    m = FusedResNet(resnet50(seed=2), device=DEV)
    eng = InferenceEngine(m.forward_u8, (224, 224, 3), 32, device=DEV, head_fn=m.topk_u8, buckets=[8])
    eng.warmup()
    assert sorted({b for _, b in eng.graphs}) == [8, 32]
    host = torch.randint(0, 256, (5, 224, 224, 3), dtype=torch.uint8).pin_memory()
    res = eng.submit(host, list(range(5)))
    res.done.synchronize()
    ref = torch.topk(torch.softmax(m.forward_u8(host.to(DEV)).float(), 1), 5, 1)
    torch.cuda.synchronize()
    assert res.top_idx.shape == (5, 5)
    assert torch.allclose(res.top_prob, ref.values.cpu(), rtol=2e-2, atol=1e-4)
