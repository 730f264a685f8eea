"""Detector -> classifier pipeline over gloo (2 CPU ranks) == local single-process pipeline."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from aiforearth_api_platform_amd.runtime.pipeline import DetectClassifyPipeline, PipelineConfig, select_crops, stage_transition

CFG = PipelineConfig(crop_hw=(32, 32), score_thresh=0.0, class_id=None, max_crops_per_image=3)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stages():
    from aiforearth_api_platform_amd.models.faster_rcnn import DetectorConfig, FasterRCNN
    from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50
    det = FasterRCNN(DetectorConfig(pre_nms_top_n=100, post_nms_top_n=50, detections_per_img=10,
                                    box_score_thresh=0.0), seed=0)
    cls = FusedResNet(resnet50(num_classes=10, seed=1))
    return det, cls.forward_u8


def _batches():
    g = torch.Generator().manual_seed(0)
    return [torch.randint(0, 256, (2, 128, 128, 3), dtype=torch.uint8, generator=g) for _ in range(3)]


def _worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    det, cls = _stages()
    p = DetectClassifyPipeline(det, cls, torch.device("cpu"), CFG)
    if p.is_detector:
        out = p.run_batches(_batches())
        p.stop()
        q.put([(b, r) for _, b, r in out])
    else:
        q.put(("classified", p.serve_classifier()))
    dist.destroy_process_group()


def test_pipeline_gloo_matches_local():
    det, cls = _stages()
    local = DetectClassifyPipeline(det, cls, torch.device("cpu"), CFG).run_batches(_batches())
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    [p.start() for p in procs]
    got = [q.get(timeout=300) for _ in range(2)]
    [p.join(60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    dist_out = next(g for g in got if isinstance(g, list))
    ncls = next(g for g in got if isinstance(g, tuple))[1]
    assert ncls == sum(b.shape[0] for b, _ in dist_out) > 0
    for (lb, lr), (_, b, r) in zip(dist_out, local):
        assert torch.equal(lb, b)
        assert torch.allclose(lr, r, atol=1e-4)


def test_select_crops_and_stage_transition():
    boxes = torch.tensor([[[0, 0, 10, 10.], [5, 5, 20, 20], [1, 1, 2, 2]]])
    scores = torch.tensor([[0.9, 0.8, 0.7]])
    labels = torch.tensor([[1, 2, 1]])
    sel = select_crops((boxes, scores, labels, torch.tensor([2])), PipelineConfig(score_thresh=0.5))
    assert [round(v, 4) for v in sel[0].tolist()] == [0, 0, 0, 10, 10, 0.9] and sel.shape == (1, 6)
    from aiforearth_api_platform_amd.store import make_store
    s = make_store()
    ids = s.create_many("http://h/v1/ct/detect", 2)
    stage_transition(s, ids, "http://h/v1/ct/classify")
    assert s.zcard("/v1/ct/classify_running") == 2 and s.zcard("/v1/ct/detect_created") == 0
