"""Detector -> classifier stage graph over gloo (CPU ranks; gloo stands in for RCCL) == the same stages in one
process: 1:1 (2 ranks) and 3:1 (4 ranks) with several batches per detector (one batch's crops on the wire while
the next is detected), plus the AddPipelineTask-style task retargeting."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from aiforearth_api_platform_amd.runtime.pipeline import PipelineConfig, StageGraphPipeline, stage_transition

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
    return det.forward_u8, cls.forward_u8


def _batches(rank):
    g = torch.Generator().manual_seed(100 + rank)
    return [torch.randint(0, 256, (2, 128, 128, 3), dtype=torch.uint8, generator=g) for _ in range(3)]


def _worker(rank, world, leaders, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    det, cls = _stages()
    p = StageGraphPipeline(det if rank < leaders else None, cls if rank >= leaders else None, torch.device("cpu"), CFG,
                           n_leaders=leaders)
    if p.is_detector:
        # the serving form (padded=True) never reads a device value on the host: every hand-off is stream-ordered
        # behind the detector's graph replay (no count.item() between replays)
        real_item, real_tolist = torch.Tensor.item, torch.Tensor.tolist

        def no_host_read(*a, **k):
            raise AssertionError("host read of a device value on the detector's hand-off path")
        torch.Tensor.item, torch.Tensor.tolist = no_host_read, no_host_read
        try:
            padded = p.run_batches(_batches(rank), padded=True)
        finally:
            torch.Tensor.item, torch.Tensor.tolist = real_item, real_tolist
        out = [(b, s_, v, r[: int(c.item())]) for b, s_, v, r, c in padded]
        p.stop()
        # numpy copies travel by value: a torch tensor would go through a shared-memory fd that the parent may only
        # open after this process has exited (FileNotFoundError in the resource sharer, a flaky failure)
        q.put((rank, [(v.numpy().copy(), r.numpy().copy()) for _, _, v, r in out]))
    else:
        q.put((rank, p.serve()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,leaders", [(2, 1), (4, 3)])
def test_stage_graph_gloo_matches_local(world, leaders):
    det, cls = _stages()
    local = StageGraphPipeline(det, cls, torch.device("cpu"), CFG)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, leaders, port, q)) for r in range(world)]
    [p.start() for p in procs]
    got = dict(q.get(timeout=600) for _ in range(world))
    [p.join(60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    total = 0
    for r in range(leaders):
        ref = local.run_batches(_batches(r))
        for (v, res), (_, _, lv, lres) in zip(got[r], ref):
            v, res = torch.from_numpy(v), torch.from_numpy(res)
            assert torch.equal(v, lv)
            assert torch.allclose(res, lres, atol=1e-4)
            total += res.shape[0]
    assert sum(got[r] for r in range(leaders, world)) == total > 0


def test_stage_transition():
    from aiforearth_api_platform_amd.store import make_store
    s = make_store()
    ids = s.create_many("http://h/v1/ct/detect", 2)
    stage_transition(s, ids, "http://h/v1/ct/classify")
    assert s.zcard("/v1/ct/classify_running") == 2 and s.zcard("/v1/ct/detect_created") == 0


def test_plan_ensemble_from_stage_rates():
    from aiforearth_api_platform_amd.runtime.pipeline import plan_ensemble

    # round 3's measured rates: detector 3.3k images/s, fp16 classifier 44.7k crops/s, 4 crops per image
    p = plan_ensemble(8, 3299.0, 44662.0, 4.0)
    stage = max((c for c in p["candidates"] if c["form"] == "stage"), key=lambda c: c["images_per_s"])
    assert (stage["leaders"], stage["classifiers"]) == (6, 2)       # 7:1 is classifier-bound at 4 crops/image
    assert p["form"] == "colocated"                                  # the detector is the heavy stage
    p1 = plan_ensemble(8, 3299.0, 56452.0, 1.0)
    assert max((c for c in p1["candidates"] if c["form"] == "stage"),
               key=lambda c: c["images_per_s"])["classifiers"] == 1  # few crops: 7:1
    # ideal colocation is never slower than a split (harmonic mean); a measured colocated rate below that
    # (e.g. two models' working sets thrashing one GPU) makes the stage graph the choice
    p2 = plan_ensemble(8, 20000.0, 8000.0, 4.0, colocated_images_per_s=1000.0)
    assert p2["form"] == "stage" and (p2["leaders"], p2["classifiers"]) == (1, 7)
