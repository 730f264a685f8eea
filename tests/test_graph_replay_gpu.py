"""Back-to-back replays of the config-5 detector-stage HIP graph (detect + crop selection + uint8 crop-resize +
compaction) with no host sync between them and eager allocations coming and going between replays — the sequence
that faulted the GPU in rounds 3-4 (profiles/r4_replay/README.md: torch.topk's multi-block path inside the graph) —
and the last replay compared with the same callable run eagerly."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _flat(res):
    out = []
    for t in res:
        out += list(t) if isinstance(t, (tuple, list)) else [t]
    return out


def test_detector_stage_graph_back_to_back_replays_match_eager():
    from aiforearth_api_platform_amd.models.faster_rcnn import DetectorConfig, FasterRCNN
    from aiforearth_api_platform_amd.runtime.pipeline import PipelineConfig, StageGraphPipeline

    dev = torch.device(DEV)
    det = FasterRCNN(DetectorConfig(box_score_thresh=0.0), seed=0, device=dev)
    pd = StageGraphPipeline(det.forward_u8, None, dev,
                            PipelineConfig(score_thresh=0.0, class_id=None, max_crops_per_image=4))
    # 640^2: the level-0 RPN slice is 160 * 160 * 3 = 76800 logits per image (the shape that took the library's
    # multi-block top-k before rpn_topk)
    imgs = torch.randint(0, 256, (8, 640, 640, 3), dtype=torch.uint8, device=dev)
    eager = [t.clone() for t in _flat(pd._detect_crop_compact(imgs))]
    first = [t.clone() for t in _flat(pd._det_graph(imgs))]  # capture + first replay
    keep = []
    for i in range(8):
        res = pd._det_graph(imgs)                              # no host sync between replays
        keep.append(torch.empty(1 << (16 + i), dtype=torch.uint8, device=dev).fill_(i))  # eager allocations
    torch.cuda.synchronize()
    last = _flat(res)
    names = ["det_boxes", "det_scores", "det_labels", "det_n", "boxes", "scores", "valid", "crops", "count"]
    for name, a, b, c in zip(names, last, first, eager):
        assert torch.equal(a, b), name                         # every replay computes the same
        if a.is_floating_point():
            assert torch.allclose(a, c, rtol=1e-4, atol=1e-3), name
        else:
            assert torch.equal(a, c), name
    assert int(last[-1]) == int(last[6].sum()) > 0
    assert all(int(k[0]) == i for i, k in enumerate(keep))     # and the graph wrote nothing into eager memory


def test_breadcrumbs_count_graph_replays():
    """The fault-locating breadcrumbs (ops/debug.py): counters bumped by kernels inside a captured graph read back
    from host-mapped memory without a copy — one per eager call and one per replay, in stream order."""
    from aiforearth_api_platform_amd.ops.debug import Breadcrumbs

    c = Breadcrumbs(8)
    dev = torch.device(DEV)
    x = torch.ones(1024, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        c.mark("a", dev)
        y = x * 2
        c.mark("b", dev)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        c.mark("a", dev)
        y = x * 2
        c.mark("b", dev)
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    assert c.read() == {"a": 6, "b": 6} and float(y[0]) == 2.0
