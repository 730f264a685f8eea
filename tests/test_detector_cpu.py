"""Faster-RCNN R50-FPN plumbing on CPU (torch reference ops): shapes, padding, NMS invariants."""
import torch

from aiforearth_api_platform_amd.models.faster_rcnn import DetectorConfig, FasterRCNN
from aiforearth_api_platform_amd.ops.detection import box_iou


def test_detector_forward_shapes_and_invariants():
    cfg = DetectorConfig(pre_nms_top_n=200, post_nms_top_n=100, detections_per_img=20, box_score_thresh=0.0)
    det = FasterRCNN(cfg, seed=0)
    img = torch.randint(0, 256, (2, 128, 128, 3), dtype=torch.uint8)
    boxes, scores, labels, n = det(img)
    assert boxes.shape == (2, 20, 4) and scores.shape == (2, 20) and n.shape == (2,)
    for b in range(2):
        k = int(n[b])
        assert k > 0
        bb, ss, ll = boxes[b, :k], scores[b, :k], labels[b, :k]
        assert torch.all(ss[:-1] >= ss[1:])
        assert torch.all((bb[:, 0] >= 0) & (bb[:, 2] <= 128) & (bb[:, 1] >= 0) & (bb[:, 3] <= 128))
        assert torch.all((ll >= 1) & (ll <= 3))
        for c in range(1, 4):  # per-class NMS: no same-class pair above the threshold
            m = ll == c
            if m.sum() > 1:
                iou = box_iou(bb[m], bb[m])
                iou.fill_diagonal_(0)
                assert iou.max() <= cfg.box_nms_thresh + 1e-6
    out = FasterRCNN.to_list((boxes, scores, labels, n))
    assert len(out) == 2 and set(out[0]["labels"]) <= {"animal", "person", "vehicle"}


def test_anchor_layout():
    det = FasterRCNN(DetectorConfig(), seed=0)
    a = det.anchors([(2, 2)], [16])[0]
    assert a.shape == (12, 4)
    # location (0,0) anchors are centred on the origin; location (0,1) shifted by the stride in x
    assert torch.allclose((a[0, :2] + a[0, 2:]) / 2, torch.zeros(2))
    assert torch.allclose(a[3] - a[0], torch.tensor([16.0, 0, 16.0, 0]))


def test_nms_reference_hand_computed():
    """Pins the greedy NMS reference the GPU kernel is tested against (torchvision is absent here):
    boxes 0/1 overlap with IoU 64/136 = 0.47, boxes 0/2 with IoU 81/100 = 0.81, box 3 is disjoint."""
    from aiforearth_api_platform_amd.ops.detection import nms_reference

    boxes = torch.tensor([[0., 0., 10., 10.], [2., 2., 12., 12.], [0., 0., 9., 9.], [50., 50., 60., 60.]])
    scores = torch.tensor([0.9, 0.8, 0.95, 0.1])
    assert abs(float(box_iou(boxes[:1], boxes[1:2])) - 64 / 136) < 1e-6
    # thr 0.5: box 2 (best) suppresses box 0 (IoU 0.81 > 0.5); box 1 vs box 2: IoU 49/151 = 0.32 -> kept
    assert nms_reference(boxes, scores, 0.5).tolist() == [2, 1, 3]
    # thr 0.9: nothing overlaps that much
    assert nms_reference(boxes, scores, 0.9).tolist() == [2, 0, 1, 3]


def test_nms_sort_rows_fit_the_graph_safe_hip_sort():
    """Both NMS-stage sorts of the default detector fit the HIP row sort at the served sizes, so no multi-kernel
    library sort (not graph-safe) can enter a captured forward; a configuration that does not fit must refuse to run
    its fallback under capture (num_classes >= 10 pushes the detections' sort past 8192)."""
    from aiforearth_api_platform_amd.models.faster_rcnn import DetectorConfig, FasterRCNN
    from aiforearth_api_platform_amd.ops.detection import ROW_SORT_MAX

    det = FasterRCNN.__new__(FasterRCNN)
    det.cfg = DetectorConfig()
    for hw in ((640, 640), (1024, 1024), (1536, 2048)):
        rows = det.sort_rows(hw)
        assert rows["rpn"] <= ROW_SORT_MAX and rows["detections"] <= ROW_SORT_MAX, (hw, rows)
    det.cfg = DetectorConfig(num_classes=10)
    assert det.sort_rows((640, 640))["detections"] > ROW_SORT_MAX


def test_sort_select_and_gather_keep_cpu_reference():
    import torch

    from aiforearth_api_platform_amd.ops.detection import gather_keep, sort_select

    sc = torch.tensor([[0.2, -1.0, 0.9, 0.2, 0.5, -1.0]])
    bx = torch.arange(24, dtype=torch.float32).reshape(1, 6, 4)
    s_s, b_s, b_o, lab, valid = sort_select(sc, bx, 100.0, group_mod=2, want_labels=True)
    assert torch.equal(s_s, torch.tensor([[0.9, 0.5, 0.2, 0.2, -1.0, -1.0]]))
    order = [2, 4, 0, 3, 1, 5]  # ties (0.2 at 0 and 3, -1 at 1 and 5) by lower index
    assert torch.equal(b_s[0], bx[0, order])
    assert lab.tolist() == [[i % 2 + 1 for i in order]]
    assert torch.equal(b_o[0], bx[0, order] + (lab[0].float() * 100.0)[:, None])
    assert valid.tolist() == [4]
    keep = torch.tensor([[1, 0, -1]], dtype=torch.int32)
    kb, ks, kl = gather_keep(keep, b_s, s_s, lab)
    assert torch.equal(kb[0, :2], b_s[0, [1, 0]]) and (kb[0, 2] == 0).all()
    assert torch.equal(ks, torch.tensor([[0.5, 0.9, 0.0]])) and kl[0, 2] == 0
