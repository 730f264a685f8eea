"""RoIAlign processing-order A/B on the detector's real proposals (batch 32 at 640², random-init weights): the
default order (image-major, proposals in score order, workgroup b on XCD b % 8) against the same RoIs taken in
y-sorted order per image and/or in contiguous ranges per XCD. The outputs are the same rows (each RoI is computed
independently); only the L2 locality of the feature gathers changes.

    python bench/roi_order_ab.py [reps 20] [rounds 3]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from aiforearth_api_platform_amd.models.faster_rcnn import DetectorConfig, FasterRCNN  # noqa: E402
from aiforearth_api_platform_amd.ops.detection import roi_align_fpn  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda:0")
B = 32
net = FasterRCNN(DetectorConfig(), seed=0, device=dev)
x = torch.randint(0, 256, (B, 640, 640, 3), dtype=torch.uint8, device=dev)
with torch.no_grad():
    from aiforearth_api_platform_amd.ops.pool import preprocess_s2d_u8

    xs = preprocess_s2d_u8(x)
    P = net.fpn(net.backbone_stages(xs))
    props, count, rois = net.proposals(P, (640, 640))
torch.cuda.synchronize()
R = rois.shape[0]
per = R // B
strides = [640 // p.shape[1] for p in P[:4]]
scales = [1.0 / s for s in strides]
yc = (rois[:, 2] + rois[:, 4]).view(B, per)
# y-sorted within each image, images kept in order
ysort = (yc.argsort(dim=1, stable=True) + torch.arange(B, device=dev)[:, None] * per).reshape(-1).to(torch.int32)
# level-major then y within each image (the level the kernel assigns)
area = ((rois[:, 3] - rois[:, 1]).clamp(min=0) * (rois[:, 4] - rois[:, 2]).clamp(min=0)).view(B, per)
lvl = torch.floor(4 + torch.log2(area.sqrt() / 224 + 1e-6)).clamp(2, 5)
lsort = ((lvl * 4096 + yc).argsort(dim=1, stable=True) + torch.arange(B, device=dev)[:, None] * per).reshape(-1)
lsort = lsort.to(torch.int32)
variants = {"base": (None, False), "xcd": (None, True), "ysort": (ysort, False), "ysort_xcd": (ysort, True),
            "lsort_xcd": (lsort, True)}
ref = roi_align_fpn(P[:4], scales, rois, (7, 7), 2)
for name, (order, xcd) in variants.items():
    out = roi_align_fpn(P[:4], scales, rois, (7, 7), 2, order=order, xcd=xcd)
    torch.cuda.synchronize()
    assert torch.equal(out, ref), name
res = {k: [] for k in variants}
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for rd in range(rounds):
    for name, (order, xcd) in variants.items():
        roi_align_fpn(P[:4], scales, rois, (7, 7), 2, order=order, xcd=xcd)
        ev0.record()
        for _ in range(reps):
            roi_align_fpn(P[:4], scales, rois, (7, 7), 2, order=order, xcd=xcd)
        ev1.record()
        torch.cuda.synchronize()
        res[name].append(ev0.elapsed_time(ev1) * 1000 / reps)
    print(f"round {rd}: " + ", ".join(f"{k} {v[-1]:.1f} us" for k, v in res.items()), flush=True)
print({k: round(min(v), 1) for k, v in res.items()})
