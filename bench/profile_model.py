"""Eager forwards of the config-3 detector or the config-4 U-Net for per-dispatch rocprofv3 counter collection
(tools/pmc_resnet.sh with PMC_MODEL=detector|unet). A spin kernel (``torch.cuda._sleep``) marks the start of the
last forward, so tools/pmc_summary.py --start spin_kernel keeps exactly that forward.

    python bench/profile_model.py detector [batch 32] [forwards 2]
    python bench/profile_model.py unet [tiles 16] [forwards 2]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

model = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else (32 if model == "detector" else 16)
n = int(sys.argv[3]) if len(sys.argv) > 3 else 2
dev = torch.device("cuda:0")
if model == "detector":
    from aiforearth_api_platform_amd.models.faster_rcnn import DetectorConfig, FasterRCNN  # noqa: E402
    net = FasterRCNN(DetectorConfig(), seed=0, device=dev)
    fwd, x = net.forward_u8, torch.randint(0, 256, (B, 640, 640, 3), dtype=torch.uint8, device=dev)
elif model == "unet":
    from aiforearth_api_platform_amd.models.unet import FusedUNet, unet_landcover  # noqa: E402
    net = FusedUNet(unet_landcover(seed=0), device=dev)
    fwd, x = net.forward_u8, torch.randint(0, 256, (B, 512, 512, 4), dtype=torch.uint8, device=dev)
else:
    raise SystemExit(f"unknown model {model}")
for i in range(n):
    if i == n - 1:
        torch.cuda.synchronize()
        torch.cuda._sleep(1000)  # marker: the last forward starts after this dispatch
    fwd(x)
torch.cuda.synchronize()
print("ok")
