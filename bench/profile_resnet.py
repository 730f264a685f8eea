"""Eager ResNet-50 forwards (no graphs) for per-dispatch rocprofv3 counter collection."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda:0")
m = FusedResNet(resnet50(seed=0), device=dev)
x = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=dev)
for _ in range(n):
    m(x)
torch.cuda.synchronize()
print("ok")
