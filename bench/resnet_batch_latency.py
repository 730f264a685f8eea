"""ResNet-50 served forward (uint8 images -> top-5) latency per batch size, HIP-graph replay on one stream: the
low-load buckets the engine captures besides the serving batch (``batch_buckets``, examples/platform.yaml).
``AI4E_CONV_TILES`` picks the tile table, so two runs A/B a table.

    python bench/resnet_batch_latency.py [B ...]      (default 8 32 128 250)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    m = FusedResNet(resnet50(seed=0), device=dev)
    out = {"tiles": os.environ.get("AI4E_CONV_TILES", "repo")}
    for b in [int(a) for a in sys.argv[1:]] or [8, 32, 128, 250]:
        img = torch.randint(0, 256, (b, 224, 224, 3), dtype=torch.uint8, device=dev)
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            m.topk_u8(img, 5)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                m.topk_u8(img, 5)
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(30):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 30
        out[f"b{b}"] = {"ms": round(ms, 4), "images_per_s": round(b / ms * 1e3, 1)}
        print(json.dumps({f"b{b}": out[f"b{b}"]}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
