"""Framework-default comparator: plain PyTorch-ROCm ResNet-50 forward vs. the fused HIP graph.

Measures pure GPU forward throughput (no H2D, no serving) for
  * ``torch``  — the ``torch.nn`` ResNet-50 in bf16, channels_last, eval BatchNorm (MIOpen convs),
                 replayed from a CUDA(HIP) graph — what a user gets from stock PyTorch-ROCm;
  * ``fused``  — ``FusedResNet.forward_u8`` (K1/K7/K8 HIP kernels) replayed from a graph, uint8 in.
Prints one JSON line per variant.  Usage: ``python bench/torch_baseline.py [batch] [iters]``.
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50  # noqa: E402


def graph_time(fn, n):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda:0")
    torch.backends.cudnn.benchmark = True
    ref = resnet50()
    fused = FusedResNet(ref, device=dev)
    m = ref.to(dev).to(torch.bfloat16).to(memory_format=torch.channels_last).eval()
    x = torch.randn(B, 3, 224, 224, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    xu8 = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=dev)
    flops = fused.flops(B)
    with torch.inference_mode():
        for name, fn in (("torch_bf16_channels_last", lambda: m(x)), ("fused_hip", lambda: fused.forward_u8(xu8))):
            dt = graph_time(fn, n)
            print(json.dumps({"variant": name, "batch": B, "ms_per_batch": round(dt * 1e3, 3),
                              "images_per_s": round(B / dt, 1), "tflops": round(flops / dt / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()
