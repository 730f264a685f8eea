"""BASELINE config #3: MegaDetector-style Faster-RCNN R50-FPN batch inference, DP over GPUs.

One rank per GPU (torchrun), each runs fixed-shape batches of synthetic uint8 images through the
whole detector (backbone, FPN, RPN, proposals + NMS, RoIAlign, box head, per-class NMS) captured in
one HIP graph. Reports whole-node images/s and per-batch latency.

    python bench/detector_bench.py [--batch 32 --size 640 --steps 20 --warmup 5 --no-graphs]
"""
import argparse

import torch

from common import Dist, build_once, timed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)  # batch inference: 32 images per GPU (8 -> 32: +42 % images/s)
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    d = Dist()
    build_once(d)
    from aiforearth_api_platform_amd.models.faster_rcnn import DetectorConfig, FasterRCNN
    det = FasterRCNN(DetectorConfig(), seed=0, device=d.device)
    g = torch.Generator().manual_seed(d.rank)
    x = torch.randint(0, 256, (a.batch, a.size, a.size, 3), dtype=torch.uint8, generator=g).to(d.device)
    fn = lambda: det(x)  # noqa: E731
    if not a.no_graphs:
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            det(x)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            out = det(x)
        fn = graph.replay
    dt = timed(fn, a.steps, a.warmup, d.sync)
    (dt,) = d.max(dt)
    imgs = a.steps * a.batch * d.world
    d.emit({"metric": "detector images/sec (whole node)", "value": round(imgs / dt, 2), "unit": "images/s",
            "n_gpus": d.world, "ms_per_batch": round(dt / a.steps * 1e3, 3), "dtype": "bf16",
            "data": "synthetic uint8 images, random-init weights",
            "config": {"model": "faster_rcnn_r50_fpn", "per_gpu_batch": a.batch, "image_size": a.size,
                       "parallelism": f"dp{d.world}", "hip_graphs": not a.no_graphs}}, a.json_out)
    d.close()


if __name__ == "__main__":
    main()
