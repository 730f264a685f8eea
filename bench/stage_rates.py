"""Stage rates of the config-5 stage graph on ONE GPU, to size its N:M ratio (models/zoo.py
``camera_trap_ensemble_group``; runtime/pipeline.py ``StageGraphPipeline``):

* detector stage: detection + crop selection + 224^2 crop-resize + compaction, one HIP graph per batch
  (``StageGraphPipeline._detect_crop_compact``), images/s at the API batch (32 x 640^2);
* classifier stage: the crop classifier in its per-bucket graph, crops/s at bucket 128, bf16 (fused K1s/K1c/K1p
  graph) and fp16 (per-conv K1 on f16 MFMA).

With ``c`` crops per image, one classifier GPU keeps up with ``rate_cls / (c * rate_det)`` detector GPUs; the
script prints that ratio per dtype. Random weights, synthetic uint8 frames.

    python bench/stage_rates.py [--batch 32 --size 640 --crops 4 --iters 20]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _timed(fn, iters: int) -> float:
    """Per-call time with a device sync after every call (as in serving: each stage output is consumed on the
    host before the next batch)."""
    import torch

    for _ in range(3):
        fn()
        torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
        torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--crops", type=int, default=4)
    ap.add_argument("--bucket", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    import torch

    from aiforearth_api_platform_amd import _build
    from aiforearth_api_platform_amd.models import zoo
    from aiforearth_api_platform_amd.models.faster_rcnn import DetectorConfig, FasterRCNN
    from aiforearth_api_platform_amd.runtime.pipeline import PipelineConfig, StageGraphPipeline

    _build.build_all()
    dev = torch.device("cuda")
    cfg = PipelineConfig(score_thresh=0.0, class_id=None, max_crops_per_image=a.crops)
    det = FasterRCNN(DetectorConfig(box_score_thresh=0.0), seed=0, device=dev)
    pd = StageGraphPipeline(det.forward_u8, None, dev, cfg)
    imgs = torch.randint(0, 256, (a.batch, a.size, a.size, 3), dtype=torch.uint8, device=dev)
    t_det = _timed(lambda: pd._det_graph(imgs), a.iters)
    out = {"detector_stage": {"batch": a.batch, "image_size": a.size, "ms_per_batch": 1e3 * t_det,
                              "images_per_s": a.batch / t_det}}
    crops = torch.randint(0, 256, (a.bucket, 224, 224, 3), dtype=torch.uint8, device=dev)
    for dt in ("bf16", "fp16"):
        pc = StageGraphPipeline(None, zoo.crop_classifier(dev, 200, 1, dt), dev, cfg)
        t = _timed(lambda: pc.classify(crops), a.iters)
        rate = a.bucket / t
        out[f"classifier_stage_{dt}"] = {"bucket": a.bucket, "ms_per_bucket": 1e3 * t, "crops_per_s": rate,
                                         "detectors_per_classifier": rate / (a.crops * out["detector_stage"]["images_per_s"])}
    line = json.dumps(out)
    print(line, flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
