"""BASELINE config #5: detector -> classifier 2-stage ensemble, crops handed GPU->GPU over RCCL.

The stage graph (runtime/pipeline.py StageGraphPipeline) without the serving path: ``--leaders`` detector ranks
feed the other ranks' classifiers (default world // 2, i.e. 1:1 pairs); world 1 runs both stages on one GPU, each
in its HIP graphs. Reports whole-node images/s (images through both stages) and crops/s.

    torchrun --nproc-per-node 2 bench/pipeline_bench.py [--batch 32 --size 640 --steps 10 --classifier-dtype fp16]
"""
import argparse

import torch

from common import Dist, build_once


def main():
    import time
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)  # batch inference: 32 images per GPU (8 -> 32: +42 % images/s)
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--leaders", type=int, default=0)
    ap.add_argument("--classifier-dtype", default="fp16", choices=("bf16", "fp16"))
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    d = Dist()
    build_once(d)
    from aiforearth_api_platform_amd.models import zoo
    from aiforearth_api_platform_amd.models.faster_rcnn import DetectorConfig, FasterRCNN
    from aiforearth_api_platform_amd.runtime.pipeline import PipelineConfig, StageGraphPipeline
    leaders = a.leaders or max(1, d.world // 2)
    is_det = d.world == 1 or d.rank < leaders
    det = FasterRCNN(DetectorConfig(), seed=0, device=d.device) if is_det else None
    cls = zoo.crop_classifier(d.device, 200, 1, a.classifier_dtype) if (d.world == 1 or not is_det) else None
    pcfg = PipelineConfig(score_thresh=0.0, class_id=None, max_crops_per_image=4)
    p = StageGraphPipeline(det.forward_u8 if det is not None else None, cls, d.device, pcfg,
                           n_leaders=leaders if d.world > 1 else 1)
    g = torch.Generator().manual_seed(d.rank)
    batches = [torch.randint(0, 256, (a.batch, a.size, a.size, 3), dtype=torch.uint8, generator=g).to(d.device)
               for _ in range(2)]
    crops = 0
    if p.is_detector:
        p.run_batches([batches[i % 2] for i in range(a.warmup)])
        torch.cuda.synchronize()
        t = time.perf_counter()
        out = p.run_batches([batches[i % 2] for i in range(a.steps)])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        crops = sum(r.shape[0] for _, _, _, r in out)
        p.stop()
    else:
        p.serve()
        dt = 0.0
    dt, = d.max(dt)
    crops, = d.sum(crops)
    imgs = a.steps * a.batch * (leaders if d.world > 1 else 1)
    d.emit({"metric": "detector->classifier ensemble images/sec (whole node)", "value": round(imgs / dt, 2),
            "unit": "images/s", "n_gpus": d.world, "crops_per_s": round(crops / dt, 2),
            "ms_per_batch": round(dt / a.steps * 1e3, 2), "dtype": "bf16 detector, " + a.classifier_dtype + " classifier",
            "wire_dtype": pcfg.wire_dtype if d.world > 1 else None,
            "data": "synthetic uint8 images, random-init weights",
            "config": {"per_detector_batch": a.batch, "image_size": a.size, "crop": 224,
                       "parallelism": f"stage{leaders}:{d.world - leaders}" if d.world > 1 else "colocated"}},
           a.json_out)
    d.close()


if __name__ == "__main__":
    main()
