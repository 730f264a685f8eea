"""BASELINE configs 3-5 as APIs, through the same production path as bench.py (one node scheduler,
one GPU worker process per GPU, per-submission payload writes, torchrun for N > 1):

* ``--model detector``  — config 3: MegaDetector-style Faster-RCNN R50-FPN batch inference, DP over GPUs
  (``/v1/animal_detection``), images/s + p50;
* ``--model landcover`` — config 4 as an API: 4096x4096 RGB+NIR mosaics, one per task, DP over GPUs
  (mosaics/s + p50; the spatial-parallel single-mosaic form is bench/landcover_bench.py);
* ``--model ensemble``  — config 5 as an API: detector -> species classifier under one TaskId (the
  AddPipelineTask hop), both stages in one HIP graph per GPU; images/s + p50.

    python bench/api_bench.py --model detector [--batch 32 --size 640 --steps 20]
    torchrun --nproc-per-node 8 bench/api_bench.py --model detector --gpus 8
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MODELS = {
    # name: (factory, path, default batch, item shape fn, unit, metric)
    "detector": ("aiforearth_api_platform_amd.models.zoo:megadetector", "/v1/animal_detection", 32,
                 lambda s: (s, s, 3), "images/s", "camera-trap detection API images/sec (whole node) + p50"),
    "landcover": ("aiforearth_api_platform_amd.models.zoo:landcover", "/v1/landcover/classify", 1,
                  lambda s: (s, s, 4), "mosaics/s", "land-cover API mosaics/sec (whole node) + p50"),
    "ensemble": ("aiforearth_api_platform_amd.models.zoo:camera_trap_ensemble", "/v1/camera-trap/ensemble/detect", 32,
                 lambda s: (s, s, 3), "images/s", "detector->classifier ensemble API images/sec (whole node) + p50"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=list(MODELS), default="detector")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--size", type=int, default=0)
    ap.add_argument("--inflight", type=int, default=2)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--http", type=int, default=0)
    ap.add_argument("--http-seconds", type=float, default=6.0)
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    from aiforearth_api_platform_amd.runtime.node_bench import run_node_bench
    from aiforearth_api_platform_amd.runtime.worker_pool import ModelSpec

    factory, path, batch, shape, unit, metric = MODELS[a.model]
    a.batch = a.batch or batch
    size = a.size or (4096 if a.model == "landcover" else 640)
    kwargs, graphs, stages = {}, not a.no_graphs, ()
    if a.model == "landcover":
        kwargs = {"height": size, "width": size, "tile": 512, "stride": 448, "tile_batch": 16}
        graphs = False
    if a.model == "ensemble":
        kwargs = {"max_crops": 4, "score_thresh": 0.0, "class_id": None}  # random weights: keep crops flowing
        stages = ("http://127.0.0.1/v1/camera-trap/ensemble/classify",)
    spec = ModelSpec(factory, shape(size), a.batch, 5, kwargs, graphs, (), stages)
    run_node_bench(a, spec, path, metric, unit,
                   config={"model": a.model, "image_size": size, "api": "async", **{k: v for k, v in kwargs.items()
                                                                                      if k != "score_thresh"}})


if __name__ == "__main__":
    main()
