"""BASELINE configs 3-5 as APIs, through the same production path as bench.py (one node scheduler,
one GPU worker process per GPU, per-submission payload writes, torchrun for N > 1):

* ``--model detector``  — config 3: MegaDetector-style Faster-RCNN R50-FPN batch inference, DP over GPUs
  (``/v1/animal_detection``), images/s + p50;
* ``--model landcover`` — config 4 as an API: 4096x4096 RGB+NIR mosaics, one per task, DP over GPUs
  (mosaics/s + p50; the spatial-parallel single-mosaic form is bench/landcover_bench.py);
* ``--model ensemble``  — config 5 as an API: detector -> species classifier under one TaskId (the
  AddPipelineTask hop), both stages in one HIP graph per GPU; images/s + p50.
* ``--model ensemble_group --group 8 [--classifiers M]`` — config 5 as an N:M stage graph over RCCL: N = group -
  M detector GPUs take batches from the scheduler, the classifier GPU(s) classify their crops (M defaults to the
  split ``plan_ensemble`` picks from the measured stage rates: 6:2 at 4 crops per image)
  (``--classifier-dtype fp16`` by default, ``--wire uint8``); ``parallelism: pipeline{N}:{M}``.
* ``--model landcover_spatial --group k`` — config 4 in its spatial form: each 4096^2 mosaic segmented by k GPUs
  together (tiles split evenly, bands scattered, halo logits over P2P); ``parallelism: spatial{k}``.

Worker-group models run from ONE process (the pool spawns one worker process per group GPU); no torchrun.

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
    "ensemble_group": ("aiforearth_api_platform_amd.models.zoo:camera_trap_ensemble_group",
                       "/v1/camera-trap/ensemble-group/detect", 32, lambda s: (s, s, 3), "images/s",
                       "detector->classifier ensemble API images/sec (N:M stage graph over RCCL) + p50"),
    "landcover_spatial": ("aiforearth_api_platform_amd.models.zoo:landcover_spatial", "/v1/landcover/spatial", 1,
                          lambda s: (s, s, 4), "mosaics/s", "land-cover API mosaics/sec (spatial over k GPUs) + p50"),
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
    ap.add_argument("--graphs", default="auto", choices=["auto", "on", "off"],
                    help="capture the whole servable per batch bucket in HIP graphs (auto: the model's default)")
    ap.add_argument("--http", type=int, default=0)
    ap.add_argument("--http-seconds", type=float, default=6.0)
    ap.add_argument("--json-out", default="")
    ap.add_argument("--group", type=int, default=2, help="GPUs per worker group (ensemble_group, landcover_spatial)")
    ap.add_argument("--classifiers", type=int, default=0,
                    help="classifier GPUs of an ensemble_group; 0 = the split runtime/pipeline.py plan_ensemble picks "
                         "from the measured stage rates (--stage-rates) at --crops-per-image")
    ap.add_argument("--stage-rates", default=os.path.join(ROOT, "profiles", "r4_stage_rates", "stage_rates.json"))
    ap.add_argument("--crops-per-image", type=float, default=4.0)
    ap.add_argument("--classifier-dtype", default="fp16", choices=["bf16", "fp16"])
    ap.add_argument("--wire", default="uint8", choices=["uint8", "float16"])
    ap.add_argument("--tile", type=int, default=512)
    ap.add_argument("--stride", type=int, default=448)
    ap.add_argument("--tile-batch", type=int, default=16, help="land-cover tiles per U-Net batch (81 tiles per mosaic)")
    a = ap.parse_args()
    from aiforearth_api_platform_amd.runtime.node_bench import run_node_bench
    from aiforearth_api_platform_amd.runtime.worker_pool import ModelSpec

    factory, path, batch, shape, unit, metric = MODELS[a.model]
    a.batch = a.batch or batch
    size = a.size or (4096 if a.model.startswith("landcover") else 640)
    kwargs, graphs, stages, group, leaders = {}, not a.no_graphs, (), 1, 1
    extra, dtype = {}, "bf16"
    if a.model.startswith("landcover"):
        kwargs = {"height": size, "width": size, "tile": a.tile, "stride": a.stride, "tile_batch": a.tile_batch}
    if a.model == "landcover_spatial":
        graphs = False  # P2P inside the servable: the U-Net runs per tile batch, eagerly
        group = a.group
        extra["parallelism"] = f"spatial{group}"
    if a.model.startswith("ensemble"):
        kwargs = {"max_crops": 4, "score_thresh": 0.0, "class_id": None}  # random weights: keep crops flowing
        stages = ("http://127.0.0.1" + path.replace("/detect", "/classify"),)
    if a.model == "ensemble_group":
        if a.classifiers == 0:  # placement from the measured stage rates
            import json

            from aiforearth_api_platform_amd.runtime.pipeline import plan_ensemble

            with open(a.stage_rates) as f:
                r = json.load(f)
            plan = plan_ensemble(a.group, r["detector_stage"]["images_per_s"],
                                 r[f"classifier_stage_{a.classifier_dtype}"]["crops_per_s"], a.crops_per_image)
            stage = max((c for c in plan["candidates"] if c["form"] == "stage"), key=lambda c: c["images_per_s"])
            a.classifiers = stage["classifiers"]
            extra["placement"] = {"best": {k: v for k, v in plan.items() if k != "candidates"},
                                  "stage_graph": stage, "crops_per_image": a.crops_per_image}
            print(f"[api_bench] placement: {plan['form']} is fastest ({plan['images_per_s']:.0f} images/s est.); "
                  f"stage graph {stage['leaders']}:{stage['classifiers']} ({stage['images_per_s']:.0f})", flush=True)
        if not 1 <= a.classifiers < a.group:
            raise SystemExit("--classifiers must leave at least one detector GPU in --group")
        group, leaders = a.group, a.group - a.classifiers
        kwargs.update(classifier_dtype=a.classifier_dtype, wire_dtype=a.wire)
        graphs = False  # each stage captures its own HIP graphs (runtime/pipeline.py StageGraphPipeline)
        extra.update(parallelism=f"pipeline{leaders}:{a.classifiers}", wire_dtype=a.wire,
                     stage_dtypes={"detector": "bf16", "classifier": a.classifier_dtype})
        dtype = a.classifier_dtype if a.classifier_dtype == "bf16" else "bf16 detector / fp16 classifier"
    if a.graphs != "auto":
        graphs = a.graphs == "on"
    spec = ModelSpec(factory, shape(size), a.batch, 5, kwargs, graphs, (), stages, group, leaders)
    run_node_bench(a, spec, path, metric, unit, dtype=dtype,
                   config={"model": a.model, "image_size": size, "api": "async", **extra,
                           **{k: v for k, v in kwargs.items() if k != "score_thresh"}})


if __name__ == "__main__":
    main()
