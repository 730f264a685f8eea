#!/usr/bin/env python
"""Headline benchmark: ResNet-50 224x224 async classification API, bf16, images/s + p50 task latency.

Metric and config from BASELINE.json ("images/sec (whole node) + p50 async-task latency,
ResNet-50 API at 1/2/4/8 GPUs"). Every image goes through the full async serving path of one
replica per GPU (one process per GPU, torch.distributed/RCCL only for the barrier and the
cross-rank MAX of the timings):

    create task (native task store, status "created")  ->  enqueue (native dispatch queue, payload =
    pinned uint8 image slot)  ->  dynamic batcher (receive up to --batch, linger)  ->  "running"  ->
    H2D on a copy stream  ->  HIP-graph replay of the fused ResNet-50 (preprocess + 53 conv kernels +
    pools + classifier, hand-written gfx950 kernels)  ->  softmax/top-5  ->  D2H  ->  "completed".

A step = one batch of --batch tasks per GPU submitted through the API; --inflight steps are kept
outstanding (closed loop). Weak scaling: per-GPU work is fixed as N grows. Data is synthetic
(random uint8 images), weights are random-init (no checkpoints offline).

    python bench.py [--gpus N --steps K --warmup W]       (N>1: torchrun, one rank per GPU)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec (whole node) + p50 async-task latency, ResNet-50 API at 1/2/4/8 GPUs"
BASELINE_VALUE = None  # the reference publishes no numbers


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    # 250, not 256: with the K1c / K1 tile sizes and occupancies on 256 CUs, 250 images fill the layer1 chains
    # (8 x 768 slots), the layer2 chains (3 x 512) and layer3's c3 convs (6 x 512) to whole waves of
    # workgroups; 256 spills a few % of tiles into an extra, nearly empty wave (+1.8-2.1 % images/s measured)
    p.add_argument("--batch", type=int, default=250, help="images per step per GPU (= max dynamic batch)")
    p.add_argument("--inflight", type=int, default=2, help="steps kept outstanding per GPU")
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"])
    p.add_argument("--no-graphs", action="store_true")
    p.add_argument("--chunk", default=None, help="ResNet micro-batching mb:nblocks for the high-res stages ('off' = none)")
    p.add_argument("--device", default="cuda")
    p.add_argument("--json-out", default="")
    return p.parse_args()


def main():
    args = parse()
    os.environ["AI4E_KERNEL_BACKEND"] = args.backend
    if args.chunk is not None:
        os.environ["AI4E_RESNET_CHUNK"] = args.chunk
    from aiforearth_api_platform_amd import _build
    from aiforearth_api_platform_amd.config import Config
    from aiforearth_api_platform_amd.gateway.control import ControlPlane
    from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50
    from aiforearth_api_platform_amd.runtime.engine import InferenceEngine, PayloadRing
    from aiforearth_api_platform_amd.runtime.hostperf import tune_gc
    from aiforearth_api_platform_amd.runtime.serving import GpuBatchWorker
    from aiforearth_api_platform_amd.utils.metrics import percentile

    from aiforearth_api_platform_amd.parallel.dist import (all_reduce_max, broadcast_tensors, destroy, env_ranks,
                                                           init_from_env, sync)

    _, world, _ = env_ranks()
    if world > 1 and args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} != WORLD_SIZE {world}")
    # rank 0 builds the in-tree HIP/C++ libraries, then everyone joins (RCCL on GPU, gloo on CPU)
    denv = init_from_env(args.device, build=_build.build_all)
    rank, device = denv.rank, denv.device

    B, S = args.batch, args.image_size
    model = FusedResNet(resnet50(seed=0), device=device)
    if world > 1:  # weights as if loaded once on rank 0: one bucketed RCCL broadcast over xGMI (survey C1)
        broadcast_tensors(model.tensors(), src=0)
    engine = InferenceEngine(model.forward_u8, (S, S, 3), B, device=device, use_graphs=not args.no_graphs,
                             head_fn=model.topk_u8)
    engine.warmup()

    cfg = Config.load(env={}, max_batch=B, max_batch_delay_ms=0.0)
    cp = ControlPlane(cfg)
    endpoint = "http://127.0.0.1/v1/ai4e/resnet50/classify"
    ring = PayloadRing(B * (args.inflight + 2), (S, S, 3))
    g = torch.Generator().manual_seed(1234 + rank)
    ring.buf.copy_(torch.randint(0, 256, ring.buf.shape, dtype=torch.uint8, generator=g))
    worker = GpuBatchWorker(cp, endpoint, engine, ring, max_batch=B, max_delay_s=0.0005).start()
    queue = cp.queue_for(endpoint)

    def submit_step():
        slots = ring.alloc(B, timeout=60)
        ids = cp.store.create_many(endpoint, B)
        queue.send_many(ids, slots)
        return ids

    def run(nsteps):
        target = worker.images + nsteps * B
        all_ids = []
        submitted = 0
        while submitted < min(args.inflight, nsteps):
            all_ids += submit_step()
            submitted += 1
        while worker.images < target:
            done_steps = (worker.images - (target - nsteps * B)) // B
            while submitted < nsteps and submitted - done_steps < args.inflight:
                all_ids += submit_step()
                submitted += 1
            time.sleep(0.0002)
        return all_ids

    def sync_all():
        sync(denv)

    run(args.warmup)
    tune_gc()
    sync_all()
    worker.phase_s.clear()
    worker.finalize_times.clear()
    t0 = time.perf_counter()
    ids = run(args.steps)
    sync_all()
    dt = time.perf_counter() - t0
    worker.stop()
    lat = sorted(cp.store.latencies(ids))
    p50, p99 = percentile(lat, 50) * 1e3, percentile(lat, 99) * 1e3
    dt, p50, p99 = all_reduce_max([dt, p50, p99], denv)  # slowest rank defines the step time
    images = args.steps * B * world
    value = images / dt
    gflop_img = model.flops(1, S, S) / 1e9
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None if BASELINE_VALUE is None else round(value / BASELINE_VALUE, 4),
        "dtype": "bf16", "data": "synthetic uint8 images, random-init weights",
        "p50_task_latency_ms": round(p50, 3), "p99_task_latency_ms": round(p99, 3),
        "tflops_effective": round(value * gflop_img / 1e3, 2),
        "config": {"model": "resnet50", "global_batch": B * world, "per_gpu_batch": B, "image_size": S,
                   "seq_len": None, "parallelism": f"dp{world}", "api": "async", "inflight_steps": args.inflight,
                   "hip_graphs": not args.no_graphs, "kernel_backend": args.backend,
                   "resnet_chunk": list(model.chunk) if model.chunk else None},
    }
    if os.environ.get("AI4E_BENCH_DEBUG"):
        import numpy as np
        ft = np.diff(np.array(worker.finalize_times)) * 1e3
        print("worker phases (s):", {k: round(v, 4) for k, v in worker.phase_s.items()}, "batches", worker.batches,
              "finalize interval ms: median %.3f min %.3f max %.3f" % (np.median(ft), ft.min(), ft.max()),
              "first finalize after t0 %.3f ms" % ((worker.finalize_times[0] - t0) * 1e3), file=sys.stderr)
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    cp.close()
    sync(denv)
    destroy(denv)


if __name__ == "__main__":
    main()
