"""Shared helpers for the per-config benchmarks (torchrun-compatible, one rank per GPU)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class Dist:
    def __init__(self, device_kind="cuda"):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if device_kind == "cuda":
                torch.cuda.set_device(self.local)
            dist.init_process_group("nccl" if device_kind == "cuda" else "gloo", rank=self.rank,
                                    world_size=self.world)
            self.dist = dist
        self.device = torch.device(f"cuda:{self.local}" if device_kind == "cuda" else "cpu")
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)

    def sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        if self.dist is not None:
            self.dist.barrier()

    def max(self, *vals):
        t = torch.tensor(vals, dtype=torch.float64, device=self.device if self.dist else "cpu")
        if self.dist is not None:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return [float(v) for v in t.cpu()]

    def sum(self, *vals):
        t = torch.tensor(vals, dtype=torch.float64, device=self.device if self.dist else "cpu")
        if self.dist is not None:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return [float(v) for v in t.cpu()]

    def emit(self, record, path=""):
        if self.rank == 0:
            line = json.dumps(record)
            print(line, flush=True)
            if path:
                with open(path, "w") as f:
                    f.write(line + "\n")

    def close(self):
        if self.dist is not None:
            self.dist.barrier()
            self.dist.destroy_process_group()


def timed(fn, steps, warmup, sync):
    for _ in range(warmup):
        fn()
    sync()
    t = time.perf_counter()
    for _ in range(steps):
        fn()
    sync()
    return time.perf_counter() - t


def build_once(d: Dist):
    from aiforearth_api_platform_amd import _build
    if d.rank == 0:
        _build.build_all()
    if d.dist is not None:
        d.dist.barrier()
