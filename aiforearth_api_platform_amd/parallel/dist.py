"""One-process-per-GPU distributed setup and the small collective helpers the runtime uses.

The reference scales by Kubernetes replicas behind a round-robin load balancer
(``APIs/Charts/templates/async-gpu/autoscaler.yaml:11-17``,
``APIs/Charts/camera-trap/detection-async/routing.yaml``); it has no collectives at all. Here every
MI355X is one process (``torchrun`` / :mod:`runtime.worker_pool`) and the few cross-GPU exchanges the
platform needs run on ``torch.distributed``:

* ``nccl`` is RCCL on ROCm — peer-to-peer over xGMI for pipeline hand-off and halo rows, broadcast
  for a mosaic, an all-reduce(MAX) of the timing triple in the benchmark;
* ``gloo`` for CPU-only runs and the multi-process tests.

xGMI is point-to-point (7 links per GPU), so the runtime prefers pairwise send/recv between
neighbouring ranks over ring collectives wherever the data flow allows it.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable, Iterable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int
    world: int
    local_rank: int
    device: torch.device
    backend: Optional[str]  # None when world == 1 (no process group)

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def initialized(self) -> bool:
        return self.backend is not None


def env_ranks() -> Tuple[int, int, int]:
    """(rank, world, local_rank) from the torchrun environment (defaults: single process)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_from_env(device_type: str = "cuda", build: Optional[Callable[[], None]] = None,
                  timeout_s: float = 600.0) -> DistEnv:
    """Pin this process to ``cuda:LOCAL_RANK`` and join the process group (RCCL on GPU, gloo on CPU).

    ``build`` (e.g. the in-tree HIP/C++ build) runs on rank 0 only, before a barrier, so the other
    ranks never load a half-written library.  The device is set *before* ``init_process_group`` so
    RCCL binds each communicator to the right GPU.
    """
    import datetime

    rank, world, local = env_ranks()
    # AI4E_REHEARSE_ONE_GPU=1: every rank on cuda:0 with gloo collectives — rehearses the multi-rank GPU path (the
    # serve topology's remote workers, HIP graphs in worker threads) on a one-GPU box; RCCL refuses two ranks per GPU
    rehearse = device_type == "cuda" and os.environ.get("AI4E_REHEARSE_ONE_GPU") == "1"
    if device_type == "cuda":
        dev_index = 0 if rehearse else local
        torch.cuda.set_device(dev_index)
        device = torch.device(f"cuda:{dev_index}")
    else:
        device = torch.device("cpu")
    if rank == 0 and build is not None:
        build()
    if world == 1:
        return DistEnv(rank, 1, local, device, None)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    backend = "nccl" if device_type == "cuda" and not rehearse else "gloo"
    kw = {"device_id": device} if backend == "nccl" else {}
    dist.init_process_group(backend, rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=timeout_s), **kw)
    dist.barrier()
    return DistEnv(rank, world, local, device, backend)


def sync(env: DistEnv) -> None:
    """Device drain + barrier: the bracket around a timed region."""
    if env.device.type == "cuda":
        torch.cuda.synchronize(env.device)
    if env.initialized:
        dist.barrier()


def all_reduce_max(values: Sequence[float], env: DistEnv) -> List[float]:
    """Element-wise MAX over ranks (one small collective; fp64 so latencies survive)."""
    t = torch.tensor(list(values), dtype=torch.float64)
    if env.initialized:
        if env.backend == "nccl":
            t = t.to(env.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.cpu().tolist()


def gather_objects(obj, env: DistEnv) -> List:
    """All ranks' Python objects on every rank (control data only — never tensors on the hot path)."""
    if not env.initialized:
        return [obj]
    out = [None] * env.world
    dist.all_gather_object(out, obj)
    return out


def pair_ranks(world: int) -> List[Tuple[int, int]]:
    """Producer/consumer pairs (2i, 2i+1): neighbours share a direct xGMI link on an 8-GPU node."""
    if world % 2:
        raise ValueError(f"pipeline pairing needs an even world size, got {world}")
    return [(i, i + 1) for i in range(0, world, 2)]


def isend_all(tensors: Iterable[torch.Tensor], dst: int, group=None) -> list:
    """Post non-blocking sends; return (work, tensor) pairs that keep the buffers alive until waited."""
    works = []
    for t in tensors:
        t = t.contiguous()
        works.append((dist.isend(t, dst, group=group), t))
    return works


def wait_all(works: list) -> None:
    for w, _ in works:
        w.wait()


def broadcast_tensors(tensors: Sequence[torch.Tensor], src: int = 0, group=None,
                      bucket_bytes: int = 256 << 20) -> None:
    """Replicate ``tensors`` from group rank ``src`` to every rank in place (survey C1: weights loaded once, then
    broadcast over xGMI). Tensors of one dtype are packed into flat buckets of up to ``bucket_bytes`` so a
    ResNet-50 (51 MB bf16) is ONE collective instead of ~160 small ones; every rank must pass tensors of the
    same shapes and order. No-op without an initialized process group."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    by_dtype: dict = {}
    for t in tensors:
        by_dtype.setdefault((t.dtype, t.device), []).append(t)
    for (dtype, device), ts in by_dtype.items():
        bucket: List[torch.Tensor] = []
        size = 0
        for t in ts + [None]:
            if t is not None and (not bucket or size + t.numel() * t.element_size() <= bucket_bytes):
                bucket.append(t)
                size += t.numel() * t.element_size()
                continue
            flat = torch.cat([b.reshape(-1) for b in bucket])
            dist.broadcast(flat, group_src=src, group=group)
            off = 0
            for b in bucket:
                b.copy_(flat[off:off + b.numel()].view_as(b))
                off += b.numel()
            bucket, size = ([t], t.numel() * t.element_size()) if t is not None else ([], 0)


def destroy(env: DistEnv) -> None:
    if env.initialized and dist.is_initialized():
        dist.destroy_process_group()
