"""parallel.dist helpers (single-process parts; the multi-rank paths run in test_bench_contract / *_dist)."""
import pytest
import torch

from aiforearth_api_platform_amd.parallel.dist import DistEnv, all_reduce_max, gather_objects, pair_ranks


def test_pair_ranks():
    assert pair_ranks(8) == [(0, 1), (2, 3), (4, 5), (6, 7)]
    with pytest.raises(ValueError):
        pair_ranks(3)


def test_single_process_helpers():
    env = DistEnv(0, 1, 0, torch.device("cpu"), None)
    assert env.is_main and not env.initialized
    assert all_reduce_max([1.5, 2.0], env) == [1.5, 2.0]
    assert gather_objects({"a": 1}, env) == [{"a": 1}]


def _bcast_worker(rank, world, port, q):
    import os

    import torch.distributed as dist

    from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50
    from aiforearth_api_platform_amd.parallel.dist import broadcast_tensors

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = FusedResNet(resnet50(seed=rank))  # different weights per rank until the broadcast
    broadcast_tensors(m.tensors(), src=0, bucket_bytes=8 << 20)  # small buckets: several collectives
    img = torch.randint(0, 256, (2, 64, 64, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(9))
    q.put((rank, m.forward_u8(img).numpy().copy()))  # (by value: see tests/test_pipeline_dist.py)
    dist.barrier()
    dist.destroy_process_group()


def test_broadcast_tensors_replicates_rank0_weights():
    """Bucketed weight broadcast (survey C1) over gloo, 2 ranks: after it, rank 1 computes rank 0's outputs."""
    import socket

    import torch.multiprocessing as mp

    from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bcast_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = {r: torch.from_numpy(o) for r, o in (q.get(timeout=300) for _ in range(2))}
    for p in procs:
        p.join(timeout=60)
    img = torch.randint(0, 256, (2, 64, 64, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(9))
    ref = FusedResNet(resnet50(seed=0)).forward_u8(img)
    assert torch.allclose(outs[0], ref) and torch.allclose(outs[1], ref)
