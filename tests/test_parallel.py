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
