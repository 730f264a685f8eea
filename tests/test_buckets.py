"""Batch-size buckets: config parsing and the engine's smallest-fitting-graph choice (CPU)."""
import torch

from aiforearth_api_platform_amd.config import Config, bucket_list
from aiforearth_api_platform_amd.runtime.engine import InferenceEngine


def test_bucket_list_parsing():
    assert bucket_list("8,32,128", 256) == [8, 32, 128, 256]
    assert bucket_list("", 64) == [64]
    assert bucket_list([300, 16, 16, 0], 256) == [16, 256]  # dedup, drop out-of-range, max always last
    assert bucket_list(" 4, 2 ", 8) == [2, 4, 8]


def test_config_env_buckets():
    cfg = Config.load(env={"AI4E_BATCH_BUCKETS": "1,16"})
    assert bucket_list(cfg.batch_buckets, 64) == [1, 16, 64]
    assert Config.load(env={}).batch_buckets == "8,32,128"


def test_engine_picks_smallest_bucket():
    calls = []

    def model(x):
        calls.append(x.shape[0])
        return torch.zeros(x.shape[0], 10)

    eng = InferenceEngine(model, (4, 4, 3), 64, device="cpu", buckets=[8, 32])
    assert eng.buckets == [8, 32, 64]
    assert [eng.bucket_for(n) for n in (1, 8, 9, 33, 64)] == [8, 8, 32, 64, 64]
    res = eng.submit(torch.zeros(5, 4, 4, 3, dtype=torch.uint8), [0, 1, 2])
    assert res.n == 3 and res.top_idx.shape == (3, 5)
