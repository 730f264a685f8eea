"""CU-partitioned streams (runtime/cu_partition.py, csrc/kernels/cu_partition.hip): mask packing and balanced CU
selection on the CPU; on the GPU box, that a masked stream's launches (eager and graph replay) stay on its CUs and
that the engine's CU-partitioned pipeline (AI4E_ENGINE_CU_SPLIT) returns what the default engine returns."""
import pytest
import torch

from aiforearth_api_platform_amd.runtime import cu_partition as cup


def test_mask_words_packs_bits():
    assert cup.mask_words([0, 1, 31, 32, 255], 256) == [0x80000003, 1, 0, 0, 0, 0, 0, 0x80000000]
    with pytest.raises(ValueError):
        cup.mask_words([256], 256)


@pytest.mark.parametrize("layout", ["interleaved", "blocked"])
def test_balanced_takes_every_xcd_evenly(layout):
    xcc = [c % 8 for c in range(256)] if layout == "interleaved" else [c // 32 for c in range(256)]
    for n in (8, 96, 128, 160):
        cus = cup.balanced(n, xcc)
        assert len(cus) == n == len(set(cus))
        per = [sum(1 for c in cus if xcc[c] == x) for x in range(8)]
        assert max(per) - min(per) <= 1
    rest = cup.balanced(128, xcc, exclude=cup.balanced(128, xcc))
    assert sorted(rest + cup.balanced(128, xcc)) == list(range(256))


@pytest.mark.gpu
def test_masked_stream_keeps_launches_on_its_cus():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from aiforearth_api_platform_amd.ops import _ext

    _ext.lib()
    total = cup.cu_count()
    xcc = cup.xcc_of_cus()
    cus = cup.balanced(total // 4, xcc)
    s = cup.masked_stream(cus)
    assert cup.stream_mask(s, total) == cus
    c = cup.census(s, nblocks=2048)
    assert c["cu_slots"] == len(cus)
    assert sorted(c["per_xcc"]) == sorted(set(xcc[i] for i in cus))


@pytest.mark.gpu
def test_engine_cu_split_matches_default(monkeypatch):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from aiforearth_api_platform_amd.models.zoo import resnet50_classifier
    from aiforearth_api_platform_amd.runtime.engine import InferenceEngine

    s = resnet50_classifier(device="cuda")
    imgs = torch.randint(0, 256, (16, 224, 224, 3), dtype=torch.uint8).pin_memory()
    ref = InferenceEngine(None, (224, 224, 3), 16, device=torch.device("cuda"), output_fn=s, buckets=[16])
    ref.warmup()
    want = ref.run_sync(imgs)
    monkeypatch.setenv("AI4E_ENGINE_CU_SPLIT", "128")
    eng = InferenceEngine(None, (224, 224, 3), 16, device=torch.device("cuda"), output_fn=s, buckets=[16])
    assert eng.front_stream is not None
    eng.warmup()
    for _ in range(3):  # several batches in flight through both partitions
        got = eng.run_sync(imgs)
        assert torch.equal(got[0], want[0])
        assert torch.allclose(got[1], want[1])
