"""Multi-GPU API forms as worker groups, on CPU ranks (gloo stands in for RCCL):

* config 5: detector -> classifier pair (leader = detector process, follower = classifier process,
  crops and results over P2P) served through the pool == the single-process ensemble;
* config 4: spatial-parallel land-cover over a 3-process group (tile rows split, halo rows over P2P,
  bands gathered on the leader) == the single-process segmentation.
"""
import os
import time

import pytest

import numpy as np
import torch

from aiforearth_api_platform_amd.config import Config
from aiforearth_api_platform_amd.gateway.control import ControlPlane
from aiforearth_api_platform_amd.runtime.worker_pool import ModelSpec, WorkerPool

DET = dict(box_score_thresh=0.0, pre_nms_top_n=100, post_nms_top_n=50, detections_per_img=10)
ENS = dict(max_crops=3, score_thresh=0.0, class_id=None, num_species=10, **DET)


def _wait(cond, t=300):
    d = time.time() + t
    while time.time() < d:
        if cond():
            return True
        time.sleep(0.05)
    return False


def _serve(spec, devices, payloads, done_path):
    cp = ControlPlane(Config.load(env={}))
    pool = WorkerPool(cp, "http://127.0.0.1/v1/group/in", spec, devices, heartbeat_interval_s=0.2,
                      heartbeat_timeout_s=120, max_delay_s=0.2).start(wait_ready_s=300)
    try:
        ids = pool.submit_many(payloads)
        assert _wait(lambda: cp.store.zcard(done_path + "_completed") == len(ids))
        time.sleep(0.6)  # one more heartbeat carries the transfer counters
        pool.refresh()
        return [pool.result(t) for t in ids], pool.stats()
    finally:
        pool.stop()
        cp.close()


def test_ensemble_pair_group_matches_single_process():
    from aiforearth_api_platform_amd.models import zoo
    from aiforearth_api_platform_amd.runtime.servable import decode_row, encode_rows
    imgs = np.random.default_rng(5).integers(0, 256, (2, 128, 128, 3), dtype=np.uint8)
    spec = ModelSpec("aiforearth_api_platform_amd.models.zoo:camera_trap_ensemble_pair", (128, 128, 3), 2, 5, ENS,
                     False, (), ("http://127.0.0.1/v1/group/classify",), 2)
    got, stats = _serve(spec, ["cpu", "cpu"], imgs, "/v1/group/classify")
    local = zoo.camera_trap_ensemble("cpu", **ENS)
    outs = [o.numpy() for o in local(torch.from_numpy(imgs))]
    rb = sum(f.nbytes for f in local.outputs)
    rows = encode_rows(outs, 2)
    for i in range(2):
        ref = local.format(decode_row(rows[i * rb:(i + 1) * rb], local.outputs))
        assert [a["species"] for a in got[i]["animals"]] == [a["species"] for a in ref["animals"]]
        assert [a["bbox"] for a in got[i]["animals"]] == [a["bbox"] for a in ref["animals"]]
    w = stats["workers"][0]
    assert w["xgmi_tx_bytes"] > 0 and w["xgmi_rx_bytes"] > 0  # crops out, classifications back


def test_spatial_landcover_group_matches_single_process():
    import base64
    import io

    from PIL import Image

    from aiforearth_api_platform_amd.models import zoo
    kw = dict(height=256, width=256, tile=128, stride=112, tile_batch=4)
    mosaic = np.random.default_rng(6).integers(0, 256, (1, 256, 256, 4), dtype=np.uint8)
    spec = ModelSpec("aiforearth_api_platform_amd.models.zoo:landcover_spatial", (256, 256, 4), 1, 5, kw, False,
                     (), (), 3)
    got, stats = _serve(spec, ["cpu", "cpu", "cpu"], mosaic, "/v1/group/in")
    cls = np.asarray(Image.open(io.BytesIO(base64.b64decode(got[0]["class_map"]))))
    # the group's CPU processes run os.cpu_count() // 3 intra-op threads each (gpu_worker._share_cpu): the reference
    # uses the same count, so the fp32 reductions (and the argmax) are the same
    nt = torch.get_num_threads()
    torch.set_num_threads(max(1, (os.cpu_count() or 1) // 3))
    try:
        ref = zoo.landcover("cpu", **kw)(torch.from_numpy(mosaic))[0][0].numpy()
    finally:
        torch.set_num_threads(nt)
    assert np.array_equal(cls, ref)
    assert stats["workers"][0]["xgmi_rx_bytes"] > 0


def test_ensemble_pair_recovers_from_failed_xgmi_handoff(monkeypatch):
    """A hand-off that fails before anything is on the wire fails the batch launch; the worker re-runs
    the batch's items one by one and every task completes (survey §5.3 fault injection)."""
    # CPU engines skip the warmup pass, so hand-off 1 is the first real batch
    monkeypatch.setenv("AI4E_FAULT_INJECTION", "xgmi_fail_batch=1")
    imgs = np.random.default_rng(8).integers(0, 256, (2, 128, 128, 3), dtype=np.uint8)
    spec = ModelSpec("aiforearth_api_platform_amd.models.zoo:camera_trap_ensemble_pair", (128, 128, 3), 2, 5, ENS,
                     False, (), ("http://127.0.0.1/v1/group/classify",), 2)
    got, stats = _serve(spec, ["cpu", "cpu"], imgs, "/v1/group/classify")
    assert all(g is not None and "animals" in g for g in got)


@pytest.mark.parametrize("world,leaders", [(4, 3), (4, 2), (8, 7), (8, 6)])
def test_stage_graph_matches_single_process(world, leaders):
    """Config 5 as an N:M stage graph through the pool: 3:1 and 7:1 (detector leaders, each its own scheduler
    connection and batches, feeding one classifier process over P2P), 2:2 and 6:2 (detectors d % 2 per
    classifier); every task equals the single-process ensemble."""
    from aiforearth_api_platform_amd.models import zoo
    from aiforearth_api_platform_amd.runtime.servable import decode_row, encode_rows

    n = 9 if world == 4 else 14
    imgs = np.random.default_rng(11).integers(0, 256, (n, 128, 128, 3), dtype=np.uint8)
    spec = ModelSpec("aiforearth_api_platform_amd.models.zoo:camera_trap_ensemble_group", (128, 128, 3), 2, 5, ENS,
                     False, (), ("http://127.0.0.1/v1/group/classify",), world, leaders)
    got, stats = _serve(spec, ["cpu"] * world, imgs, "/v1/group/classify")
    assert len(stats["workers"]) == leaders and sum(w["images"] for w in stats["workers"]) == n
    local = zoo.camera_trap_ensemble("cpu", **ENS)
    outs = [o.numpy() for o in local(torch.from_numpy(imgs))]
    rb = sum(f.nbytes for f in local.outputs)
    rows = encode_rows(outs, n)
    for i in range(n):
        ref = local.format(decode_row(rows[i * rb:(i + 1) * rb], local.outputs))
        assert [a["species"] for a in got[i]["animals"]] == [a["species"] for a in ref["animals"]]
        assert [a["bbox"] for a in got[i]["animals"]] == [a["bbox"] for a in ref["animals"]]
        assert [a["species_probability"] for a in got[i]["animals"]] == pytest.approx(
            [a["species_probability"] for a in ref["animals"]], abs=1e-4)
    assert sum(w["xgmi_tx_bytes"] for w in stats["workers"]) > 0


def test_stage_assignment():
    from aiforearth_api_platform_amd.runtime.pipeline import stage_assignment

    assert stage_assignment(7, 8) == [[0, 1, 2, 3, 4, 5, 6]]
    assert stage_assignment(6, 8) == [[0, 2, 4], [1, 3, 5]]
    with pytest.raises(ValueError):
        stage_assignment(4, 4)
