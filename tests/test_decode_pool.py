"""Image decoding for the endpoints (CPU): JPEG draft decoding stays within a level of a full decode, and
the decode worker processes write the same pixels into the shared payload ring as the in-process path."""
import io
import time

import numpy as np
import pytest
from PIL import Image

from aiforearth_api_platform_amd.config import Config
from aiforearth_api_platform_amd.gateway.control import ControlPlane
from aiforearth_api_platform_amd.runtime.decode import PayloadError, decode_image
from aiforearth_api_platform_amd.runtime.model_endpoint import ModelEndpoint
from aiforearth_api_platform_amd.runtime.worker_pool import ModelSpec, WorkerPool

SHAPE = (32, 32, 3)


def _jpeg(h, w, seed=0):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (h // 16, w // 16, 3), dtype=np.uint8)
    buf = io.BytesIO()
    Image.fromarray(base).resize((w, h), Image.BILINEAR).save(buf, "JPEG", quality=92)
    return buf.getvalue()


def _png(h, w, seed=1):
    a = np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)
    buf = io.BytesIO()
    Image.fromarray(a).save(buf, "PNG")
    return buf.getvalue(), a


def test_jpeg_draft_decode_close_to_full_decode():
    body = _jpeg(768, 1024)
    got = decode_image(body, "image/jpeg", (224, 224, 3))
    full = np.asarray(Image.open(io.BytesIO(body)).convert("RGB").resize((224, 224), Image.BILINEAR))
    assert got.shape == (224, 224, 3) and got.dtype == np.uint8
    assert np.abs(got.astype(np.int16) - full).mean() < 2.0


def test_decode_processes_write_the_ring():
    cp = ControlPlane(Config.load(env={}))
    spec = ModelSpec("aiforearth_api_platform_amd.models.toy:tiny_classifier", SHAPE, max_batch=8, topk=2,
                     use_graphs=False)
    pool = WorkerPool(cp, "http://127.0.0.1/v1/dec/classify", spec, ["cpu"], max_delay_s=0.001)
    ep = ModelEndpoint(cp, "/v1/dec/classify", worker=pool, decode_processes=2)
    seen = {}
    orig_enqueue = ep._enqueue

    def spy(slots, trace=""):  # capture the ring slot's bytes as the task is created
        seen[slots[0]] = ep.ring.buf[slots[0]].numpy().copy()
        return orig_enqueue(slots, trace)

    ep._enqueue = spy
    try:
        pool.start(wait_ready_s=120)
        png, arr = _png(*SHAPE[:2])
        jpg = _jpeg(128, 128)
        for body, ct in ((png, "image/png"), (jpg, "image/jpeg")):
            seen.clear()
            ep.submit(body, ct)
            (pixels,) = seen.values()
            assert np.array_equal(pixels, decode_image(body, ct, SHAPE))
        assert np.array_equal(decode_image(png, "image/png", SHAPE), arr)  # PNG is lossless
        d = time.time() + 60
        while time.time() < d and (cp.store.zcard("/v1/dec/classify_completed") < 2 or ep.ring.slots.used()):
            time.sleep(0.05)
        assert cp.store.zcard("/v1/dec/classify_completed") == 2 and ep.ring.slots.used() == 0
        with pytest.raises(PayloadError) as ei:
            ep.submit(b"\xff\xd8 not a jpeg", "image/jpeg")
        assert ei.value.status == 400
        assert ep.ring.slots.used() == 0  # the slot went back to the ring
    finally:
        ep.stop()
        cp.close()
