"""On-GPU JPEG reconstruction (runtime/jpeg_gpu.py, csrc/kernels/jpeg.hip, csrc/core/jpeg_span.h).

CPU tests pin every step to the CPU path the endpoints use (runtime/decode.decode_image: PIL draft decode + bilinear
resize): the numpy model of the kernels is bit-exact to it, and the parallel Huffman passes (run on the CPU by
tests/native/jpeg_span_emul.cpp, the kernels' own per-thread code) reproduce the sequential decoder's coefficients.
GPU tests check the HIP kernels against decode_image directly (bit-exact) and the CPU fallback for frames outside
the GPU envelope.
"""
import io
import os
import shutil
import subprocess

import numpy as np
import pytest
from PIL import Image

from aiforearth_api_platform_amd.runtime import jpeg_gpu as jg
from aiforearth_api_platform_amd.runtime.decode import decode_image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def frame(h, w, q=90, sub=None, gray=False, seed=0, smooth=16, **kw):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (max(h // smooth, 1), max(w // smooth, 1), 3), dtype=np.uint8)
    img = Image.fromarray(base).resize((w, h), Image.BILINEAR)
    if gray:
        img = img.convert("L")
    b = io.BytesIO()
    if sub is not None:
        kw["subsampling"] = sub
    img.save(b, "JPEG", quality=q, **kw)
    return b.getvalue()


CASES = [  # (body, model input): 1/2 scale (4x4 luma + 8x8 chroma), 1/4 (2x2 + 4x4), 1/8 (1x1 + 2x2), 4:4:4,
           # greyscale, odd sizes, no draft
    (frame(1536, 2048), (640, 640, 3)),
    (frame(1536, 2048, q=75), (224, 224, 3)),
    (frame(2000, 2600, q=80), (240, 240, 3)),
    (frame(1300, 1700, sub=0, smooth=2), (640, 640, 3)),
    (frame(777, 1023, smooth=1, seed=2), (300, 300, 3)),
    (frame(1536, 2048, gray=True), (640, 640, 3)),
    (frame(500, 600, sub=0, smooth=3), (320, 320, 3)),
]


@pytest.mark.parametrize("k", range(len(CASES)))
def test_reference_pipeline_bit_exact_vs_decode_image(k):
    body, shape = CASES[k]
    got = jg.reference_decode(body, shape)
    assert got is not None
    np.testing.assert_array_equal(got, decode_image(body, "image/jpeg", shape))


def test_pil_coefficients_match_pil_resize():
    rng = np.random.default_rng(0)
    for (sw, sh), (ow, oh) in (((1024, 768), (640, 640)), ((512, 384), (224, 224)), ((300, 200), (300, 120))):
        img = rng.integers(0, 256, (sh, sw, 3), dtype=np.uint8)
        ref = np.asarray(Image.fromarray(img).resize((ow, oh), Image.BILINEAR, reducing_gap=2.0))
        hb, hk = jg.pil_bilinear_coeffs(sw, ow)
        vb, vk = jg.pil_bilinear_coeffs(sh, oh)
        rows = np.zeros((sh, ow, 3), np.int64)
        for x in range(ow):
            x0, n = hb[x]
            rows[:, x] = np.clip(((1 << 21) + np.einsum("k,hkc->hc", hk[x, :n].astype(np.int64),
                                                        img[:, x0:x0 + n].astype(np.int64))) >> 22, 0, 255)
        out = np.zeros((oh, ow, 3), np.int64)
        for y in range(oh):
            y0, n = vb[y]
            out[y] = np.clip(((1 << 21) + np.einsum("k,kwc->wc", vk[y, :n].astype(np.int64), rows[y0:y0 + n])) >> 22,
                             0, 255)
        np.testing.assert_array_equal(out, ref)


def test_plan_envelope():
    hdr = dict(width=2048, height=1536, ncomp=3, hmax=2, vmax=2, nblocks=0,
               comp=((2, 2, 128, 96, 0, 0), (1, 1, 64, 48, 0, 1), (1, 1, 64, 48, 0, 1)))
    p = jg.plan_frame(hdr, 640, 640)
    assert (p.scale, p.ssize, p.src_w, p.src_h) == (2, (4, 8, 8), 1024, 768)
    assert jg.plan_frame(hdr, 224, 224).ssize == (2, 4, 4)
    assert jg.plan_frame(hdr, 1024, 1024) is None  # 4:2:0 at full scale needs fancy upsampling
    assert jg.plan_frame(hdr, 60, 40) is None      # resize with PIL's reducing_gap pre-reduction (256 / 60 / 2 >= 2)
    h422 = dict(hdr, vmax=1, comp=((2, 1, 128, 192, 0, 0), (1, 1, 64, 192, 0, 1), (1, 1, 64, 192, 0, 1)))
    assert jg.plan_frame(h422, 640, 640) is None   # 4:2:2 at 1/2 keeps a vertical upsample


def test_prepare_statuses():
    from aiforearth_api_platform_amd import _ai4e_core as core

    buf = np.zeros(8 << 20, np.uint8)
    body = frame(480, 640)
    st, used = core.jpeg_scan_prepare(body, buf.ctypes.data, buf.nbytes)
    hdr = jg.parse_header(buf[:160].tobytes())
    assert st == jg.ST_OK and hdr["magic"] == jg.SCAN_MAGIC and hdr["bpm"] == 6
    assert used == core.JPEG_SCAN_HEADER_BYTES + hdr["data_bytes"] + 64
    assert core.jpeg_scan_prepare(frame(480, 640, progressive=True), buf.ctypes.data, buf.nbytes)[0] == jg.ST_UNSUPPORTED
    assert core.jpeg_scan_prepare(frame(480, 640, restart_marker_blocks=4), buf.ctypes.data,
                                  buf.nbytes)[0] == jg.ST_UNSUPPORTED
    assert core.jpeg_scan_prepare(body[:1000], buf.ctypes.data, buf.nbytes)[0] in (jg.ST_OK, jg.ST_CORRUPT)
    assert core.jpeg_scan_prepare(body, buf.ctypes.data, 1000)[0] == jg.ST_NOROOM


@pytest.fixture(scope="module")
def emulator(tmp_path_factory):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path_factory.mktemp("emul") / "jpeg_span_emul")
    subprocess.run([gxx, "-O2", "-std=c++17", "-o", exe, os.path.join(ROOT, "tests", "native", "jpeg_span_emul.cpp")],
                   check=True)
    return exe


@pytest.mark.parametrize("k,span,passes", [(0, 1024, 0), (0, 4096, 0), (3, 2048, 0), (4, 512, 0), (5, 4096, 0),
                                           (4, 512, 2), (0, 256, 1)])
def test_parallel_huffman_passes_match_sequential_decoder(emulator, tmp_path, k, span, passes):
    """passes 0: sync passes until nothing changes; else that many, then the sequential fix-up walk."""
    from aiforearth_api_platform_amd import _ai4e_core as core

    body = CASES[k][0]
    buf = np.zeros(32 << 20, np.uint8)
    st, used = core.jpeg_coef_decode(body, buf.ctypes.data, buf.nbytes)
    assert st == 0
    hdr, blocks = jg.coef_planes(buf[:used].tobytes())
    prep = np.zeros(32 << 20, np.uint8)
    st, used2 = core.jpeg_scan_prepare(body, prep.ctypes.data, prep.nbytes)
    assert st == 0
    (tmp_path / "prep.bin").write_bytes(prep[:used2].tobytes())
    r = subprocess.run([emulator, str(tmp_path / "prep.bin"), str(span), str(tmp_path / "coef.bin")]
                       + ([str(passes)] if passes else []), capture_output=True, text=True, check=True)
    assert " bad 0 " in r.stdout, r.stdout
    got = np.fromfile(tmp_path / "coef.bin", np.int16).reshape(-1, 64).astype(np.int64)
    h = jg.parse_header(prep[:160].tobytes())
    u8 = prep[:core.JPEG_SCAN_HEADER_BYTES]
    bc, bdy, bdx = u8[160:176], u8[176:192], u8[192:208]
    quant = np.frombuffer(prep[:1024].tobytes(), np.uint16, 256, 224).reshape(4, 64).astype(np.int64)
    q = np.arange(len(got))
    m, kk = q // h["bpm"], q % h["bpm"]
    for c, comp in enumerate(h["comp"]):
        sel = bc[kk] == c
        row = (m[sel] // h["mcux"]) * comp[1] + bdy[kk[sel]]
        col = (m[sel] % h["mcux"]) * comp[0] + bdx[kk[sel]]
        ref = blocks[c][row, col].reshape(-1, 64)
        np.testing.assert_array_equal(got[sel] * quant[comp[5]][None], ref)


@pytest.mark.gpu
def test_gpu_decode_bit_exact_and_fallback():
    import torch

    shape = (640, 640, 3)
    bodies = [frame(1536, 2048), frame(1536, 2048, q=75, seed=1), frame(1300, 1700, sub=0, smooth=2),
              frame(1536, 2048, gray=True),
              frame(777, 1023, smooth=1, seed=2), frame(400, 500),  # 4:2:0 at full scale (no draft): CPU fallback
              frame(1536, 2048, progressive=True), frame(1536, 2048, restart_marker_blocks=8)]  # CPU fallback
    dec = jg.JpegGpuDecoder(shape, "cuda", threads=4)
    try:
        for rep in range(2):  # second round: the coefficient array was cleared by the first round's IDCT
            out = dec.decode(bodies)
            torch.cuda.synchronize()
            for i, b in enumerate(bodies):
                np.testing.assert_array_equal(out[i].cpu().numpy(), decode_image(b, "image/jpeg", shape),
                                              err_msg=f"frame {i} round {rep}")
        assert dec.stats["gpu_frames"] == 8 and dec.stats["failed"] == 0 and dec.stats["cpu_frames"] == 8
    finally:
        dec.close()


@pytest.mark.gpu
def test_gpu_decode_small_spans_and_other_sizes():
    """Smaller spans need more sync passes (tests/native/jpeg_span_emul.cpp: the noise frame settles after 27 passes at
    1024 bits, 53 at 512); what the passes leave unsettled the fix-up kernel finishes, so every frame is exact."""
    import torch

    bodies = [frame(1536, 2048, seed=s, q=70 + 5 * s) for s in range(4)] + [frame(777, 1023, smooth=1, seed=9)]
    for shape, span, passes in (((224, 224, 3), 1024, 32), ((300, 300, 3), 2048, 16), ((224, 224, 3), 512, 2),
                                ((224, 224, 3), 256, 0 + 1)):
        dec = jg.JpegGpuDecoder(shape, "cuda", threads=2, span_bits=span, sync_passes=passes)
        try:
            pend = [dec.submit(bodies), dec.submit(bodies[::-1])]  # two batches in flight
            outs = [dec.finish(p) for p in pend]
            torch.cuda.synchronize()
            for out, bs in zip(outs, (bodies, bodies[::-1])):
                for i, b in enumerate(bs):
                    np.testing.assert_array_equal(out[i].cpu().numpy(), decode_image(b, "image/jpeg", shape))
            assert dec.stats["failed"] == 0 and dec.stats["gpu_frames"] == 10, dec.stats
        finally:
            dec.close()


@pytest.mark.gpu
def test_gpu_worker_decodes_prepared_slots():
    """A GPU worker pool whose front-end prepares JPEG bodies into ring slots: the worker decodes them on the device
    into the model input (engine.py) and answers exactly as for the same frames decoded on the CPU and sent as pixels;
    a truncated frame fails as an invalid payload."""
    import json
    import time

    from aiforearth_api_platform_amd.config import Config
    from aiforearth_api_platform_amd.gateway.control import ControlPlane
    from aiforearth_api_platform_amd.runtime.model_endpoint import ModelEndpoint
    from aiforearth_api_platform_amd.runtime.worker_pool import ModelSpec, WorkerPool

    shape = (640, 640, 3)
    cp = ControlPlane(Config.load(env={}))
    spec = ModelSpec("aiforearth_api_platform_amd.models.toy:tiny_classifier", shape, max_batch=8, topk=6)
    pool = WorkerPool(cp, "http://127.0.0.1/v1/jpg/classify", spec, ["cuda:0"], max_delay_s=0.001)
    ep = ModelEndpoint(cp, "/v1/jpg/classify", worker=pool)
    try:
        assert pool.ring.jpeg_key  # GPU devices: prepared slots on by default
        pool.start(wait_ready_s=300)
        bodies = [frame(1536, 2048, seed=s, q=75 + 5 * s) for s in range(4)] + [frame(1300, 1700, sub=0, smooth=2)]
        cut = frame(1536, 2048, seed=11)
        jpeg_ids = [json.loads(ep.submit(b, "image/jpeg"))["TaskId"] for b in bodies + [cut[:len(cut) // 2]]]
        raw_ids = ep.submit_many(np.stack([decode_image(b, "image/jpeg", shape) for b in bodies]))
        deadline = time.time() + 120
        while time.time() < deadline and not all(
                cp.store.get_record(t)["BackendStatus"] in ("completed", "failed") for t in jpeg_ids + raw_ids):
            time.sleep(0.02)
        for a, b in zip(jpeg_ids, raw_ids):
            assert ep.result(a) is not None and ep.result(a) == ep.result(b)
        assert cp.store.get_record(jpeg_ids[-1])["BackendStatus"] == "failed"
    finally:
        ep.stop()
        cp.close()


@pytest.mark.gpu
def test_gpu_decode_corrupt_frame_reports_and_recovers():
    import torch

    good = frame(1536, 2048)
    bad = bytearray(good)
    mid = len(bad) // 2
    bad[mid:mid + 64] = bytes(range(64))  # garbage inside the entropy-coded data
    dec = jg.JpegGpuDecoder((640, 640, 3), "cuda", threads=2)
    try:
        out = dec.decode([good, bytes(bad), good])
        torch.cuda.synchronize()
        ref = decode_image(good, "image/jpeg", (640, 640, 3))
        np.testing.assert_array_equal(out[0].cpu().numpy(), ref)
        np.testing.assert_array_equal(out[2].cpu().numpy(), ref)
    finally:
        dec.close()


def test_span_decoder_memory_safe_on_mutated_frames(tmp_path):
    """The kernels' span decoder (compiled for the host with AddressSanitizer + UBSan, tests/native/jpeg_span_emul.cpp)
    over mutated frames: flipped scan bytes, truncations, a garbage scan. Every run must end (bounded passes) without
    a memory error, whatever the decode makes of the bits. The same per-thread code runs in the GPU kernels, whose reads
    are bounded by the same clamps."""
    from aiforearth_api_platform_amd import _ai4e_core as core

    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path / "emul_asan")
    r = subprocess.run([gxx, "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                        "-o", exe, os.path.join(ROOT, "tests", "native", "jpeg_span_emul.cpp")], capture_output=True)
    if r.returncode != 0:
        pytest.skip("sanitizer build unavailable: " + r.stderr.decode()[-200:])
    rng = np.random.default_rng(0)
    base = frame(240, 320, q=85, smooth=2)
    prep = np.zeros(4 << 20, np.uint8)
    runs = 0
    for trial in range(24):
        b = bytearray(base)
        kind = trial % 4
        if kind == 0:  # flip bytes inside the entropy-coded data
            for _ in range(1 + trial):
                i = int(rng.integers(len(b) // 3, len(b) - 2))
                b[i] = int(rng.integers(0, 256))
        elif kind == 1:  # truncate
            b = b[:int(rng.integers(len(b) // 2, len(b)))]
        elif kind == 2:  # replace the scan by noise
            b = b[:len(b) // 3] + bytes(rng.integers(0, 255, len(b) - len(b) // 3, dtype=np.uint8))
        else:  # random bytes anywhere (headers included)
            for _ in range(4):
                i = int(rng.integers(2, len(b)))
                b[i] = int(rng.integers(0, 256))
        st, used = core.jpeg_scan_prepare(bytes(b), prep.ctypes.data, prep.nbytes)
        if st != 0:
            continue
        (tmp_path / "p.bin").write_bytes(prep[:used].tobytes())
        for span, passes in ((512, 3), (2048, 0)):
            r = subprocess.run([exe, str(tmp_path / "p.bin"), str(span), str(tmp_path / "c.bin")]
                               + ([str(passes)] if passes else []), capture_output=True, text=True, timeout=120)
            assert r.returncode == 0, (trial, r.stderr[-2000:])
            runs += 1
    assert runs >= 20
