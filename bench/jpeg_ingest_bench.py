"""JPEG ingest cost of the image endpoints: decode + resize of camera frames to the model size, on CPU threads and
with the on-GPU reconstruction (``--gpu``: runtime/jpeg_gpu.py, csrc/kernels/jpeg.hip).

Real camera-trap clients post JPEG frames (the reference's detection API takes image files). The
gateway decodes them on CPU threads (`runtime/model_endpoint.decode_image`, Pillow + libjpeg-turbo,
the GIL is released while decoding); JPEG frames far larger than the model input are decoded straight
to 1/2..1/8 scale in the DCT domain ("draft") before the final bilinear resize. This measures frames/s
for both decode paths at 1 and N threads, and for N decode worker processes writing into a shared ring,
for the classifier (224x224) and detector (640x640) sizes.

    python bench/jpeg_ingest_bench.py [--frame 1536x2048 --threads 8 --seconds 3] [--gpu --batch 64]

``--gpu``: ``--threads`` CPU threads prepare the frames (header parse + unstuffed copy, ~0.2 ms each) and one GPU does
the rest, batches pipelined (batch i+1 is prepared while the GPU decodes batch i); the output of every frame is
checked against ``decode_image`` (the CPU path the endpoints use) and the maximum absolute difference reported.
"""
import argparse
import io
import json
import os
import sys
import threading
import time

import numpy as np
from PIL import Image

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.runtime.model_endpoint import decode_image  # noqa: E402


def frame_jpeg(h, w, quality=90):
    rng = np.random.default_rng(0)
    base = rng.integers(0, 256, (max(h // 16, 1), max(w // 16, 1), 3), dtype=np.uint8)
    buf = io.BytesIO()
    Image.fromarray(base).resize((w, h), Image.BILINEAR).save(buf, "JPEG", quality=quality)
    return buf.getvalue()


def full_decode(body, shape):
    h, w, _ = shape
    return np.asarray(Image.open(io.BytesIO(body)).convert("RGB").resize((w, h), Image.BILINEAR))


def rate(fn, body, shape, threads, seconds):
    stop = time.perf_counter() + seconds
    counts = [0] * threads

    def run(i):
        while time.perf_counter() < stop:
            fn(body, shape)
            counts[i] += 1

    ths = [threading.Thread(target=run, args=(i,)) for i in range(threads)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return sum(counts) / (time.perf_counter() - t0)


def gpu_rate(bodies, shape, threads, batch, seconds, span_bits=0):
    """Frames/s of the on-GPU path over `seconds`, and the max |GPU - decode_image| over the distinct bodies."""
    import torch

    from aiforearth_api_platform_amd.runtime.jpeg_gpu import DEFAULT_SPAN_BITS, JpegGpuDecoder

    dec = JpegGpuDecoder(shape, "cuda", threads=threads, span_bits=span_bits or DEFAULT_SPAN_BITS)
    frames = [bodies[i % len(bodies)] for i in range(batch)]
    out = dec.decode(frames)  # warm-up (allocations, coefficient tables)
    torch.cuda.synchronize()
    diff = 0
    for i, b in enumerate(bodies):
        ref = decode_image(b, "image/jpeg", shape)
        diff = max(diff, int(np.abs(out[i].cpu().numpy().astype(np.int16) - ref).max()))
    outs = [torch.empty((batch,) + tuple(shape), dtype=torch.uint8, device="cuda") for _ in range(2)]
    n = 0
    t0 = time.perf_counter()
    pend = None
    k = 0
    while time.perf_counter() - t0 < seconds:
        p = dec.submit(frames, outs[k & 1])
        if pend is not None:
            dec.finish(pend)
        pend = p
        n += batch
        k += 1
    dec.finish(pend)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    stats = dict(dec.stats)
    host = {name: round(v / (k + 1) * 1e3, 3) for name, v in dec.host_s.items()}  # ms per batch (k timed + warm-up)
    dec.close()
    return {"frames_per_s": round(n / dt, 1), "batch": batch, "cpu_threads": threads, "max_abs_diff_vs_decode_image":
            diff, "gpu_frames": stats["gpu_frames"], "cpu_fallback_frames": stats["cpu_frames"],
            "span_bits": dec.launcher.span_bits, "host_ms_per_batch": host}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frame", default="1536x2048")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--json-out", default="")
    ap.add_argument("--gpu", action="store_true", help="only the on-GPU reconstruction (one GPU)")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--span-bits", type=int, default=0, help="entropy-coded bits per decoder thread (0: default)")
    a = ap.parse_args()
    h, w = (int(v) for v in a.frame.split("x"))
    body = frame_jpeg(h, w)
    if a.gpu:
        bodies = [frame_jpeg(h, w, quality=q) for q in (90, 85, 80, 75)]
        out = {"metric": "JPEG frames decoded + resized per second (on-GPU reconstruction, 1 GPU)", "frame": [h, w],
               "jpeg_bytes": [len(b) for b in bodies], "threads": a.threads, "results": {}}
        for shape in ((640, 640, 3), (224, 224, 3)):
            out["results"][f"{shape[0]}x{shape[1]}"] = gpu_rate(bodies, shape, a.threads, a.batch, a.seconds,
                                                                 a.span_bits)
        line = json.dumps(out)
        print(line)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
        return
    out = {"metric": "JPEG frames decoded + resized per second (CPU)", "frame": [h, w], "jpeg_bytes": len(body),
           "threads": a.threads, "cpu_count": os.cpu_count(), "results": {}}
    for shape in ((224, 224, 3), (640, 640, 3)):
        ref = full_decode(body, shape)
        got = decode_image(body, "image/jpeg", shape)
        r = {"mean_abs_diff_vs_full_decode": round(float(np.abs(got.astype(np.int16) - ref).mean()), 3)}
        for name, fn in (("full_decode", full_decode), ("draft_decode", lambda b, s: decode_image(b, "image/jpeg", s))):
            r[name] = {"1_thread": round(rate(fn, body, shape, 1, a.seconds), 1),
                       f"{a.threads}_threads": round(rate(fn, body, shape, a.threads, a.seconds), 1)}
        out["results"][f"{shape[0]}x{shape[1]}"] = r
    # decode worker processes writing into a shared ring (runtime/decode_pool.py, `decode_processes: N`)
    from multiprocessing import shared_memory

    from aiforearth_api_platform_amd.runtime.decode_pool import DecodePool
    for shape in ((224, 224, 3), (640, 640, 3)):
        nslots = 64
        shm = shared_memory.SharedMemory(create=True, size=nslots * int(np.prod(shape)))
        pool = DecodePool(a.threads, shm.name, nslots, shape)
        try:
            pool.decode_into(0, body, "image/jpeg")  # start the processes
            slot_of = {}
            lock = threading.Lock()

            def one(b, s):
                with lock:
                    k = slot_of.setdefault(threading.get_ident(), len(slot_of))
                pool.decode_into(k, b, "image/jpeg")

            out["results"][f"{shape[0]}x{shape[1]}"][f"decode_processes_{a.threads}"] = round(
                rate(one, body, shape, 2 * a.threads, a.seconds), 1)
        finally:
            pool.close()
            shm.close()
            shm.unlink()
    line = json.dumps(out)
    print(line)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
