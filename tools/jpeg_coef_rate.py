"""CPU entropy-decode rate of the native JPEG coefficient decoder vs PIL's draft decode (threads, frames/s)."""
import io
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd import _ai4e_core as core  # noqa: E402
from aiforearth_api_platform_amd.runtime.decode import decode_image  # noqa: E402


def rate(fn, threads, seconds=2.0):
    stop = time.perf_counter() + seconds
    counts = [0] * threads

    def run(i):
        while time.perf_counter() < stop:
            fn(i)
            counts[i] += 1
    ths = [threading.Thread(target=run, args=(i,)) for i in range(threads)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return sum(counts) / (time.perf_counter() - t0)


import importlib.util  # noqa: E402
_spec = importlib.util.spec_from_file_location(
    "jib", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench", "jpeg_ingest_bench.py"))
jib = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(jib)
body = jib.frame_jpeg(1536, 2048)
bufs = [np.zeros(8 << 20, np.uint8) for _ in range(32)]
for th in (1, 8, 16):
    r1 = rate(lambda i: core.jpeg_coef_decode(body, bufs[i].ctypes.data, bufs[i].nbytes), th)
    r2 = rate(lambda i: decode_image(body, "image/jpeg", (640, 640, 3)), th)
    print(f"threads {th}: coef decode {r1:.0f} frames/s, PIL draft+resize {r2:.0f} frames/s", flush=True)
