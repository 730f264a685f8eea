"""Host-side capacity probe for the serving path (runs on the GPU box, CPU only).

Measures what one scheduler process can do per second on this machine: uint8 image copies into a
shared-memory payload ring (the per-request ingest write), at 1 thread and at the torch intra-op
thread count, so the bench's ingest design is sized from numbers, not guesses.
"""
import json
import os
import time
from multiprocessing import shared_memory

import numpy as np
import torch


def main():
    B, S = 250, 224
    img = S * S * 3
    src = torch.randint(0, 256, (B * 4, S, S, 3), dtype=torch.uint8)
    shm = shared_memory.SharedMemory(create=True, size=B * 8 * img)
    try:
        dst = torch.frombuffer(shm.buf, dtype=torch.uint8, count=B * 8 * img).view(B * 8, S, S, 3)
        out = {"cpu_count": os.cpu_count(), "torch_threads": torch.get_num_threads(),
               "affinity": len(os.sched_getaffinity(0))}
        for threads in (1, 4, torch.get_num_threads()):
            torch.set_num_threads(threads)
            n = 40
            t0 = time.perf_counter()
            for i in range(n):
                dst[(i % 8) * B:(i % 8 + 1) * B].copy_(src[(i % 4) * B:(i % 4 + 1) * B])
            dt = time.perf_counter() - t0
            out[f"ring_copy_GBps_t{threads}"] = round(n * B * img / dt / 1e9, 2)
            out[f"ring_copy_img_per_s_t{threads}"] = round(n * B / dt)
        # per-image copies (one request at a time, as an HTTP front end would do)
        torch.set_num_threads(1)
        t0 = time.perf_counter()
        n = 2000
        for i in range(n):
            dst[i % (B * 8)].copy_(src[i % (B * 4)])
        out["per_image_copy_img_per_s"] = round(n / (time.perf_counter() - t0))
        del dst
    finally:
        shm.close()
        shm.unlink()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
