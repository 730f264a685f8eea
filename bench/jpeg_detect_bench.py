"""Camera-trap detection API fed with JPEG frames (one MI355X): the request path of a real camera-trap client.

Client threads POST-equivalent ``ModelEndpoint.submit(body, "image/jpeg")`` calls of 2048x1536 camera frames to the
detector endpoint (Faster-RCNN R50-FPN 640^2, batch 32, ``models.zoo:megadetector``) and keep a bounded number of
requests outstanding; images/s = tasks completed per second in the timed window. Modes:

* ``gpu``: the front-end prepares each frame into its ring slot (headers + unstuffed scan, ~0.2 ms) and the worker
  decodes it on the GPU into the detector's input (runtime/jpeg_gpu.py);
* ``cpu``: the front-end decodes on CPU threads (PIL draft decode + resize, ``decode_image``) into the slot;
* ``raw``: the frames are decoded once up front and submitted as pixels (the detector's own rate, no decode).

    python bench/jpeg_detect_bench.py [--modes gpu,cpu,raw --threads 16 --seconds 10]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))


def run_http(mode, body, shape, seconds, batch, frontends, max_queue_ms, conc):
    """The same detector behind the REST front door: 4 native front-ends, the C++ load generator posting the JPEG
    frame as ``image/jpeg`` from 4 processes x ``conc`` connections. gpu: the front-ends prepare frames into ring
    slots; cpu: they proxy JPEG bodies to the serving process, which decodes them with PIL. (At ~4k images/s a 15 ms
    budget holds ~60 requests: 128 clients always find it full and back off; 4 x 12 keeps about a budget in flight.)"""
    from aiforearth_api_platform_amd.config import Config
    from aiforearth_api_platform_amd.gateway.control import ControlPlane
    from aiforearth_api_platform_amd.runtime.node_bench import http_phase
    from aiforearth_api_platform_amd.runtime.worker_pool import ModelSpec, WorkerPool

    cp = ControlPlane(Config.load(env={}))
    spec = ModelSpec("aiforearth_api_platform_amd.models.zoo:megadetector", shape, batch, 5)
    pool = WorkerPool(cp, "http://127.0.0.1/v1/bench/async", spec, ["cuda:0"], jpeg_slots=(mode == "gpu"),
                      frontends=frontends)
    try:
        pool.start(wait_ready_s=900)
        res = http_phase(cp, pool, 2 * seconds, batch, shape, "/v1/bench/async", frontends=frontends,
                         max_queue_ms=max_queue_ms, jpeg=body, phases=("jpeg_route",), jpeg_conc=conc)
        r = res["jpeg_route"]
        return {k: r.get(k) for k in ("images_per_s", "busy_429", "errors", "p50_task_latency_ms",
                                      "p99_task_latency_ms", "server_cpu_s", "server_cpu_split_s", "client_cpu_s",
                                      "window_s", "connections", "p50_request_latency_ms", "p99_request_latency_ms")}
    finally:
        pool.stop()
        cp.close()


def run(mode, bodies, shape, threads, seconds, outstanding, batch):
    from aiforearth_api_platform_amd.config import Config
    from aiforearth_api_platform_amd.gateway.control import ControlPlane
    from aiforearth_api_platform_amd.runtime.decode import decode_image
    from aiforearth_api_platform_amd.runtime.model_endpoint import ModelEndpoint
    from aiforearth_api_platform_amd.runtime.worker_pool import ModelSpec, WorkerPool

    cp = ControlPlane(Config.load(env={}))
    spec = ModelSpec("aiforearth_api_platform_amd.models.zoo:megadetector", shape, batch, 5)
    pool = WorkerPool(cp, "http://127.0.0.1/v1/animal_detection", spec, ["cuda:0"], jpeg_slots=(mode == "gpu"))
    ep = ModelEndpoint(cp, "/v1/animal_detection", worker=pool)
    done_path = "/v1/animal_detection_completed"
    try:
        pool.start(wait_ready_s=900)
        raw = np.stack([decode_image(b, "image/jpeg", shape) for b in bodies]) if mode == "raw" else None
        sem = threading.Semaphore(outstanding)
        stop = time.perf_counter() + seconds + 3.0
        submitted = [0] * threads

        def on_done(_tid):
            sem.release()

        def client(i):
            k = i
            while time.perf_counter() < stop:
                sem.acquire()
                if raw is not None:
                    ep.submit(raw[k % len(raw)].tobytes(), "application/octet-stream", on_done=on_done)
                else:
                    ep.submit(bodies[k % len(bodies)], "image/jpeg", on_done=on_done)
                submitted[i] += 1
                k += threads

        ths = [threading.Thread(target=client, args=(i,), daemon=True) for i in range(threads)]
        for t in ths:
            t.start()
        time.sleep(3.0)  # warm-up: graphs replaying, ring in steady state
        c0, t0 = cp.store.zcard(done_path), time.perf_counter()
        time.sleep(seconds)
        c1, t1 = cp.store.zcard(done_path), time.perf_counter()
        for t in ths:
            t.join(60)
        w = pool.stats()["workers"][0] if pool.stats().get("workers") else {}
        return {"images_per_s": round((c1 - c0) / (t1 - t0), 1), "completed": c1 - c0, "threads": threads,
                "outstanding": outstanding, "worker": {k: w.get(k) for k in ("batches", "images", "gpu_busy_ms")}}
    finally:
        ep.stop()
        cp.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="gpu,cpu,raw")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--outstanding", type=int, default=128)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--http", action="store_true", help="through the REST front door (native front-ends)")
    ap.add_argument("--frontends", type=int, default=4)
    ap.add_argument("--max-queue-ms", type=float, default=15.0)
    ap.add_argument("--conc", type=int, default=12, help="connections per load-generator process (4 processes)")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    from jpeg_ingest_bench import frame_jpeg

    bodies = [frame_jpeg(1536, 2048, quality=q) for q in (90, 85, 80, 75)]
    out = {"metric": "camera-trap detection API images/s with JPEG clients (1 GPU)", "frame": [1536, 2048],
           "model": "megadetector (Faster-RCNN R50-FPN, random init)", "input": [640, 640, 3], "results": {}}
    for mode in a.modes.split(","):
        if a.http:
            if mode == "raw":
                continue
            out["results"][f"http_{mode}"] = run_http(mode, bodies[0], (640, 640, 3), a.seconds, a.batch, a.frontends,
                                                      a.max_queue_ms, a.conc)
            print(f"http_{mode}", out["results"][f"http_{mode}"], flush=True)
            continue
        out["results"][mode] = run(mode, bodies, (640, 640, 3), a.threads, a.seconds, a.outstanding, a.batch)
        print(mode, out["results"][mode], flush=True)
    line = json.dumps(out)
    print(line)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
