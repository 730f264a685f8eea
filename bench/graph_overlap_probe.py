"""Do back-to-back replays of one HIP graph on one stream serialize?  A fault-free probe (elementwise torch ops
and a sleep kernel only, no indices, nothing that can address out of bounds) of the topology the config-5 stage
graphs have: a side-stream fork / join inside the capture (models/resnet.py ``_c1_down_parallel``).

Each graph replay does: head ``x = 0`` -> [side branch: sleep, ``x += 1``] beside [main: ``y += 1``] -> join ->
tail ``acc += x``.  Serialized replays leave ``acc == replays`` exactly; a replay whose head runs before the
previous replay's side branch (or whose tail runs before its own side branch) leaves a different count.  The
linear form (the same ops on one stream, no fork) is the control.  One JSON line per case.

    python bench/graph_overlap_probe.py [--replays 200 --sleep-cycles 200000]
"""
import argparse
import json
import time

import torch


def build(topology: str, sleep_cycles: int, dev):
    x = torch.zeros(1, device=dev)
    y = torch.zeros(1, device=dev)
    acc = torch.zeros(1, device=dev, dtype=torch.float64)
    cap = torch.cuda.Stream(device=dev)
    side = torch.cuda.Stream(device=dev)

    def body():
        x.zero_()
        if topology == "forkjoin":
            main = torch.cuda.current_stream(dev)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                torch.cuda._sleep(sleep_cycles)
                x.add_(1)
            y.add_(1)
            main.wait_stream(side)
        else:
            torch.cuda._sleep(sleep_cycles)
            x.add_(1)
            y.add_(1)
        acc.add_(x.double())

    cap.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(cap):
        body()  # eager warmup
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        body()
    torch.cuda.synchronize(dev)
    acc.zero_()
    y.zero_()
    torch.cuda.synchronize(dev)
    return g, acc, y


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replays", type=int, default=200)
    ap.add_argument("--sleep-cycles", type=int, default=200000)
    a = ap.parse_args()
    dev = torch.device("cuda")
    for topology in ("linear", "forkjoin"):
        for synced in (True, False):
            g, acc, y = build(topology, a.sleep_cycles, dev)
            t = time.perf_counter()
            for _ in range(a.replays):
                g.replay()
                if synced:
                    torch.cuda.synchronize(dev)
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t
            got, ys = float(acc.item()), float(y.item())
            rec = {"topology": topology, "host_sync_between_replays": synced, "replays": a.replays,
                   "acc": got, "y": ys, "serialized": got == a.replays and ys == a.replays,
                   "ms_per_replay": round(dt / a.replays * 1e3, 4)}
            print(json.dumps(rec), flush=True)
    print(json.dumps({"probe": "graph_overlap", "done": True}), flush=True)


if __name__ == "__main__":
    main()
