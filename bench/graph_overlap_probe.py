"""Do back-to-back replays of one HIP graph on one stream serialize?  A fault-free probe of the topology and
size of the config-5 detector-stage graph: side-stream fork / joins inside the capture (models/resnet.py
``_c1_down_parallel``), a thousand-plus nodes, graph-pool temporaries, ~10 ms of GPU work per replay, so that
the host runs far ahead of the GPU (a deep queue of pending replays) when nothing syncs between them.

Only elementwise ops on fixed-size tensors (no indices, no gathers): a broken order shows up as a wrong count,
never as an out-of-bounds access.  Each replay: ``x = 0``, then ``nodes`` steps of ``x = x + 1`` through fresh
graph-pool temporaries, every ``nodes // forks``-th step on a side stream forked from and joined back into the
capture stream while the main stream bumps ``y``; tail ``acc += x``.  Serialized replays leave
``acc == replays * nodes`` and ``y == replays * forks``.  The linear form (no fork) is the control; ``--inflight``
bounds the replays in flight (0 = unbounded, 1 = host sync after each replay).  One JSON line per case.

``--copy-in-mb N``: the graph's head also reads a static N-MB input that a device-to-device ``copy_`` refreshes
before every replay, on the launch stream (the pattern of runtime/pipeline.py ``_GraphRunner``: ``static_in.copy_(x);
graph.replay()``).

    python bench/graph_overlap_probe.py [--replays 100 --nodes 1500 --forks 4 --elems 1048576 --copy-in-mb 0]
"""
import argparse
import collections
import json
import time

import torch


def build(topology: str, nodes: int, forks: int, elems: int, dev, static_in=None):
    x0 = torch.zeros(elems, device=dev)
    y = torch.zeros(1, device=dev)
    acc = torch.zeros(1, device=dev, dtype=torch.float64)
    cap = torch.cuda.Stream(device=dev)
    side = torch.cuda.Stream(device=dev)
    every = max(1, nodes // max(forks, 1))

    def body():
        x = x0.mul(0.0)
        if static_in is not None:  # read the copied-in input (all zeros): x stays 0
            x = x + static_in[:elems].float()
        for i in range(nodes):
            if topology == "forkjoin" and forks and i % every == every - 1:
                main = torch.cuda.current_stream(dev)
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    t = x + 1.0
                y.add_(1.0)
                main.wait_stream(side)
                t.record_stream(main)
                x = t
            else:
                x = x + 1.0
        acc.add_(x[:1].double())

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
    ap.add_argument("--replays", type=int, default=100)
    ap.add_argument("--nodes", type=int, default=1500)
    ap.add_argument("--forks", type=int, default=4)
    ap.add_argument("--elems", type=int, default=1 << 20)
    ap.add_argument("--copy-in-mb", type=int, default=0)
    a = ap.parse_args()
    dev = torch.device("cuda")
    src = static_in = None
    if a.copy_in_mb:
        n = max(a.copy_in_mb << 20, a.elems)
        src = torch.zeros(n, dtype=torch.uint8, device=dev)
        static_in = torch.zeros_like(src)
    for topology in ("linear", "forkjoin"):
        for inflight in (1, 2, 0):
            g, acc, y = build(topology, a.nodes, a.forks, a.elems, dev, static_in)
            pend = collections.deque()
            t = time.perf_counter()
            ahead = 0
            for _ in range(a.replays):
                if inflight and len(pend) >= inflight:
                    pend.popleft().synchronize()
                if static_in is not None:
                    static_in.copy_(src)
                g.replay()
                ev = torch.cuda.Event()
                ev.record()
                pend.append(ev)
                while len(pend) > 1 and pend[0].query():
                    pend.popleft()
                ahead = max(ahead, len(pend))
            t_host = time.perf_counter() - t
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t
            want_y = a.replays * a.forks if topology == "forkjoin" else 0
            got, ys = float(acc.item()), float(y.item())
            print(json.dumps({"topology": topology, "nodes": a.nodes, "copy_in_mb": a.copy_in_mb,
                              "inflight_bound": inflight or None,
                              "replays": a.replays, "acc": got, "want_acc": float(a.replays * a.nodes), "y": ys,
                              "want_y": float(want_y), "serialized": got == a.replays * a.nodes and ys == want_y,
                              "max_pending_seen": ahead, "host_enqueue_ms": round(t_host * 1e3, 2),
                              "ms_per_replay": round(dt / a.replays * 1e3, 4)}), flush=True)
            del g
    print(json.dumps({"probe": "graph_overlap", "done": True}), flush=True)


if __name__ == "__main__":
    main()
