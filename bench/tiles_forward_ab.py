"""In-process A/B of a whole model forward under two K1 tile tables: both forwards are captured as HIP graphs in ONE
process (the table is read when a conv launches, i.e. at capture) and their replays are interleaved over rounds, so
box-to-box and run-to-run drift cancel (a single bench.py run varies by a few % between processes on one box).

    python bench/tiles_forward_ab.py MODEL TABLE_B [rounds 8] [replays 20]

MODEL: resnet (batch 250 at 224^2), detector (batch 32 at 640^2) or unet (16 tiles of 512^2). TABLE_B: a JSON tile
table (ops/conv_tiles.json format), or ``NAME=VALUE[,NAME=VALUE]`` module switches of ops/conv.py for B (e.g.
``PAIR_X=1``, ``PAIR_TILE=64``: the values its environment variables would set; ``net.par_down=1``: a model
attribute), comma-separated, a table and switches mixed; A is the committed state. Prints one JSON line: median ms per forward of each,
B / A, and the largest output difference (split-K reorders fp32 sums only)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.ops import conv as convmod  # noqa: E402


def build(model: str, dev):
    g = torch.Generator().manual_seed(0)
    if model == "resnet":
        from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50
        net = FusedResNet(resnet50(), device=dev)
        x = torch.randint(0, 256, (250, 224, 224, 3), dtype=torch.uint8, generator=g).to(dev)
    elif model == "detector":
        from aiforearth_api_platform_amd.models.faster_rcnn import DetectorConfig, FasterRCNN
        net = FasterRCNN(DetectorConfig(), seed=0, device=dev)
        x = torch.randint(0, 256, (32, 640, 640, 3), dtype=torch.uint8, generator=g).to(dev)
    elif model == "unet":
        from aiforearth_api_platform_amd.models.unet import FusedUNet, unet_landcover
        net = FusedUNet(unet_landcover(seed=0), device=dev)
        x = torch.randint(0, 256, (16, 512, 512, 4), dtype=torch.uint8, generator=g).to(dev)
    else:
        raise SystemExit(f"unknown model {model}")
    return net, x


def capture(net, x):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            net.forward_u8(x)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        out = net.forward_u8(x)
    torch.cuda.synchronize()
    return gr, out


def first_tensor(out):
    return out if torch.is_tensor(out) else out[0]


def main():
    model, table_b = sys.argv[1], sys.argv[2]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    dev = torch.device("cuda:0")
    net, x = build(model, dev)
    convmod._TILES = None
    ga, oa = capture(net, x)  # committed table
    saved = {}
    for kv in table_b.split(","):
        if kv.endswith(".json"):
            with open(kv) as f:
                convmod._TILES = json.load(f)
        else:
            k, v = kv.split("=")
            obj, k = (net, k[4:]) if k.startswith("net.") else (convmod, k)  # net.X: a model attribute
            saved[(obj, k)] = getattr(obj, k)
            setattr(obj, k, type(saved[(obj, k)])(int(v)))
    gb, ob = capture(net, x)
    convmod._TILES = None
    for (obj, k), v in saved.items():
        setattr(obj, k, v)
    ga.replay()
    gb.replay()
    torch.cuda.synchronize()
    diff = (first_tensor(oa).float() - first_tensor(ob).float()).abs().max().item()
    times = {"A": [], "B": []}
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(rounds):
        for name, gr in (("A", ga), ("B", gb)) if r % 2 == 0 else (("B", gb), ("A", ga)):
            gr.replay()
            st.record()
            for _ in range(reps):
                gr.replay()
            en.record()
            torch.cuda.synchronize()
            times[name].append(st.elapsed_time(en) / reps)
    ma, mb = statistics.median(times["A"]), statistics.median(times["B"])
    print(json.dumps({"model": model, "table_b": os.path.basename(table_b), "ms_A": round(ma, 4),
                      "ms_B": round(mb, 4), "B_over_A": round(mb / ma, 4), "max_out_diff": diff,
                      "A": [round(t, 3) for t in times["A"]], "B": [round(t, 3) for t in times["B"]]}), flush=True)


if __name__ == "__main__":
    main()
