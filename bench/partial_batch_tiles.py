"""Partial serving batches and the tile table: the K1 table is tuned at the serving batch (250) and looked up by
exact shape, so a dynamic batch of another size falls back to the default tile config. This times the ResNet-50
forward (graph replay) at partial batch sizes with the committed table and with one whose entries for those sizes are
copied from the batch-250 entries.

    python bench/partial_batch_tiles.py [sizes 64,128,192]
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TILES = os.path.join(HERE, "aiforearth_api_platform_amd", "ops", "conv_tiles.json")


def child(sizes):
    import torch

    sys.path.insert(0, HERE)
    from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50

    dev = torch.device("cuda:0")
    m = FusedResNet(resnet50(seed=0), device=dev)
    res = {}
    for n in sizes:
        x = torch.randint(0, 256, (n, 224, 224, 3), dtype=torch.uint8, device=dev)
        for _ in range(3):
            m.forward_u8(x)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            m.forward_u8(x)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(3):
            e0.record()
            for _ in range(20):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / 20)
        res[n] = round(n / best * 1e3, 1)
    print(json.dumps(res), flush=True)


def main():
    sizes = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "64,128,192").split(",")]
    if os.environ.get("PBT_CHILD"):
        return child(sizes)
    with open(TILES) as f:
        t = json.load(f)
    ext = dict(t)
    for k, v in t.items():
        if "n250h" in k:
            for n in sizes:
                ext.setdefault(k.replace("n250h", f"n{n}h"), v)
    alt = os.path.join(HERE, "gpurun_out", "tiles_partial.json")
    os.makedirs(os.path.dirname(alt), exist_ok=True)
    with open(alt, "w") as f:
        json.dump(ext, f)
    for rnd in range(2):
        for name, env in (("committed", {}), ("copied_250", {"AI4E_CONV_TILES": alt})):
            out = subprocess.run([sys.executable, __file__, ",".join(map(str, sizes))], capture_output=True, text=True,
                                 env=dict(os.environ, PBT_CHILD="1", **env), timeout=600)
            line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
            print(f"round {rnd} {name}: images/s {line[-1] if line else out.stderr[-500:]}", flush=True)


if __name__ == "__main__":
    main()
