"""Per-shape tile-config sweep of the K1 conv kernel over every ResNet-50 layer (batch 256).

Prints one JSON line per layer shape with the time of each tile config; ``--write`` stores the
winners in ``aiforearth_api_platform_amd/ops/conv_tiles.json`` (the runtime dispatch table).
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50  # noqa: E402
from aiforearth_api_platform_amd.ops.conv import conv2d_nhwc, tile_key  # noqa: E402


def main():
    B = int(os.environ.get("B", "256"))
    dev = torch.device("cuda:0")
    m = FusedResNet(resnet50(), device=dev)
    h = w = 112
    shapes = [("stem", m.stem, h, w, False)]
    h, w = 56, 56
    for c1, c2, c3, d in m.blocks:
        if d is not None:
            shapes.append(("down", d, h, w, False))
        shapes += [("c1", c1, h, w, False), ("c2", c2, h, w, False)]
        h2, w2 = c2.out_hw(h, w)
        shapes.append(("c3", c3, h2, w2, True))
        h, w = h2, w2
    shapes.append(("fc", m.fc, 1, 1, False))
    seen, table = set(), {}
    for name, pc, hh, ww, res in shapes:
        key = tile_key(pc, B, hh, ww, res)
        if key in seen:
            continue
        seen.add(key)
        x = torch.randn(B, hh, ww, pc.cin_pad, device=dev).bfloat16()
        oh, ow = pc.out_hw(hh, ww)
        r = torch.randn(B, oh, ow, pc.cout, device=dev).bfloat16() if res else None
        times = {}
        for cfg in (1, 2, 3, 4, 5, 6):
            try:
                conv2d_nhwc(x, pc, residual=r, relu=True, tile_cfg=cfg)
            except RuntimeError:
                continue  # config not valid for this shape
            for _ in range(3):
                conv2d_nhwc(x, pc, residual=r, relu=True, tile_cfg=cfg)
            torch.cuda.synchronize()
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(10):
                conv2d_nhwc(x, pc, residual=r, relu=True, tile_cfg=cfg)
            en.record()
            torch.cuda.synchronize()
            times[cfg] = st.elapsed_time(en) / 10 * 1e3
        best = min(times, key=times.get)
        table[key] = best
        print(json.dumps({"layer": name, "key": key, "us": {k: round(v, 1) for k, v in times.items()}, "best": best}),
              flush=True)
    if "--write" in sys.argv:
        path = os.environ.get("TILES_OUT") or os.path.join(
            os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "aiforearth_api_platform_amd", "ops",
            "conv_tiles.json")
        with open(path, "w") as f:
            json.dump(table, f, indent=1, sort_keys=True)
        print("wrote", path)


if __name__ == "__main__":
    main()
