"""Per-shape K1 tile-config sweep for the convs one model forward actually runs (U-Net land-cover tiles,
Faster-RCNN detector batches): records every ``tuned_tile`` lookup during a forward, times tile configs
1-8 on each distinct shape in isolation and, with ``--write``, MERGES the winners into
``aiforearth_api_platform_amd/ops/conv_tiles.json`` (existing keys of other shapes are kept).

    [B=16] python bench/conv_tune_model.py unet [--write]   # B tiles x 512^2 x 4 (bench/landcover_bench.py)
    [B=32] python bench/conv_tune_model.py detector [--write]  # B x 640^2 x 3 (bench/detector_bench.py)
    [B=250] python bench/conv_tune_model.py resnet [--write]   # B x 224^2 x 3 (bench.py serving batch)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.ops import conv as convmod  # noqa: E402

TILES = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "aiforearth_api_platform_amd", "ops",
                     "conv_tiles.json")


def record(run):
    seen = {}
    orig = convmod.tuned_tile

    def rec(pc, n, h, w, residual):
        seen.setdefault(convmod.tile_key(pc, n, h, w, residual), (pc, n, h, w, residual))
        return orig(pc, n, h, w, residual)

    convmod.tuned_tile = rec
    try:
        run()
        torch.cuda.synchronize()
    finally:
        convmod.tuned_tile = orig
    return seen


def time_cfg(pc, n, h, w, res, cfg, dev):
    x = torch.randn(n, h, w, pc.cin_pad, device=dev).bfloat16()
    oh, ow = pc.out_hw(h, w)
    r = torch.randn(n, oh, ow, pc.cout, device=dev).bfloat16() if res else None
    try:
        convmod.conv2d_nhwc(x, pc, residual=r, relu=True, tile_cfg=cfg)
    except RuntimeError:
        return None  # config not valid for this shape
    for _ in range(2):
        convmod.conv2d_nhwc(x, pc, residual=r, relu=True, tile_cfg=cfg)
    torch.cuda.synchronize()
    if PAIR:
        return time_pair(x, pc, r, cfg)
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(5):
        convmod.conv2d_nhwc(x, pc, residual=r, relu=True, tile_cfg=cfg)
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / 5 * 1e3


# TUNE_PAIR=1: time the conv as the serving worker runs it — two compute streams sharing the chip, so a
# grid that leaves CUs idle is not charged for them (per-conv time = wall / launches over both streams)
PAIR = os.environ.get("TUNE_PAIR", "0") == "1"


def time_pair(x, pc, r, cfg, reps=int(os.environ.get("TUNE_REPS", "6"))):
    cur = torch.cuda.current_stream()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    xs = [x, x.clone()]
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record(cur)
    done = []
    for s, xi in zip(streams, xs):
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            for _ in range(reps):
                convmod.conv2d_nhwc(xi, pc, residual=r, relu=True, tile_cfg=cfg)
            e = torch.cuda.Event()
            e.record(s)
            done.append(e)
    for e in done:
        cur.wait_event(e)
    en.record(cur)
    torch.cuda.synchronize()
    return st.elapsed_time(en) / (2 * reps) * 1e3


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "unet"
    dev = torch.device("cuda:0")
    if which == "unet":
        from aiforearth_api_platform_amd.models.unet import FusedUNet, unet_landcover
        m = FusedUNet(unet_landcover(seed=0), device=dev)
        nb = int(os.environ.get("B", "16"))  # tiles per forward (bench/landcover_bench.py --tile-batch)
        img = torch.randint(0, 256, (nb, 512, 512, 4), dtype=torch.uint8, device=dev)
        shapes = record(lambda: m.forward_u8(img))
    elif which == "detector":
        from aiforearth_api_platform_amd.models.faster_rcnn import DetectorConfig, FasterRCNN
        m = FasterRCNN(DetectorConfig(), seed=0, device=dev)
        img = torch.randint(0, 256, (int(os.environ.get("B", "32")), 640, 640, 3), dtype=torch.uint8, device=dev)
        shapes = record(lambda: m.forward_u8(img))
    elif which == "resnet":
        from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50
        m = FusedResNet(resnet50(seed=0), device=dev)
        img = torch.randint(0, 256, (int(os.environ.get("B", "250")), 224, 224, 3), dtype=torch.uint8, device=dev)
        shapes = record(lambda: m.forward_u8(img))
    else:
        raise SystemExit(f"unknown model {which}")
    table = {}
    for key, (pc, n, h, w, res) in shapes.items():
        times = {c: t for c in (1, 2, 3, 4, 5, 6, 7, 8, 9, 10) if (t := time_cfg(pc, n, h, w, res, c, dev)) is not None}
        best = min(times, key=times.get)
        table[key] = best
        print(json.dumps({"key": key, "us": {k: round(v, 1) for k, v in times.items()}, "best": best}), flush=True)
    out_path = os.environ.get("TUNE_OUT")  # write the merged table here instead of the repo table (A/B runs)
    if "--write" in sys.argv or out_path:
        try:
            with open(TILES) as f:
                merged = json.load(f)
        except (OSError, ValueError):
            merged = {}
        merged.update(table)
        with open(out_path or TILES, "w") as f:
            json.dump(merged, f, indent=1, sort_keys=True)
        print("merged", len(table), "entries into", out_path or TILES, flush=True)


if __name__ == "__main__":
    main()
