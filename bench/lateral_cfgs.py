"""Time the detector's FPN lateral convs (1x1 + nearest-2x top-down residual, batch 32 at 640²) on every K1 tile
config, alone on the chip (CUDA events, 20 calls, best of 3 rounds).

    python bench/lateral_cfgs.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.ops.conv import conv2d_nhwc, pack_conv, tuned_tile  # noqa: E402

dev = torch.device("cuda:0")
for (h, c) in ((160, 256), (80, 512)):
    pc = pack_conv(torch.randn(256, c, 1, 1) / c ** 0.5, torch.zeros(256)).to(dev)
    x = torch.randn(32, h, h, c, device=dev).bfloat16()
    res = torch.randn(32, h // 2, h // 2, 256, device=dev).bfloat16()
    ref = conv2d_nhwc(x, pc, residual=res, residual_up2=True)
    tuned = tuned_tile(pc, 32, h, h, True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = {}
    for rd in range(3):
        for cfg in range(1, 11):
            try:
                y = conv2d_nhwc(x, pc, residual=res, residual_up2=True, tile_cfg=cfg)
            except Exception as exc:  # a config that refuses the shape
                best[cfg] = str(exc)[:40]
                continue
            e0.record()
            for _ in range(20):
                conv2d_nhwc(x, pc, residual=res, residual_up2=True, tile_cfg=cfg)
            e1.record()
            torch.cuda.synchronize()
            assert (y.float() - ref.float()).abs().max().item() < 0.1
            t = e0.elapsed_time(e1) * 50
            best[cfg] = min(best.get(cfg, 1e9), t) if isinstance(best.get(cfg, 0), float) or cfg not in best else t
    print(f"lateral h{h} c{c} (tuned cfg {tuned}): " + ", ".join(
        f"{k}: {v:.1f}" if isinstance(v, float) else f"{k}: {v}" for k, v in best.items()), flush=True)
