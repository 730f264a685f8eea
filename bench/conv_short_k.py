"""Short-K 1x1 convs (the detector's P2 FPN lateral and stride-2 downsamples, ResNet-50's layer2 downsample) on
their tuned K1 tile config against K1w (tile config 11), alone on the chip: CUDA events, 20 calls, best of 3 rounds.

    python bench/conv_short_k.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.ops.conv import conv2d_nhwc, pack_conv, tuned_tile  # noqa: E402

dev = torch.device("cuda:0")
SHAPES = [  # name, n, h, c, k, stride, residual
    ("det P2 lateral + top-down", 32, 160, 256, 256, 1, "up2"),
    ("det layer2 downsample", 32, 160, 256, 512, 2, None),
    ("resnet layer2 downsample", 250, 56, 256, 512, 2, None),
]
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for name, n, h, c, k, s, res in SHAPES:
    pc = pack_conv(torch.randn(k, c, 1, 1) / c ** 0.5, torch.zeros(k), stride=s).to(dev)
    x = torch.randn(n, h, h, c, device=dev).bfloat16()
    oh = pc.out_hw(h, h)[0]
    r = torch.randn(n, oh // 2, oh // 2, k, device=dev).bfloat16() if res == "up2" else None
    cfgs = [tuned_tile(pc, n, h, h, r is not None) or 1, 11]
    kw = dict(residual=r, residual_up2=res == "up2", relu=r is None)
    outs = [conv2d_nhwc(x, pc, tile_cfg=cf, **kw) for cf in cfgs]
    torch.cuda.synchronize()
    err = (outs[0].float() - outs[1].float()).abs().max().item()
    best = {}
    for rd in range(3):
        for cf in cfgs:
            e0.record()
            for _ in range(20):
                conv2d_nhwc(x, pc, tile_cfg=cf, **kw)
            e1.record()
            torch.cuda.synchronize()
            best[cf] = min(best.get(cf, 1e9), e0.elapsed_time(e1) * 50)
    print(f"{name}: " + ", ".join(f"cfg {cf}: {t:.1f} us" for cf, t in best.items()) + f" (max diff {err:.3g})",
          flush=True)
