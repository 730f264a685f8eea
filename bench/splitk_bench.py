"""Split-K A/B for the small-grid ResNet-50 convs at the serving batch (250): each shape's committed tile config
against the 256-wide configs with K split over two workgroups per output tile (``ops.conv.split_cfg``).

Prints one JSON line per shape: microseconds per launch (CUDA events over 20 launches) and the largest deviation
of each config's output from the committed config's (split-K only reorders the fp32 sums)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.ops.conv import conv2d_nhwc, pack_conv, tuned_tile  # noqa: E402

# name, cin, cout, k, stride, pad, h, w, residual
SHAPES = [
    ("l4_c2", 512, 512, 3, 1, 1, 7, 7, False),
    ("l4_c2_s2", 512, 512, 3, 2, 1, 14, 14, False),
    ("l3_c2_s2", 256, 256, 3, 2, 1, 28, 28, False),
    ("l3_c2", 256, 256, 3, 1, 1, 14, 14, False),
    ("l4_c1", 2048, 512, 1, 1, 0, 7, 7, False),
    ("l4_c3", 512, 2048, 1, 1, 0, 7, 7, True),
    ("l4_down", 1024, 2048, 1, 2, 0, 14, 14, False),
    ("l3_c1", 1024, 256, 1, 1, 0, 14, 14, False),
    ("l2_down", 256, 512, 1, 2, 0, 56, 56, False),
    ("l3_down", 512, 1024, 1, 2, 0, 28, 28, False),
    ("l4_c1_first", 1024, 512, 1, 1, 0, 14, 14, False),
    ("l2_c1_first", 256, 128, 1, 1, 0, 56, 56, False),
    ("fc", 2048, 1000, 1, 1, 0, 1, 1, False),          # the classifier (1x1 conv over the pooled features)
    # the detector's backbone / FPN (batch 32 at 640^2) and the U-Net's deepest level (16 tiles of 512^2)
    ("det_l4_c2_s2", 512, 512, 3, 2, 1, 40, 40, False, 32),
    ("det_l4_c2", 512, 512, 3, 1, 1, 20, 20, False, 32),
    ("det_fpn_p4", 256, 256, 3, 1, 1, 40, 40, False, 32),
    ("det_fpn_p5", 256, 256, 3, 1, 1, 20, 20, False, 32),
    ("det_lat_c4", 1024, 256, 1, 1, 0, 40, 40, True, 32),
    ("unet_l4", 512, 512, 3, 1, 1, 32, 32, False, 16),
    ("unet_l3", 512, 512, 3, 1, 1, 64, 64, False, 16),
]
CFGS = [6, 9, 10, 6 | 2 << 4, 9 | 2 << 4, 10 | 2 << 4]


def main():
    B = int(os.environ.get("B", "250"))
    cfgs = [int(c) for c in os.environ["SPLITK_CFGS"].split(",")] if os.environ.get("SPLITK_CFGS") else CFGS
    only = set(os.environ["SPLITK_LAYERS"].split(",")) if os.environ.get("SPLITK_LAYERS") else None
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    for name, cin, cout, k, s, p, h, w, res, *nb in SHAPES:
        if only and name not in only:
            continue
        B = nb[0] if nb else int(os.environ.get("B", "250"))
        wt = torch.randn(cout, cin, k, k) / (cin * k * k) ** 0.5
        pc = pack_conv(wt, torch.randn(cout) * 0.1, stride=s, pad=p).to(dev)
        x = torch.randn(B, h, w, pc.cin_pad, device=dev).bfloat16()
        oh, ow = pc.out_hw(h, w)
        r = torch.randn(B, oh, ow, cout, device=dev).bfloat16() if res else None
        base = tuned_tile(pc, B, h, w, res)
        ref = conv2d_nhwc(x, pc, residual=r, relu=True, tile_cfg=base).float()
        us, dev_max = {}, {}
        for cfg in [base] + [c for c in cfgs if c != base]:
            try:
                y = conv2d_nhwc(x, pc, residual=r, relu=True, tile_cfg=cfg)
            except RuntimeError:
                continue
            torch.cuda.synchronize()
            dev_max[cfg] = round((y.float() - ref).abs().max().item(), 4)
            for _ in range(3):
                conv2d_nhwc(x, pc, residual=r, relu=True, tile_cfg=cfg)
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(20):
                conv2d_nhwc(x, pc, residual=r, relu=True, tile_cfg=cfg)
            en.record()
            torch.cuda.synchronize()
            us[cfg] = round(st.elapsed_time(en) / 20 * 1e3, 1)
        best = min(us, key=us.get)
        print(json.dumps({"layer": name, "base": base, "us": us, "maxdev": dev_max, "best": best}), flush=True)


if __name__ == "__main__":
    main()
