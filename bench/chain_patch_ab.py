"""A/B of K1c chain tile configs (CHAIN_CFGS, default: LDS-DMA ring (tile 1 / 0) vs the LDS input patch (tile 3);
+16 = 2 x 2 phase-A split, +32 = padded MID-128 patch), ResNet-50 shapes
at batch 250. Each shape is timed alone and as two launches on two streams at once (the serving worker's two
compute streams share the chip)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50  # noqa: E402
from aiforearth_api_platform_amd.ops.conv import conv_chain  # noqa: E402


def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(n):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / n * 1e3


def main():
    B = int(os.environ.get("B", "250"))
    dev = torch.device("cuda:0")
    m = FusedResNet(resnet50(), device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    cases = []
    l1, l2 = m.stages[0], m.stages[1]
    cases.append(("layer1 next64", 56, l1[1][1], l1[1][2], l1[2][0]))
    cases.append(("layer1 next128", 56, l1[2][1], l1[2][2], l2[0][0]))
    cases.append(("layer2 next128", 28, l2[1][1], l2[1][2], l2[2][0]))
    cases.append(("layer2 last", 28, l2[3][1], l2[3][2], None))
    for name, hw, c2, c3, c1n in cases:
        mid = c2.cout
        t1 = [torch.randn(B, hw, hw, mid, device=dev).relu().bfloat16() for _ in range(2)]
        res = [torch.randn(B, hw, hw, 4 * mid, device=dev).bfloat16() for _ in range(2)]
        r = {"case": name, "B": B}
        cfgs = [int(c) for c in os.environ.get("CHAIN_CFGS", "").split(",") if c] or [1 if mid == 64 else 0, 3]
        ref = cfgs[0]
        outs = {}
        for cfg in cfgs:
            r[f"tile{cfg}_us"] = round(timed(lambda: conv_chain(t1[0], c2, c3, res[0], c1n=c1n, tile_cfg=cfg)), 1)

            def pair():
                cur = torch.cuda.current_stream()
                s1.wait_stream(cur)
                s2.wait_stream(cur)
                with torch.cuda.stream(s1):
                    conv_chain(t1[0], c2, c3, res[0], c1n=c1n, tile_cfg=cfg)
                with torch.cuda.stream(s2):
                    conv_chain(t1[1], c2, c3, res[1], c1n=c1n, tile_cfg=cfg)
                cur.wait_stream(s1)
                cur.wait_stream(s2)
            r[f"tile{cfg}_2streams_us"] = round(timed(pair), 1)
            y, t = conv_chain(t1[0], c2, c3, res[0], c1n=c1n, tile_cfg=cfg)
            outs[cfg] = (y.float(), None if t is None else t.float())
        torch.cuda.synchronize()
        for cfg in cfgs[1:]:
            r[f"max_abs_diff_y_{cfg}"] = (outs[ref][0] - outs[cfg][0]).abs().max().item()
            if outs[ref][1] is not None:
                r[f"max_abs_diff_t1n_{cfg}"] = (outs[ref][1] - outs[cfg][1]).abs().max().item()
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
