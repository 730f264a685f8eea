"""Time the K1c chain kernel per ResNet-50 stage shape and tile config (batch 256) vs the unfused K1 convs."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50  # noqa: E402
from aiforearth_api_platform_amd.ops.conv import conv2d_nhwc, conv_chain  # noqa: E402


def timed(fn, n=10):
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
    B = int(os.environ.get("B", "256"))
    dev = torch.device("cuda:0")
    m = FusedResNet(resnet50(), device=dev)
    for si, (hw, st) in enumerate([(56, 0), (28, 1)]):
        blocks = m.stages[st]
        _, c2, c3, _ = blocks[1]
        c1n = blocks[2][0]
        mid = c2.cout
        t1 = torch.randn(B, hw, hw, mid, device=dev).relu().bfloat16()
        res = torch.randn(B, hw, hw, 4 * mid, device=dev).bfloat16()
        r = {"stage": st + 1, "mid": mid}
        for cfg in (0, 1):
            try:
                r[f"chain_next_cfg{cfg}"] = round(timed(lambda: conv_chain(t1, c2, c3, res, c1n=c1n, tile_cfg=cfg)), 1)
                r[f"chain_last_cfg{cfg}"] = round(timed(lambda: conv_chain(t1, c2, c3, res, tile_cfg=cfg)), 1)
            except RuntimeError as e:
                r[f"cfg{cfg}"] = str(e)[:60]

        def unfused():
            y2 = conv2d_nhwc(t1, c2, relu=True)
            y = conv2d_nhwc(y2, c3, residual=res, relu=True)
            conv2d_nhwc(y, c1n, relu=True)
        r["unfused_next"] = round(timed(unfused), 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
