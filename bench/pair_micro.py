"""K1p micro-bench: the ResNet-50 layer3 (and layer4) 1x1 pair at the serving batch, fused (one K1p launch per
tile height) vs unfused (c3 + residual on K1, then the next c1 on K1, tuned tiles), HIP-graph replay.

    python bench/pair_micro.py [B]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.ops.conv import conv2d_nhwc, conv_pair, pack_conv  # noqa: E402


def timed(fn, iters=50):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(10):
                fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / (iters * 10)  # us per call


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 250
    dev = "cuda"
    out = {}
    for mid, hw, tiles, midn in ((256, 14, tuple(int(t) for t in os.environ.get("PAIR_TILES", "96,64").split(",")), 256),
                                 (128, 28, (96, 98), 256), (256, 14, (64, 98), 512), (512, 7, (32, 98), 512)):
        c4 = 4 * mid
        torch.manual_seed(0)
        c3 = pack_conv(torch.randn(c4, mid, 1, 1) / mid ** 0.5, torch.randn(c4) * 0.1).to(dev)
        c1n = pack_conv(torch.randn(midn, c4, 1, 1) / c4 ** 0.5, torch.randn(midn) * 0.1).to(dev)
        t2 = torch.randn(B, hw, hw, mid, device=dev).relu().to(torch.bfloat16)
        res = torch.randn(B, hw, hw, c4, device=dev).to(torch.bfloat16)
        y = torch.empty(B, hw, hw, c4, device=dev, dtype=torch.bfloat16)
        t1 = torch.empty(B, hw, hw, midn, device=dev, dtype=torch.bfloat16)

        def unfused():
            conv2d_nhwc(t2, c3, residual=res, relu=True, out=y)
            conv2d_nhwc(y, c1n, relu=True, out=t1)

        r = {"unfused_us": round(timed(unfused), 2),
             "c3_res_us": round(timed(lambda: conv2d_nhwc(t2, c3, residual=res, relu=True, out=y)), 2),
             "c1_us": round(timed(lambda: conv2d_nhwc(y, c1n, relu=True, out=t1)), 2)}
        for t in tiles:
            r[f"pair_bm{t}_us"] = round(timed(lambda t=t: conv_pair(t2, c3, res, c1n, out=y, t1n_out=t1, tile_cfg=t)), 2)
        out[f"mid{mid}_{midn}"] = r
        print(json.dumps({f"mid{mid}_{midn}": r}), flush=True)
    print(json.dumps({"batch": B, **out}))


if __name__ == "__main__":
    main()
