"""K1 conv micro-benchmark on arbitrary shapes: TFLOP/s per tile config (+ hipBLASLt GEMM of equal size).
CFGS=9,10 picks the tile configs; TWO=1 also times two copies on two streams at once (the serving worker's
two compute streams), reported as TFLOP/s of both together.

    python bench/conv_micro.py N H W C K ksize stride [N H W C K ksize stride ...]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.ops.conv import conv2d_nhwc, pack_conv  # noqa: E402


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
    a = [int(v) for v in sys.argv[1:]]
    dev = torch.device("cuda:0")
    for i in range(0, len(a), 7):
        n, h, w, c, k, ks, s = a[i:i + 7]
        pc = pack_conv(torch.randn(k, c, ks, ks) / (c * ks * ks) ** 0.5, torch.zeros(k), stride=s, pad=ks // 2).to(dev)
        x = torch.randn(n, h, w, pc.cin_pad, device=dev).bfloat16()
        oh, ow = pc.out_hw(h, w)
        M, K = n * oh * ow, ks * ks * pc.cin_pad
        flops = 2.0 * M * k * K
        out = {"shape": f"n{n} {h}x{w} {c}->{k} k{ks} s{s}", "M": M, "N": k, "K": K}
        cfgs = [int(c) for c in os.environ.get("CFGS", "1,2,3,4,5,6").split(",")]
        x2 = x.clone()
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        for cfg in cfgs:
            try:
                t = timed(lambda: conv2d_nhwc(x, pc, relu=True, tile_cfg=cfg))
            except RuntimeError:
                continue
            out[f"cfg{cfg}"] = round(flops / t / 1e6, 1)
            out[f"cfg{cfg}_us"] = round(t, 1)
            if os.environ.get("TWO"):
                def two():
                    cur = torch.cuda.current_stream()
                    s1.wait_stream(cur)
                    s2.wait_stream(cur)
                    with torch.cuda.stream(s1):
                        conv2d_nhwc(x, pc, relu=True, tile_cfg=cfg)
                    with torch.cuda.stream(s2):
                        conv2d_nhwc(x2, pc, relu=True, tile_cfg=cfg)
                    cur.wait_stream(s1)
                    cur.wait_stream(s2)
                t2 = timed(two)
                out[f"cfg{cfg}_2s"] = round(2 * flops / t2 / 1e6, 1)
        A = torch.randn(M, K, device=dev).bfloat16()
        B = torch.randn(K, k, device=dev).bfloat16()
        out["gemm"] = round(flops / timed(lambda: A @ B) / 1e6, 1)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
