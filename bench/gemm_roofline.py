"""Per-layer roofline check: the K1 conv vs. hipBLASLt on the equivalent plain GEMM vs. MIOpen.

For every unique ResNet-50 conv shape at batch B it times
  * ``k1``      — our implicit-GEMM conv (tuned tile config, fused bias/ReLU/residual);
  * ``gemm``    — ``torch.matmul`` of the im2col-sized GEMM [M,K]x[K,N] in bf16 (hipBLASLt), i.e. the
                  same FLOPs with no gather, no epilogue: a practical ceiling for a library GEMM;
  * ``miopen``  — ``F.conv2d`` bf16 channels_last (+bias, no fusion), what stock PyTorch-ROCm runs.
One JSON line per shape (µs and TFLOP/s).  Usage: ``python bench/gemm_roofline.py [B]``.
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50  # noqa: E402
from aiforearth_api_platform_amd.ops.conv import conv2d_nhwc  # noqa: E402


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
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    dev = torch.device("cuda:0")
    m = FusedResNet(resnet50(), device=dev)
    shapes = [("stem", m.stem, 112, 112, False)]
    h = w = 56
    for c1, c2, c3, d in m.blocks:
        if d is not None:
            shapes.append(("down", d, h, w, False))
        shapes += [("c1", c1, h, w, False), ("c2", c2, h, w, False)]
        h2, w2 = c2.out_hw(h, w)
        shapes.append(("c3", c3, h2, w2, True))
        h, w = h2, w2
    seen = set()
    tot = {"k1": 0.0, "gemm": 0.0, "miopen": 0.0}
    for name, pc, hh, ww, res in shapes:
        key = (pc.kh, pc.kw, pc.stride, pc.cin, pc.cout, hh, res)
        if key in seen:
            continue
        seen.add(key)
        oh, ow = pc.out_hw(hh, ww)
        M, N, K = B * oh * ow, pc.cout, pc.kh * pc.kw * pc.cin_pad
        flops = 2.0 * M * N * K
        x = torch.randn(B, hh, ww, pc.cin_pad, device=dev).bfloat16()
        r = torch.randn(B, oh, ow, pc.cout, device=dev).bfloat16() if res else None
        t_k1 = timed(lambda: conv2d_nhwc(x, pc, residual=r, relu=True))
        a = torch.randn(M, K, device=dev).bfloat16()
        b = torch.randn(K, N, device=dev).bfloat16()
        t_gemm = timed(lambda: torch.matmul(a, b))
        del a
        xc = x[..., :pc.cin].permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        wc = pc.w_ref.to(dev).bfloat16().contiguous(memory_format=torch.channels_last)
        bc = pc.b_ref.to(dev).bfloat16()
        pad = pc.pad
        if pc.pad_hi is not None and pc.pad_hi != pc.pad:
            xc = F.pad(xc, (pc.pad, pc.pad_hi, pc.pad, pc.pad_hi)).contiguous(memory_format=torch.channels_last)
            pad = 0
        t_mi = timed(lambda: F.conv2d(xc, wc, bc, stride=pc.stride, padding=pad))
        cnt = sum(1 for s in shapes if (s[1].kh, s[1].kw, s[1].stride, s[1].cin, s[1].cout, s[2], s[4]) == key)
        tot["k1"] += t_k1 * cnt
        tot["gemm"] += t_gemm * cnt
        tot["miopen"] += t_mi * cnt
        print(json.dumps({"layer": name, "shape": f"{pc.kh}x{pc.kw}/s{pc.stride} {pc.cin}->{pc.cout} @{hh}",
                          "count": cnt, "M": M, "N": N, "K": K,
                          "us": {"k1": round(t_k1, 1), "gemm": round(t_gemm, 1), "miopen": round(t_mi, 1)},
                          "tflops": {"k1": round(flops / t_k1 / 1e6, 1), "gemm": round(flops / t_gemm / 1e6, 1),
                                     "miopen": round(flops / t_mi / 1e6, 1)}}), flush=True)
    print(json.dumps({"total_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
