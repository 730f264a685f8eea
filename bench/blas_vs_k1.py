"""1x1 stride-1 convs of ResNet-50 (batch 256) as K1 launches vs hipBLASLt GEMMs with the bias + ReLU
epilogue (torch._addmm_activation) and, for the residual convs, addmm with the residual as C then ReLU.

    python bench/blas_vs_k1.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.ops.conv import conv2d_nhwc, pack_conv  # noqa: E402


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
    dev = torch.device("cuda:0")
    B = 256
    shapes = [(56, 256, 64), (56, 64, 256), (28, 512, 128), (28, 128, 512), (28, 512, 256), (14, 1024, 256),
              (14, 256, 1024), (14, 1024, 512), (7, 2048, 512), (7, 512, 2048)]
    for hw, cin, cout in shapes:
        pc = pack_conv(torch.randn(cout, cin, 1, 1) / cin ** 0.5, torch.randn(cout) * 0.1).to(dev)
        x = torch.randn(B, hw, hw, cin, device=dev).bfloat16()
        res = torch.randn(B, hw, hw, cout, device=dev).bfloat16()
        w = pc.w_packed[:cout, :cin].contiguous()
        bb = pc.bias[:cout].bfloat16()
        x2 = x.reshape(-1, cin)
        t_k1 = timed(lambda: conv2d_nhwc(x, pc, relu=True))
        t_bl = timed(lambda: torch._addmm_activation(bb, x2, w.t()))
        t_k1r = timed(lambda: conv2d_nhwc(x, pc, residual=res, relu=True))
        r2 = res.reshape(-1, cout)
        t_blr = timed(lambda: torch.relu_(torch.addmm(r2, x2, w.t())))
        y1 = conv2d_nhwc(x, pc, relu=True).reshape(-1, cout).float()
        y2 = torch._addmm_activation(bb, x2, w.t()).float()
        err = (y1 - y2).abs().max().item()
        print(f"{hw:3d}x{hw:<3d} {cin:5d}->{cout:<5d} K1 {t_k1:7.1f} us  blas+bias+relu {t_bl:7.1f} us   "
              f"K1+res {t_k1r:7.1f} us  blas(addmm res)+relu {t_blr:7.1f} us   maxdiff {err:.3f}", flush=True)


if __name__ == "__main__":
    main()
