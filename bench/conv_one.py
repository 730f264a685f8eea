"""Run ONE K1 conv shape/config repeatedly (for rocprofv3 PMC passes).

    python bench/conv_one.py N H W C K ksize stride tile_cfg [iters]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.ops.conv import conv2d_nhwc, pack_conv  # noqa: E402


def main():
    n, h, w, c, k, ks, s, cfg = (int(v) for v in sys.argv[1:9])
    iters = int(sys.argv[9]) if len(sys.argv) > 9 else 20
    dev = torch.device("cuda:0")
    pc = pack_conv(torch.randn(k, c, ks, ks) / (c * ks * ks) ** 0.5, torch.zeros(k), stride=s, pad=ks // 2).to(dev)
    x = torch.randn(n, h, w, pc.cin_pad, device=dev).bfloat16()
    for _ in range(iters):
        conv2d_nhwc(x, pc, relu=True, tile_cfg=cfg)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
