"""Segment shares of the 256-wide K1 (config 9: 192-pixel tiles, 4-phase ping-pong) from its s_memtime diagnostic build.

    python tools/k256_stamps.py            (builds the variant library, then re-runs itself with it loaded)

(build: ``_build.build_kernels(defines=['AI4E_K256_STAMPS=1'], variant='k256st')``). Times the ResNet-50 layer3 3x3
(14x14, 256 -> 256, K 2304) and layer4 3x3 (7x7, 512 -> 512, K 4608) convs at the serving batch (250) with config 9,
reads the per-wave segment sums of the last launch and prints each segment's share of a wave's life. Shares, not
lengths: every stamp drains the wave's outstanding LDS reads, which moves their latency into the issue segment."""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = ["reads + DMA issue", "vmcnt wait", "barriers (+ lgkmcnt)", "MFMA", "prologue", "epilogue"]
NSEG, MAXW = 6, 32768


def measure():
    import numpy as np
    import torch

    from aiforearth_api_platform_amd.ops import _ext
    from aiforearth_api_platform_amd.ops.conv import conv2d_nhwc, pack_conv

    assert hasattr(_ext.lib(), "ai4e_k256_stamps_read"), "run with AI4E_KERNEL_LIB=<a k256 stamps build>"
    out = {}
    for name, (n, hw, c, k) in {"layer3_3x3": (250, 14, 256, 256), "layer4_3x3": (250, 7, 512, 512)}.items():
        torch.manual_seed(0)
        pc = pack_conv(torch.randn(k, c, 3, 3) / (9 * c) ** 0.5, torch.zeros(k), pad=1).to("cuda")
        x = torch.randn(n, hw, hw, c, device="cuda").bfloat16()
        for _ in range(3):
            conv2d_nhwc(x, pc, relu=True, tile_cfg=9)
        torch.cuda.synchronize()
        nwaves = 8 * ((n * hw * hw + 191) // 192) * ((k + 255) // 256)
        buf = np.zeros(MAXW * NSEG, np.uint64)
        _ext.call("ai4e_k256_stamps_read", buf.ctypes.data_as(ctypes.c_void_p))
        w = buf.reshape(-1, NSEG)[:nwaves].astype(np.float64)
        tot = w.sum(0)
        # the two wave groups (waves 0-3 lead, 4-7 trail by one barrier) separately
        grp = w.reshape(-1, 8, NSEG)
        out[name] = {"waves": int(nwaves), "cycles_per_wave_mean": round(float(w.sum(1).mean()), 1),
                     "shares": {nm: round(float(v / tot.sum()), 4) for nm, v in zip(NAMES, tot)},
                     "shares_leading_group": {nm: round(float(v), 4) for nm, v in
                                              zip(NAMES, grp[:, :4].sum((0, 1)) / grp[:, :4].sum())},
                     "shares_trailing_group": {nm: round(float(v), 4) for nm, v in
                                               zip(NAMES, grp[:, 4:].sum((0, 1)) / grp[:, 4:].sum())}}
    print(json.dumps(out, indent=1))


def main():
    if os.environ.get("AI4E_KERNEL_LIB"):
        measure()
        return
    from aiforearth_api_platform_amd import _build

    so = _build.build_kernels(defines=["AI4E_K256_STAMPS=1"], variant="k256st")
    env = dict(os.environ, AI4E_KERNEL_LIB=str(so))
    sys.exit(subprocess.call([sys.executable, os.path.abspath(__file__)], env=env))


if __name__ == "__main__":
    main()
