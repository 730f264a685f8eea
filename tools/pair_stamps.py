"""Segment shares of the K1p fused 1x1 pair (layer3: c3 + residual + next c1) from its s_memtime diagnostic build.

    python tools/pair_stamps.py            (builds the variant library, then re-runs itself with it loaded)

(build: ``_build.build_kernels(defines=['AI4E_PAIR_STAMPS=1'], variant='pairst')``). Times the ResNet-50 layer3
pair (14x14, 256 -> 1024 + residual -> 256, BM 96) at the serving batch (250), reads the per-wave segment sums of the
last launch and prints each segment's share of a wave's life (shares, not lengths: a stamp drains LDS reads)."""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = ["prologue (T2 tile, first operands)", "C-weight issue + B phase (incl. weight wait)",
         "residual wait + Y epilogue + barrier", "next-pass loads issue + Y copy-out",
         "C phase (incl. weight wait)", "T1' epilogue + stores (drained)"]
NSEG, MAXW = 6, 32768


def measure():
    import numpy as np
    import torch

    from aiforearth_api_platform_amd.ops import _ext
    from aiforearth_api_platform_amd.ops.conv import conv_pair, pack_conv

    assert hasattr(_ext.lib(), "ai4e_pair_stamps_read"), "run with AI4E_KERNEL_LIB=<a pair stamps build>"
    B, hw, mid, midn, bm = 250, 14, 256, 256, 96  # both variants run 96-pixel tiles
    c4 = 4 * mid
    torch.manual_seed(0)
    c3 = pack_conv(torch.randn(c4, mid, 1, 1) / mid ** 0.5, torch.randn(c4) * 0.1).to("cuda")
    c1n = pack_conv(torch.randn(midn, c4, 1, 1) / c4 ** 0.5, torch.randn(midn) * 0.1).to("cuda")
    t2 = torch.randn(B, hw, hw, mid, device="cuda").relu().bfloat16()
    res = torch.randn(B, hw, hw, c4, device="cuda").bfloat16()
    out = {}
    for cfg in (96, 98):  # 96: loads + stores in a burst after the Y barrier; 98 (default): spread over the C phase
        for _ in range(3):
            conv_pair(t2, c3, res, c1n, tile_cfg=cfg)
        torch.cuda.synchronize()
        nwaves = 8 * ((B * hw * hw + bm - 1) // bm)
        buf = np.zeros(MAXW * NSEG, np.uint64)
        _ext.call("ai4e_pair_stamps_read", buf.ctypes.data_as(ctypes.c_void_p))
        w = buf.reshape(-1, NSEG)[:nwaves].astype(np.float64)
        tot = w.sum(0)
        out[f"layer3_pair_cfg{cfg}"] = {"waves": int(nwaves), "cycles_per_wave_mean": round(float(w.sum(1).mean()), 1),
                                        "shares": {n: round(float(v / tot.sum()), 4) for n, v in zip(NAMES, tot)}}
    print(json.dumps(out, indent=1))


def main():
    if os.environ.get("AI4E_KERNEL_LIB"):
        measure()
        return
    from aiforearth_api_platform_amd import _build

    so = _build.build_kernels(defines=["AI4E_PAIR_STAMPS=1"], variant="pairst")
    env = dict(os.environ, AI4E_KERNEL_LIB=str(so))
    sys.exit(subprocess.call([sys.executable, os.path.abspath(__file__)], env=env))


if __name__ == "__main__":
    main()
