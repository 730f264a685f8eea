"""Phase shares of the direct stem kernel (K1s + fused c1) from its s_memtime diagnostic build.

    AI4E_KERNEL_LIB=aiforearth_api_platform_amd/_lib/libai4e_kernels_stamps.so python tools/stem_stamps.py

(build: ``_build.build_kernels(defines=['AI4E_STEM_STAMPS=1'], variant='stamps')``). Runs the stem + c1 at
the serving batch once eagerly, reads every wave's per-phase cycle sums and prints each phase's share of
the wave's loop time. The stamped build is slower than the real kernel (each stamp drains LDS reads): read
shares, not lengths (cdna_hip_programming.md, In-kernel stamps)."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50  # noqa: E402
from aiforearth_api_platform_amd.ops import _ext  # noqa: E402
from aiforearth_api_platform_amd.ops.conv import stem_pool_c1  # noqa: E402
from aiforearth_api_platform_amd.ops.pool import preprocess_s2d_u8  # noqa: E402

NAMES = ["footprint wait + barrier", "MFMA loop (8 K steps)", "barrier + next footprint DMA issue",
         "epilogue tile writes + barrier", "c1 operand loads + pooling + pooled stores",
         "c1 operand staging + barriers", "c1 MFMA + t1 stores + barrier", "loop overhead"]


def main():
    assert hasattr(_ext.lib(), "ai4e_stem_stamps_read"), "run with AI4E_KERNEL_LIB=<a stamps build>"
    m = FusedResNet(resnet50(seed=0), device="cuda")
    img = torch.randint(0, 256, (250, 224, 224, 3), dtype=torch.uint8, device="cuda")
    x = preprocess_s2d_u8(img)
    c1 = m.stages[0][0][0]
    for _ in range(2):
        stem_pool_c1(x, m.stem, c1)
    torch.cuda.synchronize()
    buf = np.zeros(2048 * 4 * 8, np.uint64)
    _ext.call("ai4e_stem_stamps_read", buf.ctypes.data_as(ctypes.c_void_p))
    per_wave = buf.reshape(-1, 8).astype(np.float64)
    live = per_wave[per_wave.sum(1) > 0]
    tot = live.sum(0)
    out = {"waves": int(live.shape[0]), "cycles_per_wave_mean": float(live.sum(1).mean()),
           "shares": {n: round(float(v / tot.sum()), 4) for n, v in zip(NAMES, tot)}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
