"""Phase shares of the K1c chain kernels from their s_memtime diagnostic build.

    AI4E_KERNEL_LIB=aiforearth_api_platform_amd/_lib/libai4e_kernels_chainst.so python tools/chain_stamps.py

(build: ``_build.build_kernels(defines=['AI4E_CHAIN_STAMPS=1'], variant='chainst')``). Runs the ResNet-50
stem and layer1 at the serving batch, reads the per-wave phase sums of the LAST chain launch (layer1's third
block: MID 64, next c1 128 wide), then layer2 (last chain: MID 128) and prints each phase's share of a wave's
life. Shares, not lengths (the stamps drain LDS reads)."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50  # noqa: E402
from aiforearth_api_platform_amd.ops import _ext  # noqa: E402
from aiforearth_api_platform_amd.ops.pool import preprocess_s2d_u8  # noqa: E402

NAMES = ["phase A (3x3 main loop)", "B/C weight prologue + T2 epilogue", "passes (B, residual + Y epilogue, C)",
         "T1' epilogue + copy-out (stores drained)", "phase A patch DMA + wait (patch mode)"]


def read(nwaves):
    buf = np.zeros(65536 * 5, np.uint64)
    _ext.call("ai4e_chain_stamps_read", buf.ctypes.data_as(ctypes.c_void_p))
    w = buf.reshape(-1, 5)[:nwaves].astype(np.float64)
    tot = w.sum(0)
    return {"waves": int(nwaves), "cycles_per_wave_mean": round(float(w.sum(1).mean()), 1),
            "shares": {n: round(float(v / tot.sum()), 4) for n, v in zip(NAMES, tot)},
            "cycles_per_wave": {n: round(float(v / max(1, nwaves)), 1) for n, v in zip(NAMES, tot)}}


def main():
    assert hasattr(_ext.lib(), "ai4e_chain_stamps_read"), "run with AI4E_KERNEL_LIB=<a chain stamps build>"
    m = FusedResNet(resnet50(seed=0), device="cuda")
    img = torch.randint(0, 256, (250, 224, 224, 3), dtype=torch.uint8, device="cuda")
    out = {}
    with torch.no_grad():
        for _ in range(2):
            y, t1 = m._stem_t1(preprocess_s2d_u8(img))
            y1, t11 = m._stages_chained(y, t1=t1, s0=0, s1=1)
        torch.cuda.synchronize()
        out["layer1_last_chain"] = read(4 * ((250 * 56 * 56 + 127) // 128))
        for _ in range(2):
            m._stages_chained(y1, t1=t11, s0=1, s1=2)
        torch.cuda.synchronize()
        out["layer2_last_chain"] = read(4 * ((250 * 28 * 28 + 127) // 128))
        # wall time of the whole layer1 / layer2 stages (stamped build: compare variants, not against the release build)
        for name, fn in (("layer1_ms", lambda: m._stages_chained(y, t1=t1, s0=0, s1=1)),
                         ("layer2_ms", lambda: m._stages_chained(y1, t1=t11, s0=1, s1=2))):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            fn()
            ev[0].record()
            for _ in range(10):
                fn()
            ev[1].record()
            torch.cuda.synchronize()
            out[name] = round(ev[0].elapsed_time(ev[1]) / 10, 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
