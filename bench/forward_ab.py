"""Low-noise A/B of model-level variants: HIP-graph replay of the fused ResNet-50 forward (uint8 in, logits
out), variants interleaved over several rounds on one GPU.

    python bench/forward_ab.py chain64=0 chain64=1 [chain=0] [chain=1] ...
A variant is ``key=value[,key=value]`` over: t.<conv tile key> (tile config), chain (K1c on/off), stemu8 (preprocess fused into K1s), chain64 / chain128 (K1c tile config),
pair / pairtile / pairl4 (K1p fused 1x1 pair on/off, tile height, layer4 too), pardown (side-stream downsample).
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50  # noqa: E402
from aiforearth_api_platform_amd.ops import conv as convmod  # noqa: E402


_TILES0 = None


def apply(m, variant):
    global _TILES0
    convmod.tuned_tile(m.stem, 1, 1, 1, False)  # load the measured table, then undo earlier variants' overrides
    _TILES0 = dict(convmod._TILES) if _TILES0 is None else _TILES0
    convmod._TILES = dict(_TILES0)
    m.chain_mb = None
    m.stem_c1 = True
    m.fc_blas = True
    convmod.BLAS_1X1 = False
    convmod.PAIR, convmod.PAIR_TILE, convmod.PAIR_L4, convmod.PAIR_X, convmod.PAIR_B = True, 0, False, False, False
    m.par_down = False
    for kv in variant.split(","):
        if kv == "base":
            continue
        k, v = kv.split("=")
        if k == "chain":
            m.chain = v == "1"
        elif k.startswith("t."):  # t.<tile_key>=<cfg>: override one conv's tile config (ops/conv_tiles.json)
            convmod._TILES[k[2:]] = int(v)
        elif k == "mb":  # chained micro-batching mb:nstages (0 = off)
            m.chain_mb = tuple(int(t) for t in v.split(":")) if ":" in v else None
        elif k == "blas1x1":
            convmod.BLAS_1X1 = v == "1"
        elif k == "fcblas":
            m.fc_blas = v == "1"
        elif k == "stemc1":
            m.stem_c1 = v == "1"
        elif k == "stemu8":
            m.stem_u8 = v == "1"
        elif k == "pair":  # K1p fused c3 + residual + next c1 (layer3; pairl4=1 adds layer4)
            convmod.PAIR = v == "1"
        elif k == "pardown":  # stage-entry downsample on a side stream beside the first c1
            m.par_down = v == "1"
        elif k == "pairtile":
            convmod.PAIR_TILE = int(v)
        elif k == "pairb":  # the layer2 -> layer3 boundary as K1 3x3 + K1p
            convmod.PAIR_B = v == "1"
        elif k == "pairx":  # the layer3 -> layer4 pair (512-wide c1)
            convmod.PAIR_X = v == "1"
        elif k == "pairl4":
            convmod.PAIR_L4 = v == "1"
        elif k.startswith("chain"):
            convmod.CHAIN_TILE[int(k[5:])] = int(v)
        else:
            raise SystemExit(f"unknown variant key {k}")


def main():
    dev = torch.device("cuda:0")
    B = int(os.environ.get("B", "256"))
    variants = sys.argv[1:] or ["chain=1", "chain=0"]
    m = FusedResNet(resnet50(seed=0), device=dev)
    img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=dev)
    graphs = {}
    for v in variants:
        apply(m, v)
        s0 = torch.cuda.Stream(device=dev)
        s0.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s0):
            m.forward_u8(img)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s0):
                m.forward_u8(img)
        torch.cuda.synchronize()
        graphs[v] = g
    res = {v: [] for v in variants}
    for _ in range(4):
        for v in variants:
            g = graphs[v]
            for _ in range(5):
                g.replay()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(40):
                g.replay()
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t) / 40 * 1e3)
    for v in variants:
        r = sorted(res[v])
        print(f"{v:30s} ms/fwd min {r[0]:.3f} median {r[len(r) // 2]:.3f}  ({B / r[len(r) // 2] * 1e3:.0f} img/s)",
              flush=True)


if __name__ == "__main__":
    main()
