"""In-process A/B of the U-Net forward (16 tiles of 512^2, the config-4 tile batch) with HIP-graph replays, variants
interleaved over rounds in ONE process (cdna guide §5.4 rule 24). Variant "base" is the shipped code; "no256stats"
takes the 256-wide K1 configs' fused GroupNorm statistics away again (the round-4 behaviour: those GroupNorms run
their own statistics pass). (Round 5 also measured the decoder
GroupNorm folded into the upsample and a raw level-1 skip with this script: neutral, see profiles/r5_pruned/.)

    python bench/unet_forward_ab.py [rounds 6] [replays 10]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from aiforearth_api_platform_amd.models.unet import FusedUNet, unet_landcover  # noqa: E402
from aiforearth_api_platform_amd.ops import conv as convmod  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dev = torch.device("cuda:0")
model = unet_landcover(seed=0)
net = FusedUNet(model, device=dev)
x = torch.randint(0, 256, (16, 512, 512, 4), dtype=torch.uint8, device=dev)
orig = convmod.conv2d_gn_nhwc


def no256(xx, pc, groups, out=None, out_coff=0):
    n, h, w, _ = xx.shape
    if convmod.tuned_tile(pc, n, h, w, False) in (6, 9, 10):
        return convmod.conv2d_nhwc(xx, pc, out=out, out_coff=out_coff), None
    return orig(xx, pc, groups, out=out, out_coff=out_coff)


import aiforearth_api_platform_amd.models.unet as unetmod  # noqa: E402

variants = {"base": (orig, net), "no256stats": (no256, net)}
graphs = {}
for name, (fn, nn_) in variants.items():
    unetmod.conv2d_gn_nhwc = fn
    for _ in range(2):
        nn_.forward_u8(x)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        nn_.forward_u8(x)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        out = nn_.forward_u8(x)
    torch.cuda.synchronize()
    graphs[name] = (g, out)
unetmod.conv2d_gn_nhwc = orig
graphs["base"][0].replay()  # (capture runs nothing: replay before reading an output)
torch.cuda.synchronize()
ref = graphs["base"][1].clone()
err = {}
for k in ("no256stats",):
    graphs[k][0].replay()
    torch.cuda.synchronize()
    err[k] = (graphs[k][1].float() - ref.float()).abs().max().item()
res = {k: [] for k in graphs}
for r in range(rounds):
    for name, (g, _) in graphs.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        g.replay()
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        res[name].append(e0.elapsed_time(e1) / reps)
print(json.dumps({"ms_per_forward_16_tiles": {k: sorted(round(v, 4) for v in vs) for k, vs in res.items()},
                  "median": {k: round(sorted(vs)[len(vs) // 2], 4) for k, vs in res.items()},
                  "max_abs_diff_logits": err}))
