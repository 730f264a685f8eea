"""CU-partition probe (runtime/cu_partition.py): does a CU mask hold for eager launches and graph replays, what
is the mask-bit -> XCD layout, and how fast does the ResNet-50 serving forward run as a two-stage pipeline
(front = stem .. layer2 on F CUs, back = layer3 .. top-k on the other 256 - F) against the engine's default
(whole-forward graphs alternating over two full-chip streams)? Batch 250, 3 buffers, graph replay.

    python bench/cu_split_probe.py [F ...]
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50  # noqa: E402
from aiforearth_api_platform_amd.ops import _ext  # noqa: E402
from aiforearth_api_platform_amd.runtime import cu_partition as cup  # noqa: E402


def p(obj):
    print(json.dumps(obj), flush=True)


def pipeline_rate(run_batch, nb, warm=6):
    for k in range(warm):
        run_batch(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(warm, warm + nb):
        run_batch(k)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / nb * 1e3


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    _ext.lib()
    total = cup.cu_count(dev)
    # ---- 1. layout and mask checks
    full = torch.cuda.Stream(dev)
    p({"cus": total, "full_stream": cup.census(full)})
    xcc = cup.xcc_of_cus(dev)
    p({"layout": "blocked" if xcc[1] == xcc[0] else "interleaved", "xcc_of_first_16": xcc[:16]})
    half = cup.balanced(total // 2, xcc)
    sh = cup.masked_stream(half, dev)
    p({"half_mask_reported": len(cup.stream_mask(sh, total)), "half_eager": cup.census(sh)})
    out = torch.full((4096, 2), -1, dtype=torch.int32, device=dev)
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(dev)
    with torch.cuda.stream(cap):
        _ext.call("ai4e_cu_census", out.data_ptr(), 4096, 20000, cap.cuda_stream)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=cap):
            _ext.call("ai4e_cu_census", out.data_ptr(), 4096, 20000, cap.cuda_stream)
    with torch.cuda.stream(sh):
        out.fill_(-1)
        g.replay()
    sh.synchronize()
    o = out.cpu().tolist()
    p({"half_graph_replay_per_xcc": {x: sum(1 for r in o if r[0] == x) for x in range(8)},
       "half_graph_cu_slots": len({(r[0], (r[1] >> 8) & 0xFF) for r in o})})

    # ---- 2. ResNet-50 front/back graphs
    B = int(os.environ.get("B", "250"))
    m = FusedResNet(resnet50(seed=0), device=dev)
    assert m.can_split()
    nbuf = 3
    imgs = [torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=dev) for _ in range(nbuf)]
    cap = torch.cuda.Stream(dev)
    gf, gb, gfull, mids, outs = [], [], [], [], []
    with torch.cuda.stream(cap):
        for i in range(nbuf):  # eager warm-up (kernel load, tuning tables)
            m.back_topk(*m.front_u8(imgs[i]))
            m.topk_u8(imgs[i], 5)
        torch.cuda.synchronize()
        for i in range(nbuf):
            g1, g2, g3 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1, stream=cap):
                mid = m.front_u8(imgs[i])
            with torch.cuda.graph(g2, stream=cap):
                o = m.back_topk(*mid)
            with torch.cuda.graph(g3, stream=cap):
                o3 = m.topk_u8(imgs[i], 5)
            gf.append(g1); gb.append(g2); gfull.append(g3); mids.append(mid); outs.append((o, o3))
    torch.cuda.synchronize()
    nb = int(os.environ.get("NB", "60"))

    # baseline: the engine default (whole forward, batches alternating over two full-chip streams)
    s2 = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    done = {}

    def base(k):
        st = s2[k % 2]
        if k - nbuf in done:
            st.wait_event(done.pop(k - nbuf))
        with torch.cuda.stream(st):
            gfull[k % nbuf].replay()
        e = torch.cuda.Event()
        e.record(st)
        done[k] = e
    ms = pipeline_rate(base, nb)
    p({"mode": "2 full-chip streams, whole-forward graphs", "ms_per_batch": round(ms, 4),
       "images_per_s": round(B / ms * 1e3, 1)})

    def serial(stream, graphs):
        def run(k):
            with torch.cuda.stream(stream):
                graphs[k % nbuf].replay()
        return run
    p({"front_alone_full_ms": round(pipeline_rate(serial(full, gf), 20), 4),
       "back_alone_full_ms": round(pipeline_rate(serial(full, gb), 20), 4),
       "whole_forward_one_stream_ms": round(pipeline_rate(serial(full, gfull), 20), 4), "batch": B})

    fs = [int(a) for a in sys.argv[1:]] or ([] if os.environ.get("NO_SPLIT") else [96, 112, 128, 144, 160])
    for F in fs:
        for layout in (("balanced", "contiguous") if F == 128 else ("balanced",)):
            fcus = cup.balanced(F, xcc) if layout == "balanced" else list(range(F))
            bcus = [c for c in range(total) if c not in set(fcus)]
            sf, sb = cup.masked_stream(fcus, dev), cup.masked_stream(bcus, dev)
            evf, evb = {}, {}

            def split(k):
                if k - nbuf in evb:
                    sf.wait_event(evb.pop(k - nbuf))
                with torch.cuda.stream(sf):
                    gf[k % nbuf].replay()
                e = torch.cuda.Event()
                e.record(sf)
                sb.wait_event(e)
                with torch.cuda.stream(sb):
                    gb[k % nbuf].replay()
                e2 = torch.cuda.Event()
                e2.record(sb)
                evb[k] = e2
            ms = pipeline_rate(split, nb)
            p({"mode": "cu split", "layout": layout, "front_cus": F, "back_cus": total - F,
               "ms_per_batch": round(ms, 4), "images_per_s": round(B / ms * 1e3, 1),
               "front_alone_ms": round(pipeline_rate(serial(sf, gf), 20), 4),
               "back_alone_ms": round(pipeline_rate(serial(sb, gb), 20), 4)})
            torch.cuda.synchronize()
            for st in (sf, sb):
                _ext.call("ai4e_stream_destroy", st.cuda_stream)
    # correctness of the split path: same top-k as the whole-forward graph
    torch.cuda.synchronize()
    (oi, op), (ri, rp) = outs[0]
    p({"split_equals_full_topk": bool(torch.equal(oi, ri)), "max_prob_diff": (op - rp).abs().max().item()})


if __name__ == "__main__":
    main()
