"""Does running the batch as S independent sub-batches on S streams (concurrent kernels fill the CUs a
single kernel's tile grid leaves idle) beat one stream? Eager and HIP-graph timings of FusedResNet."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B = int(os.environ.get("B", "256"))
    m = FusedResNet(resnet50(seed=0), device=dev)
    img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=dev)
    for split in (1, 2, 4):
        streams = [torch.cuda.Stream(device=dev) for _ in range(split)]

        def fwd():
            cur = torch.cuda.current_stream()
            outs = []
            for s, xc in zip(streams, img.chunk(split)):
                s.wait_stream(cur)
                with torch.cuda.stream(s):
                    outs.append(m.forward_u8(xc))
            for s in streams:
                cur.wait_stream(s)
            return outs

        for _ in range(3):
            fwd()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            fwd()
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t) / 10 * 1e3
        g = torch.cuda.CUDAGraph()
        s0 = torch.cuda.Stream(device=dev)
        s0.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s0):
            fwd()
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s0):
                fwd()
        torch.cuda.synchronize()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(20):
            g.replay()
        torch.cuda.synchronize()
        graph = (time.perf_counter() - t) / 20 * 1e3
        print(f"split {split}: eager {eager:.3f} ms  graph {graph:.3f} ms  ({B / graph * 1e3:.0f} img/s graph)", flush=True)


if __name__ == "__main__":
    main()
