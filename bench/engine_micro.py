"""Engine micro-benchmark: graph replay alone, H2D alone, and both overlapped (where does a step go?)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50  # noqa: E402
from aiforearth_api_platform_amd.runtime.engine import InferenceEngine  # noqa: E402


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    dev = torch.device("cuda:0")
    m = FusedResNet(resnet50(), device=dev)
    eng = InferenceEngine(m.forward_u8, (224, 224, 3), B, device=dev)
    eng.warmup()
    host = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8).pin_memory()
    g = eng.graphs[(0, B)]
    t_graph = timeit(lambda: g.replay())
    t_h2d = timeit(lambda: eng.inputs[0].copy_(host, non_blocking=True))
    s2 = torch.cuda.Stream()

    def both():
        with torch.cuda.stream(s2):
            eng.inputs[1].copy_(host, non_blocking=True)
        g.replay()

    t_both = timeit(both)
    t_submit = timeit(lambda: eng.submit(host, list(range(B))).done.synchronize())

    def pipelined():
        r = [eng.submit(host, list(range(B))) for _ in range(4)]
        r[-1].done.synchronize()

    t_pipe = timeit(pipelined, 5) / 4
    print(f"B={B} graph {t_graph:.3f} ms | h2d {t_h2d:.3f} ms ({B*224*224*3/t_h2d/1e6:.1f} GB/s) | "
          f"overlap {t_both:.3f} ms | submit+sync {t_submit:.3f} ms | pipelined/batch {t_pipe:.3f} ms")


if __name__ == "__main__":
    main()
