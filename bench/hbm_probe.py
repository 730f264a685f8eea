"""HBM rate probe: what the chip sustains for the access mixes the ResNet kernels use — read-only (sum),
write-only (fill), copy (read + write, 1:1) and read-2 / write-1 — on bf16 tensors of ResNet activation size
(batch 250: 100 MB, 400 MB), one stream and two streams at once. Numbers are bytes moved by the kernel's
definition (not PMC), per second.

    python bench/hbm_probe.py
"""
import json

import torch


def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e-3  # s


def main():
    dev = "cuda"
    out = []
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for mb in (100, 400):
        n = mb * (1 << 20) // 2
        x = [torch.randn(n, device=dev).bfloat16() for _ in range(2)]
        y = [torch.empty(n, device=dev, dtype=torch.bfloat16) for _ in range(2)]
        z = [torch.randn(n, device=dev).bfloat16() for _ in range(2)]
        nb = n * 2
        cases = {
            "read": (lambda i: x[i].sum(), nb),
            "write": (lambda i: y[i].fill_(1.0), nb),
            "copy": (lambda i: y[i].copy_(x[i]), 2 * nb),
            "add_r2w1": (lambda i: torch.add(x[i], z[i], out=y[i]), 3 * nb),
        }
        for name, (fn, byts) in cases.items():
            t1 = timed(lambda: fn(0))

            def two():
                cur = torch.cuda.current_stream()
                s1.wait_stream(cur)
                s2.wait_stream(cur)
                with torch.cuda.stream(s1):
                    fn(0)
                with torch.cuda.stream(s2):
                    fn(1)
                cur.wait_stream(s1)
                cur.wait_stream(s2)
            t2 = timed(two)
            out.append({"MB": mb, "op": name, "TBps_1stream": round(byts / t1 / 1e12, 2),
                        "TBps_2streams": round(2 * byts / t2 / 1e12, 2), "us": round(t1 * 1e6, 1)})
            print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
