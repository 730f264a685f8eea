"""How busy and how concurrent is the GPU while serving?  From a rocprofv3 kernel trace of bench.py
(``rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_serve -o serve -- python bench.py --steps 200``):

* window: from the ``--skip``-th to the last-but-``--tail`` preprocess launch (steady state, no capture/warmup);
* busy: union of kernel intervals / window; idle gaps histogram;
* concurrency: time with 0 / 1 / 2 / 3+ kernels resident, mean concurrency over the busy time;
* per kernel family: summed duration per step, and how much of it overlapped another kernel.

    python tools/concurrency.py gpurun_out/prof_serve/serve_kernel_trace.csv [--skip 30 --tail 5]
"""
import argparse
import collections
import csv


def short(n: str) -> str:
    n = n.replace("(anonymous namespace)::", "")
    n = n[5:] if n.startswith("void ") else n
    return n.split("(")[0][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=30)
    ap.add_argument("--tail", type=int, default=5)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    pre = [s for s, _, n in ks if "preprocess" in n]
    pre = pre[a.skip:len(pre) - a.tail]
    spans = sorted(b - a_ for a_, b in zip(pre, pre[1:]))
    med = spans[len(spans) // 2]
    # steady-state steps only: a step (preprocess to preprocess) longer than 2x the median is a pause (capture,
    # REST phase, ...) and is left out
    steps = [(x, y) for x, y in zip(pre, pre[1:]) if y - x <= 2 * med]
    at = collections.Counter()
    gaps, total, span = [], 0, 0
    fam = collections.defaultdict(float)
    j0 = 0
    for t0, t1 in steps:
        while j0 < len(ks) and ks[j0][1] <= t0 - 50_000_000:  # kernels are shorter than 50 ms
            j0 += 1
        win = []
        for s_, e_, n in ks[j0:]:
            if s_ >= t1:
                break
            if e_ > t0:
                win.append((max(s_, t0), min(e_, t1), n))
        ev = sorted([(x, 1) for x, _, _ in win] + [(y, -1) for _, y, _ in win])
        level, last = 0, t0
        for t, d in ev:
            if t > last:
                at[min(level, 3)] += t - last
                if level == 0:
                    gaps.append(t - last)
            level += d
            last = t
        if t1 > last:
            at[0] += t1 - last
        span += t1 - t0
        for x, y, n in win:
            total += y - x
            fam[short(n)] += y - x
    busy = span - at[0]
    n = len(steps)
    print(f"{n} steady-state steps (median step {med / 1e3:.1f} us), {span / 1e6:.2f} ms")
    print(f"busy {100 * busy / span:.1f} %  | idle {at[0] / 1e3 / n:.1f} us/step in {len(gaps) / n:.1f} gaps/step "
          f"(p50 {sorted(gaps)[len(gaps) // 2] / 1e3 if gaps else 0:.1f} us)")
    print(f"time at 1 kernel {100 * at[1] / span:.1f} %, 2 kernels {100 * at[2] / span:.1f} %, 3+ {100 * at[3] / span:.1f} %;"
          f" mean concurrency while busy {total / busy:.2f}")
    print(f"kernel time per step (sum of durations) {total / 1e3 / n:.1f} us")
    steps = n
    print(f"{'us/step':>8}  kernel")
    for k, v in sorted(fam.items(), key=lambda x: -x[1])[:25]:
        print(f"{v / 1e3 / steps:8.1f}  {k}")


if __name__ == "__main__":
    main()
