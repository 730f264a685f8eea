"""Per-dispatch PMC summary of one eager ResNet-50 forward (tools/pmc_resnet.sh output).

    python tools/pmc_summary.py gpurun_out/pmc [> profiles/.../pmc_summary.txt]
    python tools/pmc_summary.py gpurun_out/pmc_detector --start spin_kernel --by-kernel

``--start NAME``: the forward begins after the last dispatch whose name contains NAME (default: at the last
``preprocess`` launch); ``--by-kernel``: one line per kernel name (summed over its dispatches, sorted by time).

Joins the counter passes by dispatch order (the profiled program is deterministic), keeps the last
forward (from the last preprocess launch on), and prints per dispatch: duration, MFMA busy fraction
(SQ_VALU_MFMA_BUSY_CYCLES over the SIMD-cycles the kernel spanned), HBM-side bytes (FETCH_SIZE + WRITE_SIZE,
KiB counters) and the resulting bandwidth, L2 hit rate, LDS bank-conflict share and wave-wait share.
"""
import collections
import csv
import glob
import os
import sys

CUS, SIMDS, CLK_GHZ = 256, 4, 2.4


def load(path):
    by = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        d = by.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"]),
                                                  "t": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return list(by.values())


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    n = n[5:] if n.startswith("void ") else n
    return n.split("(")[0][:44]


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("dir", nargs="?", default="gpurun_out/pmc")
    ap.add_argument("--start", default="")
    ap.add_argument("--by-kernel", action="store_true")
    a = ap.parse_args()
    d = a.dir
    passes = [load(p) for p in sorted(glob.glob(os.path.join(d, "pass*_counter_collection.csv")))]
    n = min(len(p) for p in passes)
    rows = []
    for i in range(n):
        r = {}
        for p in passes:
            r.update({k: v for k, v in p[i].items() if k not in r or k not in ("t",)})
        r["t"] = min(p[i]["t"] for p in passes)
        rows.append(r)
    if a.start:
        seg = rows[[i for i, r in enumerate(rows) if a.start in r["name"]][-1] + 1:]
    else:
        seg = rows[[i for i, r in enumerate(rows) if "preprocess" in r["name"]][-1]:]
    if a.by_kernel:
        agg = collections.OrderedDict()
        for r in seg:
            k = short(r["name"])
            g = agg.setdefault(k, {"name": r["name"], "grid": r["grid"], "t": 0.0, "n": 0})
            g["n"] += 1
            for key, v in r.items():
                if key not in ("name", "grid"):
                    g[key] = g.get(key, 0.0) + v if key != "n" else g[key]
        seg = sorted(agg.values(), key=lambda g: -g["t"])
    print(f"{'us':>7} {'mfma%':>6} {'HBM MB':>8} {'TB/s':>5} {'L2hit%':>6} {'ldsconf%':>8} {'wait%':>6}  kernel")
    tot_t = tot_b = 0.0
    for r in seg:
        t = r["t"]
        span_simd_cycles = t * 1e-6 * CLK_GHZ * 1e9 * CUS * SIMDS
        mfma = 100 * r.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / span_simd_cycles if t else 0
        b = (r.get("FETCH_SIZE", 0) + r.get("WRITE_SIZE", 0)) * 1024
        hit = r.get("TCC_HIT_sum", 0)
        miss = r.get("TCC_MISS_sum", 0)
        lds = r.get("SQ_LDS_IDX_ACTIVE", 0)
        conf = 100 * r.get("SQ_LDS_BANK_CONFLICT", 0) / lds if lds else 0
        wc = r.get("SQ_WAVE_CYCLES", 0)
        wait = 100 * r.get("SQ_WAIT_ANY", 0) / wc if wc else 0
        tot_t += t
        tot_b += b
        print(f"{t:7.1f} {mfma:6.1f} {b / 1e6:8.1f} {b / t / 1e6 if t else 0:5.2f} "
              f"{100 * hit / (hit + miss) if hit + miss else 0:6.1f} {conf:8.1f} {wait:6.1f}  {short(r['name'])} "
              + (f"x{r['n']}" if a.by_kernel else f"g{r['grid']}"))
    print(f"total {tot_t:.1f} us, {tot_b / 1e9:.2f} GB HBM-side")


if __name__ == "__main__":
    main()
