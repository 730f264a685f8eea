"""Per-step kernel breakdown from a rocprofv3 kernel trace (one bench step = preprocess .. preprocess)."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "preprocess" in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
seg = rows[a:b]
span = (int(rows[b]["Start_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
print("step span us %.1f, kernels %d" % (span, len(seg)))
agg = collections.defaultdict(lambda: [0.0, 0])
for r in seg:
    n = r["Kernel_Name"]
    base = n.replace("(anonymous namespace)::", "")
    base = base[5:] if base.startswith("void ") else base
    k = base.split("(")[0]
    k = k.replace("(anonymous namespace)::", "")[:70]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg[k][0] += d
    agg[k][1] += 1
for k, (v, c) in sorted(agg.items(), key=lambda x: -x[1][0]):
    print("%8.1f us  %3d  %s" % (v, c, k))
if "-v" in sys.argv:
    for r in seg:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        print("%8.1f  grid %-8s %s" % (d, r["Grid_Size_X"], r["Kernel_Name"][:90]))
