"""Attribute a rocprofv3 kernel trace of the ResNet-50 forward to layers (one forward = last N dispatches)."""
import csv
import sys

sys.path.insert(0, ".")


def main(path, batch=256, size=224):
    from aiforearth_api_platform_amd.models.resnet import FusedResNet, resnet50
    rows = [r for r in csv.DictReader(open(path)) if r["Kind"] == "KERNEL_DISPATCH"]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    convs = [r for r in rows if "conv_igemm" in r["Kernel_Name"]]
    m = FusedResNet(resnet50())
    layers = m.layers()
    n = len(layers)
    last = convs[-n:]
    # replay shapes
    h = w = size
    shapes = []
    h, w = m.stem.out_hw(h // 2, w // 2); shapes.append(("stem", m.stem, size // 2, size // 2)); h, w = (h + 1) // 2, (w + 1) // 2
    for bi, (c1, c2, c3, d) in enumerate(m.blocks):
        if d is not None:
            shapes.append((f"b{bi}.down", d, h, w))
        shapes.append((f"b{bi}.c1", c1, h, w)); shapes.append((f"b{bi}.c2", c2, h, w))
        h2, w2 = c2.out_hw(h, w); shapes.append((f"b{bi}.c3", c3, h2, w2)); h, w = h2, w2
    shapes.append(("fc", m.fc, 1, 1))
    tot = 0
    agg = {}
    for (name, pc, hh, ww), r in zip(shapes, last):
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        oh, ow = pc.out_hw(hh, ww)
        fl = 2 * batch * oh * ow * pc.cout * pc.kh * pc.kw * pc.cin
        by = 2 * batch * (hh * ww * pc.cin_pad + oh * ow * pc.cout * (2 if name.endswith("c3") else 1))
        tot += us
        key = f"{pc.kh}x{pc.kw}/s{pc.stride} {pc.cin_pad}->{pc.cout} @{hh}"
        a = agg.setdefault(key, [0, 0.0, fl, by])
        a[0] += 1; a[1] += us
    print(f"{'layer shape':34s} {'n':>3s} {'us/call':>9s} {'TFLOPs':>7s} {'TB/s':>6s} {'sum_us':>8s}")
    for k, (cnt, us, fl, by) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:34s} {cnt:3d} {us / cnt:9.1f} {fl / (us / cnt) / 1e6:7.1f} {by / (us / cnt) / 1e6:6.2f} {us:8.1f}")
    print("conv total us", round(tot, 1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 256)
