"""Per-conv timing of ONE training step from a tools/step_profile.py kernel trace:
the conv launches of the last step in issue order, mapped onto the ResNet50 conv
list (forward order; backward in the trunk's reversed op order), next to the
per-conv roofline of tools/conv_roof.py.

    python tools/trace_layers.py OUT/run_kernel_trace.csv
"""
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_roof import resnet50_convs  # noqa: E402


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "pinhole_z_fwd_kernel" in r["Kernel_Name"]]
    win = rows[marks[-2] + 1:marks[-1]]
    # the last step of the window
    packs = [i for i, r in enumerate(win) if "pack_kernel" in r["Kernel_Name"]]
    if packs:   # (rounds <= 4: the step opened with the weight-packing launch)
        step = win[packs[-1]:]
    else:       # since round 5 the step ends with the AdamW launch that packs the weights
        opt = [i for i, r in enumerate(win) if "adamw" in r["Kernel_Name"]]
        step = win[opt[-2] + 1:opt[-1] + 1]
    conv = [r for r in step if any(k in r["Kernel_Name"] for k in ("conv_lds", "conv_igemm", "conv_bwd",
                                                                    "conv_wgrad_kernel", "conv_wgrad_lds"))]
    convs = resnet50_convs()
    B = 32
    fwd = conv[:len(convs)]
    bwd = conv[len(convs):]
    # backward issue order: reversed trunk ops -> per block: c3, c2, c1, ds
    order = []
    blocks = {}
    for c in convs[1:]:
        blocks.setdefault(c[0].rsplit(".", 1)[0], []).append(c)
    for blk in reversed(list(blocks.values())):
        names = {c[0].rsplit(".", 1)[1]: c for c in blk}
        for k in ("c3", "c2", "c1", "ds"):
            if k in names:
                order.append(names[k])
    order.append(convs[0])
    tot = [0.0, 0.0, 0.0, 0.0]
    print(f"{'conv':10s} {'fwd us':>8s} {'ideal':>6s} {'bwd us':>8s} {'ideal':>6s}  kernels")
    bmap = {c[0]: r for c, r in zip(order, bwd)}
    for c, r in zip(convs, fwd):
        n, H, ci, co, k, s, Ho = c
        M, K = B * Ho * Ho, k * k * ci
        f = 2 * M * co * K
        by = (B * H * H * ci + M * co + co * K) * 2
        ideal = max(f / 2.5e15, by / 6.3e12) * 1e6
        tf = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
        rb = bmap.get(n)
        tb = (int(rb["End_Timestamp"]) - int(rb["Start_Timestamp"])) * 1e-3 if rb else 0.0
        ideal_b = max(2 * f / 2.5e15, 2 * by / 6.3e12) * 1e6
        tot[0] += tf; tot[1] += ideal; tot[2] += tb; tot[3] += ideal_b
        kn = r["Kernel_Name"].split("(")[0][-40:]
        kb = rb["Kernel_Name"].split("(")[0][-30:] if rb else ""
        print(f"{n:10s} {tf:8.1f} {ideal:6.1f} {tb:8.1f} {ideal_b:6.1f}  {kn} | {kb}")
    print(f"{'total':10s} {tot[0]:8.1f} {tot[1]:6.1f} {tot[2]:8.1f} {tot[3]:6.1f}")


if __name__ == "__main__":
    main()
