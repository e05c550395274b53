"""The kernel sequence of the last traced training step (tools/step_profile.py
markers): one line per launch -- index, duration, short name -- so per-layer
costs of non-conv kernels (BatchNorm passes, pools) can be read off in issue order.
usage: python tools/trace_seq.py OUT/run_kernel_trace.csv > seq.txt"""
import csv
import re
import sys


def short(n):
    m = re.search(r"N12_GLOBAL__N_1\d+(\w+?)I", n) or re.search(r"namespace\)::(\w+)", n)
    return m.group(1) if m else n[:60]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "pinhole_z_fwd_kernel" in r["Kernel_Name"]]
    win = rows[marks[-2] + 1:marks[-1]]
    packs = [i for i, r in enumerate(win) if "pack_kernel" in r["Kernel_Name"]]
    if packs:   # (rounds <= 4: the step opened with the weight-packing launch)
        step = win[packs[-1]:]
    else:       # since round 5 the step ends with the AdamW launch that packs the weights
        opt = [i for i, r in enumerate(win) if "adamw" in r["Kernel_Name"]]
        step = win[opt[-2] + 1:opt[-1] + 1]
    for i, r in enumerate(step):
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
        print(f"{i:4d} {d:8.1f} {short(r['Kernel_Name'])} grid={r.get('Grid_Size', '')}")


if __name__ == "__main__":
    main()
