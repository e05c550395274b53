"""Ordered kernel list of ONE step between the step_profile markers: duration,
gap before it, grid, LDS and a short name (for per-layer attribution)."""
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(anonymous namespace\)::|_ZN12_GLOBAL__N_1\d*", "", n)
    n = re.sub(r"\(.*", "", n)
    return n[:60]


rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "pinhole_z_fwd_kernel" in r["Kernel_Name"]]
win = rows[marks[-2] + 1:marks[-1]]
per = len(win) // steps
step = win[-per:]
prev = None
for r in step:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    prev = e
    grid = int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1)
    print(f"{(e - s) / 1e3:8.1f} {gap:6.1f}  g={grid:6d}x{r['Grid_Size_Y']:>4}  lds={r['LDS_Block_Size']:>6}  "
          f"{short(r['Kernel_Name'])}")
