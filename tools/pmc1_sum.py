"""Summarise tools/pmc_one.sh output: per kernel symbol (matching a filter), the mean
per dispatch of every counter over all passes, plus derived per-wave fractions.
usage: python tools/pmc1_sum.py gpurun_out/pmc1_TAG [substring]"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import demangle  # noqa: E402


def main():
    root = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for (d, c), v in per.items():
            vals[demangle(names[d])][c].append(v)
    for k, cs in vals.items():
        if sub not in k:
            continue
        print(k[:110])
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        for c in sorted(m):
            print(f"   {c:34s} {m[c]:16.1f}")
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_LDS"):
                if c in m:
                    print(f"   {c + ' / wave cycles':48s} {m[c] / wc:6.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
            pass


if __name__ == "__main__":
    main()
