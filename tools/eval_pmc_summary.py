"""Join rocprofv3 --pmc passes of tools/eval_pmc.py per launch position of the eval
forward (dispatches between the two pinhole_z_fwd markers, averaged over the reps).
    python tools/eval_pmc_summary.py DIR1 [DIR2 ...]   (each a --pmc pass output dir)"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import demangle  # noqa: E402


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return None, {}
    rows = list(csv.DictReader(open(f[0])))
    by = collections.OrderedDict()
    for r in rows:
        k = (int(r["Dispatch_Id"]), r["Kernel_Name"])
        by.setdefault(k, {})[r["Counter_Name"]] = float(r["Counter_Value"])
    seq = [(k[1], v) for k, v in sorted(by.items())]
    idx = [i for i, (n, _) in enumerate(seq) if "pinhole_z_fwd" in n]
    if len(idx) < 2:
        return None, {}
    win = seq[idx[0] + 1:idx[-1]]
    return win, set(c for _, v in win for c in v)


def main():
    passes = [load(d) for d in sys.argv[1:]]
    passes = [p for p in passes if p[0]]
    if not passes:
        print("no data")
        return
    n0 = len(passes[0][0])
    reps = int(os.environ.get("REPS", "3"))
    per = n0 // reps
    cols = []
    for win, names in passes:
        cols += sorted(names)
    print("pos kernel " + " ".join(cols))
    for i in range(per):
        vals = {}
        name = passes[0][0][i][0]
        for win, names in passes:
            for c in names:
                vals[c] = sum(win[r * per + i][1].get(c, 0.0) for r in range(reps)) / reps
        print(f"{i:3d} {demangle(name)[:60]:60s} " + " ".join(f"{vals[c]:.4g}" for c in cols))


if __name__ == "__main__":
    main()
