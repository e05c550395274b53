"""Per-kernel in-step averages from a rocprofv3 --kernel-trace of bench.py's replayed
step (rocpd .db or kernel_trace.csv): the step windows are the kernels between two
adamw launches (the step's last kernel); averages over the last K windows.
usage: python tools/trace_summary.py PROF_DIR [K] > profiles/<tag>_step_trace.txt"""
import csv
import glob
import os
import sqlite3
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "6d-pose-estimation_amd")]
from pose6d.steptime import short_name  # noqa: E402


def load(d):
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    if dbs:
        c = sqlite3.connect(dbs[0])
        return [(n, s, e) for n, s, e in c.execute("select name, start, end from kernels order by start")]
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(f))]
    return sorted(rows, key=lambda r: r[1])


def name(n):
    if n.startswith("_Z"):
        return short_name(n.encode())
    n = n.replace("(anonymous namespace)::", "")
    n = n[5:] if n.startswith("void ") else n
    depth = 0
    for i, ch in enumerate(n):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return n[:i]
    return n


def main():
    rows = load(sys.argv[1])
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ends = [i for i, r in enumerate(rows) if "adamw" in r[0]]
    wins = list(zip(ends[-k - 1:-1], ends[-k:]))
    per = {}
    walls = []
    for a, b in wins:
        seg = rows[a + 1:b + 1]
        walls.append((seg[-1][2] - seg[0][1]) / 1e3)
        for n, s, e in seg:
            per.setdefault(name(n), []).append((e - s) / 1e3)
    nk = (wins[0][1] - wins[0][0])
    print(f"# rocprofv3 kernel trace, last {len(wins)} step windows (between adamw launches): {nk} kernels/step, "
          f"step wall {statistics.mean(walls):.1f} us")
    print(f"# {'kernel':60s} {'launches/step':>13s} {'avg us':>8s} {'median us':>9s} {'ms/step':>8s}")
    for n, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"{n[:62]:62s} {len(d) / len(wins):13.1f} {statistics.mean(d):8.2f} {statistics.median(d):9.2f} "
              f"{sum(d) / len(wins) / 1e3:8.3f}")


if __name__ == "__main__":
    main()
