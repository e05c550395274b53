"""Sum rocprofv3 kernel-trace rows between the two pinhole_z_fwd markers of
tools/step_profile.py, per step: time per kernel symbol, its share, and the
wall span (first start .. last end) per step."""
import argparse
import collections
import csv


def short(name, n=90):
    return name if len(name) <= n else name[:n - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    key_s = "Start_Timestamp" if "Start_Timestamp" in rows[0] else "Start"
    key_e = "End_Timestamp" if "End_Timestamp" in rows[0] else "End"
    rows.sort(key=lambda r: int(r[key_s]))
    marks = [i for i, r in enumerate(rows) if "pinhole_z_fwd_kernel" in r["Kernel_Name"]]
    lo, hi = marks[-2], marks[-1]
    win = rows[lo + 1:hi]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in win:
        d = (int(r[key_e]) - int(r[key_s])) * 1e-3
        agg[r["Kernel_Name"]][0] += 1
        agg[r["Kernel_Name"]][1] += d
    busy = sum(v[1] for v in agg.values()) / a.steps
    span = (int(win[-1][key_e]) - int(win[0][key_s])) * 1e-3 / a.steps
    print(f"per step: wall span {span:8.1f} us, kernel busy {busy:8.1f} us, {len(win) / a.steps:.0f} launches")
    for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t / a.steps:9.1f} us {n / a.steps:6.1f}x {t / n:7.1f} us  {100 * t / a.steps / busy:5.1f}%  {short(name)}")


if __name__ == "__main__":
    main()
