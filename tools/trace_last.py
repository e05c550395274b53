"""Print the kernel sequence (duration, name) of the last `n` launches of a rocprofv3
kernel trace -- e.g. the last replay of a graph.  usage: trace_last.py TRACE.csv N"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2])
    ks = "Start_Timestamp" if "Start_Timestamp" in rows[0] else "Start"
    ke = "End_Timestamp" if "End_Timestamp" in rows[0] else "End"
    rows.sort(key=lambda r: int(r[ks]))
    tail = rows[-n:]
    tot = 0.0
    for i, r in enumerate(tail):
        d = (int(r[ke]) - int(r[ks])) * 1e-3
        tot += d
        name = r["Kernel_Name"]
        name = name.split("(")[0] if not name.startswith("_Z") else name[:60]
        print(f"{i:4d} {d:8.1f} us  grid={r.get('Grid_Size', '')}  {name[:90]}")
    span = (int(tail[-1][ke]) - int(tail[0][ks])) * 1e-3
    print(f"busy {tot:.1f} us, span {span:.1f} us")


if __name__ == "__main__":
    main()
