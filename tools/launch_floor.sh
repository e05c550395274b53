set -e
mkdir -p gpurun_out/lf
timeout -k 10 120 python3 tools/launch_floor.py > gpurun_out/lf/plain.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/lf/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/launch_floor.py > $GRAFT_REPO_ROOT/gpurun_out/lf/prof.txt 2>&1
cd $GRAFT_REPO_ROOT
S=$(ls gpurun_out/lf/prof/*/run_kernel_stats.csv gpurun_out/lf/prof/run_kernel_stats.csv 2>/dev/null | head -1)
cp $S gpurun_out/lf/stats.csv
T=$(ls gpurun_out/lf/prof/*/run_kernel_trace.csv gpurun_out/lf/prof/run_kernel_trace.csv 2>/dev/null | head -1)
python3 - "$T" > gpurun_out/lf/durs.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    d[(r["Kernel_Name"][:60], int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in d.items():
    v.sort()
    print(len(v), k, "min %.2f med %.2f" % (v[0], v[len(v) // 2]))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(rows, rows[1:])]
gaps.sort()
print("gap start-to-prev-end: med %.2f p10 %.2f p90 %.2f" % (gaps[len(gaps)//2], gaps[len(gaps)//10], gaps[9*len(gaps)//10]))
PY
rm -rf gpurun_out/lf/prof
