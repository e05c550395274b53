"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:n]:
    name = r['Name']
    if name.startswith('_Z'):
        import subprocess
        name = subprocess.run(['c++filt', name], capture_output=True, text=True).stdout.strip()
    name = name.replace('(anonymous namespace)::', '')
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {int(r['Calls']):6d} x {float(r['AverageNs'])/1e3:8.1f} us {float(r['TotalDurationNs'])/tot*100:5.1f}%  {name[:100]}")
print('total ms', round(tot / 1e6, 2))
