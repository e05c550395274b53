"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time."""
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import demangle  # noqa: E402

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:n]:
    name = demangle(r['Name'])
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {int(r['Calls']):6d} x {float(r['AverageNs'])/1e3:8.1f} us "
          f"{float(r['TotalDurationNs'])/tot*100:5.1f}%  {name[:100]}")
print('total ms', round(tot / 1e6, 2))
