#!/usr/bin/env python
"""Print the top kernels of a rocprofv3 kernel_stats.csv: name, calls, average / total us."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
for r in rows[:n]:
    name = r["Name"]
    name = name[name.find("k_"):] if "k_" in name else name
    print(f"{name[:58]:60s} calls={r['Calls']:>5} avg_us={float(r['AverageNs']) / 1e3:9.1f} "
          f"total_us={float(r['TotalDurationNs']) / 1e3:10.1f} pct={float(r['Percentage']):5.1f}")
