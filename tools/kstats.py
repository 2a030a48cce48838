#!/usr/bin/env python3
"""Print a rocprofv3 kernel_stats.csv summary: name, calls, total ms, avg us."""
import csv
import sys

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 14
rows = list(csv.DictReader(open(path)))
for x in rows[:top]:
    print(f"{x['Name'][:52]:52s} {int(x['Calls']):6d} {float(x['TotalDurationNs'])/1e6:9.2f} ms "
          f"avg {float(x['AverageNs'])/1e3:9.2f} us  {float(x['Percentage']):5.1f}%")
