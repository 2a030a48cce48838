#!/usr/bin/env python3
"""Per-pass kernel timeline from a rocprofv3 kernel trace (tools/trace_pass.sh):
the last pass of the bench's untimed loop -- each kernel's start offset,
duration and the idle gap before it on the device.
usage: python tools/timeline.py gpurun_out/trace_pass [first_kernel_substring]"""
import csv
import glob
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/trace_pass"
first = sys.argv[2] if len(sys.argv) > 2 else "k_linearize_chunk"
f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
# passes = linearize .. next linearize; take the second-to-last complete pass
a, b = starts[-3], starts[-2]
t0 = int(rows[a]["Start_Timestamp"])
busy_end = t0
tot_gap = 0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = max(0, s - busy_end)
    tot_gap += gap
    busy_end = max(busy_end, e)
    name = r["Kernel_Name"].split("(")[0][:40]
    print(f"{(s - t0) / 1e3:8.1f} us  +{(e - s) / 1e3:7.1f} us  gap {gap / 1e3:5.1f}  {name}")
print(f"pass {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us, idle gaps {tot_gap / 1e3:.1f} us")
