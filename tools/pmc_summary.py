#!/usr/bin/env python3
"""Per-kernel mean of rocprofv3 PMC counters (one row per kernel, one column
per counter), from every *counter_collection.csv under the given directories.

usage: tools/pmc_summary.py DIR [DIR ...] [--top N]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    top = 16
    if "--top" in sys.argv:
        top = int(sys.argv[sys.argv.index("--top") + 1])
        args = [a for a in args if a != str(top)]
    vals = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [per dispatch]
    for d in args:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(float)   # (dispatch, kernel, counter) -> summed over dims
            for r in csv.DictReader(open(path)):
                per[(r["Dispatch_Id"], r["Kernel_Name"], r["Counter_Name"])] += float(
                    r["Counter_Value"])
            for (_, k, c), v in per.items():
                vals[k][c].append(v)
    counters = sorted({c for k in vals for c in vals[k]})
    kern = sorted(vals, key=lambda k: -len(next(iter(vals[k].values()))))[:top]
    print("kernel," + ",".join(counters) + ",dispatches")
    for k in kern:
        row = [k.split("(")[0][:48]]
        n = 0
        for c in counters:
            v = vals[k].get(c)
            row.append(f"{sum(v) / len(v):.6g}" if v else "")
            n = max(n, len(v) if v else 0)
        print(",".join(row) + f",{n}")


if __name__ == "__main__":
    main()
