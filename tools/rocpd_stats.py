#!/usr/bin/env python3
"""Kernel statistics (calls, total / average duration, share) from a rocprofv3
SQLite output (rocpd *.db: the default output format of ROCm 7.2's rocprofv3
when no --output-format is given) -- the same table as --stats'
kernel_stats.csv.  usage: tools/rocpd_stats.py RESULTS.db [top]"""
import collections
import sqlite3
import sys


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    c = sqlite3.connect(path)
    t = {r[0].split("_0000")[0]: r[0]
         for r in c.execute("select name from sqlite_master where type='table'")}
    names = {r[0]: r[1] for r in c.execute(
        f"select id, kernel_name from {t['rocpd_info_kernel_symbol']}")}
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for kid, s, e in c.execute(f"select kernel_id, start, end from {t['rocpd_kernel_dispatch']}"):
        nm = names.get(kid, str(kid)).split("(")[0].replace("void ", "")
        tot[nm] += e - s
        cnt[nm] += 1
    allns = sum(tot.values())
    print(f"{'Name':60s} {'Calls':>7s} {'Total ms':>10s} {'Avg us':>10s} {'%':>6s}")
    for nm in sorted(tot, key=lambda k: -tot[k])[:top]:
        print(f"{nm[:60]:60s} {cnt[nm]:7d} {tot[nm] / 1e6:10.3f} {tot[nm] / cnt[nm] / 1e3:10.2f} "
              f"{100 * tot[nm] / allns:6.1f}")


if __name__ == "__main__":
    main()
