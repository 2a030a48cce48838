"""Sum the [vlgba setup] phase lines (VLGBA_SETUP_TRACE=1) of a log: total
and mean per phase over every context the run created.
usage: python tools/setup_phase_sum.py LOG"""
import re
import sys
from collections import defaultdict

tot, cnt = defaultdict(float), defaultdict(int)
n = 0
for line in open(sys.argv[1], errors="replace"):
    if not line.startswith("[vlgba setup]"):
        continue
    n += 1
    for k, v in re.findall(r" (\w+)=(\d+)us", line):
        tot[k] += int(v)
        cnt[k] += 1
print(f"{n} contexts")
for k in sorted(tot, key=lambda k: -tot[k]):
    print(f"  {k:12s} total {tot[k] / 1e6:7.3f} s  mean {tot[k] / max(1, cnt[k]) / 1e3:7.3f} ms "
          f"({cnt[k]} contexts)")
print(f"  {'sum':12s} total {sum(tot.values()) / 1e6:7.3f} s")
