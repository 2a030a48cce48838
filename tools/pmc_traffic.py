#!/usr/bin/env python3
"""HBM traffic per kernel launch from separate rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE, kilobytes per dispatch), corrected as
/opt/skills/guides/MI355X_MICROARCH.md 'HBM' prescribes for gfx950:
FETCH_SIZE counts half of the bytes of wide coalesced streaming reads, so
it is doubled; WRITE_SIZE is taken as is.  Kernels are keyed by their base
name (template arguments and signature dropped).

With --valu DIR (a pass that collected SQ_INSTS_VALU) each kernel also gets
its VALU wave-instructions per dispatch ("valu_winst"), for the VALU-issue roof
bench.py reports beside the HBM one.

usage: tools/pmc_traffic.py FETCH_DIR WRITE_DIR [--valu DIR] [--config cfg3] > profiles/...json
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def per_dispatch(d, counter):
    vals = defaultdict(lambda: defaultdict(float))
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"]
            name = re.sub(r"^void ", "", name).split("(")[0].split("<")[0]
            vals[name][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in vals.items()}


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    cfg = sys.argv[sys.argv.index("--config") + 1] if "--config" in sys.argv else "cfg3"
    fetch = per_dispatch(fdir, "FETCH_SIZE")
    write = per_dispatch(wdir, "WRITE_SIZE")
    valu = per_dispatch(sys.argv[sys.argv.index("--valu") + 1], "SQ_INSTS_VALU") \
        if "--valu" in sys.argv else {}
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, 0.0), write.get(k, 0.0)
        out[k] = {"fetch_kb": f, "write_kb": w, "bytes": (2.0 * f + w) * 1024.0}
        if k in valu:
            out[k]["valu_winst"] = valu[k]
    json.dump({"config": cfg, "correction": "bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024",
               "kernels": out}, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main()
