#!/usr/bin/env python3
"""Per-kernel resources from a device assembly file (hipcc --cuda-device-only -S):
name, VGPRs, AGPRs, SGPRs, spills, scratch and static LDS bytes.

usage: tools/kres.py file.s [name-substring ...]
"""
import re
import sys

import yaml


def main():
    text = open(sys.argv[1]).read()
    m = re.search(r"\.amdgpu_metadata\n(.*?)\.end_amdgpu_metadata", text, re.S)
    meta = yaml.safe_load(m.group(1).replace("\t", "    "))
    pats = sys.argv[2:]
    for k in meta["amdhsa.kernels"]:
        name = k[".name"]
        if pats and not any(p in name for p in pats):
            continue
        print(f"{name[:60]:60s} vgpr {k['.vgpr_count']:3d} agpr {k.get('.agpr_count', 0):3d} "
              f"sgpr {k['.sgpr_count']:3d} spill v{k['.vgpr_spill_count']}/s{k['.sgpr_spill_count']} "
              f"scratch {k['.private_segment_fixed_size']} lds {k['.group_segment_fixed_size']}")


if __name__ == "__main__":
    main()
