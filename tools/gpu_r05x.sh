#!/bin/bash
# round 5x: pivot-chain factor variants (tools/ubench_f16v.hip) + a cfg3 pass line
set -o pipefail
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 60 tools/build/ubench_f16v > $O/ubench_f16v.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-other-configs > $O/bench_cfg3.log 2>&1 || exit 2
