#!/bin/bash
# round 5z7: kernel trace of the ladybug pass bench with the envelope runner
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05z7; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python3 bench.py --config ladybug --steps 10 --warmup 3 --no-cpu-baseline > $O/trace.log 2>&1 || exit 11
