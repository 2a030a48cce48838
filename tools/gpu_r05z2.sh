#!/bin/bash
# round 5z: final validation, part 2 -- the default bench line, its rocprofv3
# kernel-trace --stats, a per-pass timeline, the cfg5x replay line
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05z2; mkdir -p $O
timeout -k 10 600 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-other-configs > $O/trace.log 2>&1 || exit 2
python3 tools/timeline.py $O/trace k_update_linearize > $O/timeline.txt 2>&1
timeout -k 10 600 python3 -u bench.py --config cfg5x > $O/bench_cfg5x.json 2> $O/bench_cfg5x.log || exit 3
