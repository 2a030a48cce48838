#!/bin/bash
# round-2h profile (GPU box, repo root): cfg3 trace + PMC passes, the
# bench lines, a ladybug kernel trace
set -o pipefail
export TMPDIR=/tmp
bash tools/profile_round.sh gpurun_out/r02h_cfg3 --steps 10 --warmup 2 --no-cpu-baseline || exit $?
bash tools/bench_r02.sh gpurun_out/r02h_bench || exit $?
mkdir -p gpurun_out/r02h_ladybug
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02h_ladybug/trace -o trace \
  --output-format csv -- python3 bench.py --config ladybug --steps 5 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r02h_ladybug/trace.log 2>&1
