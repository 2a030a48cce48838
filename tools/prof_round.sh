#!/bin/bash
# One round's profile evidence (GPU box, repo root): the cfg3 kernel trace +
# PMC passes (tools/profile_round.sh), the bench lines (tools/bench_lines.sh)
# and a ladybug kernel trace, all under gpurun_out/<TAG>_*.
# usage: tools/prof_round.sh TAG        (e.g. r03a)
set -o pipefail
export TMPDIR=/tmp
tag=${1:?usage: tools/prof_round.sh TAG}
bash tools/profile_round.sh "gpurun_out/${tag}_cfg3" --steps 10 --warmup 2 --no-cpu-baseline || exit $?
bash tools/bench_lines.sh "gpurun_out/${tag}_bench" || exit $?
mkdir -p "gpurun_out/${tag}_ladybug"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/${tag}_ladybug/trace" -o trace \
  --output-format csv -- python3 bench.py --config ladybug --steps 5 --warmup 1 --no-cpu-baseline \
  > "gpurun_out/${tag}_ladybug/trace.log" 2>&1
