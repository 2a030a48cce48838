#!/bin/bash
# round-2 profile after the solve / plan work (GPU box, repo root)
set -o pipefail
export TMPDIR=/tmp
bash tools/profile_round.sh gpurun_out/r02c_cfg3 --steps 10 --warmup 2 --no-cpu-baseline || exit $?
bash tools/bench_r02.sh gpurun_out/r02c_bench
