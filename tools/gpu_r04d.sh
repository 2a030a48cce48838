#!/bin/bash
# Round 4d checks on the GPU box (from the repo root): the CR timeline and the
# cfg3 bench, per-column envelope stamps, context-setup phases and the cfg5x
# replay with two prefetch workers.
# Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== cfg3 $(date +%T)"
timeout -k 10 200 python -u tools/cr_timeline.py cfg3 > gpurun_out/cr_timeline_base.txt 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_cfg3.json 2> gpurun_out/bench_cfg3.log || exit 1
echo "== stamps $(date +%T)"
VLGBA_LIB=bundleadjustmentmatlab_amd/libvlgba_stamps.so timeout -k 10 200 \
  python -u tools/step_stamps.py cfg5x:900 auto > gpurun_out/stamps_cfg5x900.txt 2>&1 || exit 1
echo "== setup $(date +%T)"
timeout -k 10 300 python -u tools/prof_cfg5x_setup.py 300 600 900 1000 > gpurun_out/setup_trace.log 2>&1 || exit 1
echo "== cfg5x $(date +%T)"
timeout -k 10 600 python -u bench.py --config cfg5x > gpurun_out/bench_cfg5x.json \
  2> gpurun_out/bench_cfg5x.log || exit 1
echo "== done $(date +%T)"
