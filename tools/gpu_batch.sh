#!/bin/bash
# One GPU-box call of several checks, each under its own time limit, stopping at
# the first failure (run from the repo root on the box):
#   ab     bit identity of the working tree's library against tools/build/ab/base
#          (tools/ab_build.sh base REV) on the long-track scenes (da_dump / da_compare)
#   tests  pytest -m gpu (the whole GPU suite) -> gpurun_out/gputest.log
#   cfg5x  bench.py --config cfg5x -> gpurun_out/bench_cfg5x.json
#   cfg3   bench.py (default) -> gpurun_out/bench_cfg3.json
# usage: tools/gpu_batch.sh step [step ...]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    ab)
      for sc in long "cfg5x 600"; do
        tag=${sc// /_}
        VLGBA_LIB=tools/build/ab/base/libvlgba.so timeout -k 10 300 python -u tools/da_dump.py \
          gpurun_out/ab_base_$tag.npz $sc > gpurun_out/ab_$tag.log 2>&1 &&
        timeout -k 10 300 python -u tools/da_dump.py gpurun_out/ab_new_$tag.npz $sc \
          >> gpurun_out/ab_$tag.log 2>&1 &&
        python tools/da_compare.py gpurun_out/ab_base_$tag.npz gpurun_out/ab_new_$tag.npz \
          | tee -a gpurun_out/ab_$tag.log || exit 1
      done ;;
    tests)
      timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 900 \
        --timeout-method thread > gpurun_out/gputest.log 2>&1; rc=$?
      tail -5 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc ;;
    cfg5x)
      timeout -k 10 600 python -u bench.py --config cfg5x > gpurun_out/bench_cfg5x.json \
        2> gpurun_out/bench_cfg5x.log || exit 1
      cat gpurun_out/bench_cfg5x.json ;;
    cfg3)
      timeout -k 10 600 python -u bench.py > gpurun_out/bench_cfg3.json \
        2> gpurun_out/bench_cfg3.log || exit 1
      cat gpurun_out/bench_cfg3.json ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
