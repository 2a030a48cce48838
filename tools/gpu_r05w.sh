#!/bin/bash
# round 5w: k_schur_long_acc default, trailing-workgroup cap sweep at
# cfg5x-900, the cfg5x replay and ladybug with the new defaults
set -o pipefail
O=gpurun_out/r05w; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_long_acc.py tests/test_gpu_nd.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for c in 0 320 384 448 512 0 320 384 448 512; do
  VLGBA_TRAIL_WGS=$c timeout -k 10 200 python -u tools/prof_cfg5x_solve.py 600 900 >> $O/solve_t$c.txt 2>&1 || exit 2
done
for c in 0 384; do
  VLGBA_TRAIL_WGS=$c timeout -k 10 300 python3 -u bench.py --config ladybug --steps 10 --warmup 2 --no-cpu-baseline > $O/ladybug_t$c.log 2>&1 || exit 3
done
timeout -k 10 600 python3 -u bench.py --config cfg5x --steps 1 --warmup 0 --no-cpu-baseline > $O/cfg5x.log 2>&1 || exit 4
