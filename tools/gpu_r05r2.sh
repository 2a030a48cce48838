#!/bin/bash
# round 5r2: the envelope runner with per-row flags instead of launch-end flags
set -o pipefail
O=gpurun_out/r05r2; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_nd.py -x -v --timeout 120 --timeout-method thread > $O/tests_nd.log 2>&1 || exit 1
for r in 0 1 0 1; do
  VLGBA_ENV_RUNNER=$r timeout -k 10 200 python -u tools/pass_time.py 600 900 ladybug >> $O/pass_r$r.txt 2>&1 || exit 2
done
for r in 1 0; do
  VLGBA_ENV_RUNNER=$r timeout -k 10 300 python3 -u bench.py --config cfg5x --steps 1 --warmup 0 --no-cpu-baseline > $O/cfg5x_r$r.log 2>&1 || exit 3
done
