#!/bin/bash
# round 5r: the envelope runner (VLGBA_ENV_RUNNER=1) -- bit identity against
# the column launches alone, untimed pass times with and without
set -o pipefail
O=gpurun_out/r05r; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_nd.py -x -v -k "runner" --timeout 120 --timeout-method thread > $O/tests_runner.log 2>&1 || exit 1
for r in 0 1 0 1; do
  VLGBA_ENV_RUNNER=$r timeout -k 10 200 python -u tools/pass_time.py 600 900 ladybug >> $O/pass_r$r.txt 2>&1 || exit 2
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_nd.py -x -q --timeout 120 --timeout-method thread > $O/tests_nd.log 2>&1 || exit 3
