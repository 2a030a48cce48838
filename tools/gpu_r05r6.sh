#!/bin/bash
# round 5r6: runner threshold 8 columns, one runner stream per device
set -o pipefail
O=gpurun_out/r05r6; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_nd.py -x -v -k runner --timeout 120 --timeout-method thread > $O/tests_runner.log 2>&1 || exit 11
VLGBA_ENV_RUNNER=1 timeout -k 10 200 python -u tools/pass_time.py 600 900 ladybug > $O/pass_r1.txt 2>&1 || exit 12
VLGBA_ENV_RUNNER=1 timeout -k 10 300 python3 -u bench.py --config cfg5x --steps 1 --warmup 0 --no-cpu-baseline > $O/cfg5x_r1.log 2>&1 || exit 13
VLGBA_ENV_RUNNER=0 timeout -k 10 300 python3 -u bench.py --config cfg5x --steps 1 --warmup 0 --no-cpu-baseline > $O/cfg5x_r0.log 2>&1 || exit 14
VLGBA_ENV_RUNNER=1 timeout -k 10 300 python3 -u bench.py --config ladybug --steps 20 --warmup 5 --no-cpu-baseline > $O/ladybug_r1.log 2>&1 || exit 15
VLGBA_ENV_RUNNER=0 timeout -k 10 300 python3 -u bench.py --config ladybug --steps 20 --warmup 5 --no-cpu-baseline > $O/ladybug_r0.log 2>&1 || exit 16
