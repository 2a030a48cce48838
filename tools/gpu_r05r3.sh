#!/bin/bash
# round 5r3: the envelope runner in the cfg5x replay (many streams in one
# process): with the process-wide disable after a hand-off timeout, and with
# more hardware queues
set -o pipefail
O=gpurun_out/r05r3; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_nd.py -x -v -k runner --timeout 120 --timeout-method thread > $O/tests_runner.log 2>&1 || exit 11
VLGBA_ENV_RUNNER=1 timeout -k 10 300 python3 -u bench.py --config cfg5x --steps 1 --warmup 0 --no-cpu-baseline > $O/cfg5x_r1.log 2>&1 || exit 12
VLGBA_ENV_RUNNER=1 GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 -u bench.py --config cfg5x --steps 1 --warmup 0 --no-cpu-baseline > $O/cfg5x_r1_q8.log 2>&1 || exit 13
VLGBA_ENV_RUNNER=0 timeout -k 10 300 python3 -u bench.py --config cfg5x --steps 1 --warmup 0 --no-cpu-baseline > $O/cfg5x_r0.log 2>&1 || exit 14
