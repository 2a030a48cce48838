#!/bin/bash
# round 5z8: the runner's minimum run length (VLGBA_ENV_RUNNER_MIN) on untimed passes
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05z8; mkdir -p $O
for m in 1 4 8 16 1000; do
  VLGBA_ENV_RUNNER_MIN=$m timeout -k 10 200 python -u tools/pass_time.py 300 600 900 ladybug > $O/pass_min$m.txt 2>&1 || exit 11
done
