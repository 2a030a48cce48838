#!/bin/bash
# round 5z5: the whole GPU suite with the envelope runner on everywhere
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1 VLGBA_ENV_RUNNER=1
O=gpurun_out/r05z5; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > $O/gputest.log 2>&1 || exit 11
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 12
timeout -k 10 300 python3 -u bench.py --config ladybug --steps 20 --warmup 5 --no-cpu-baseline > $O/ladybug.log 2>&1 || exit 13
