#!/bin/bash
# round 5z6: the final default tree (runner on): the GPU suite, smoke, the
# default bench line, the cfg5x replay
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05z6; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > $O/gputest.log 2>&1 || exit 11
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 12
timeout -k 10 600 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.log || exit 14
timeout -k 10 300 python3 -u bench.py --config cfg5x --steps 1 --warmup 0 --no-cpu-baseline > $O/cfg5x.json 2> $O/cfg5x.log || exit 15
