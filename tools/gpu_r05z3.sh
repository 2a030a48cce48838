#!/bin/bash
# round 5z3: final validation after the envelope-runner change (runner off by
# default): the whole GPU suite, smoke, cfg5x-900 kernel times, the default bench
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05z3; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > $O/gputest.log 2>&1 || exit 11
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 12
timeout -k 10 200 python -u tools/prof_cfg5x_solve.py 900 > $O/solve_900.txt 2>&1 || exit 13
timeout -k 10 600 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.log || exit 14
