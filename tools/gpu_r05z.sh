#!/bin/bash
# round 5z: final validation, part 1 -- bit identity against the round's start
# (tools/build/ab/base = 53419a9) on the long-track scenes, the whole GPU
# suite, smoke()
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash tools/gpu_batch.sh ab tests || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit 2
