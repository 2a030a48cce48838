#!/bin/bash
# round 5u: grouped k_factor_multi workgroup order -- ND tests, stamps and
# per-pass times on cfg5x-900 with the grouped and the arc-major order
set -o pipefail
O=gpurun_out/r05u; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_nd.py -x -v --timeout 120 --timeout-method thread > $O/nd_tests.log 2>&1 || exit 1
for g in 1 0; do
  VLGBA_ND_GROUPED=$g VLGBA_LIB=tools/build/ab/stamps/libvlgba.so timeout -k 10 200 python -u tools/step_stamps.py cfg5x:900 > $O/stamps_g$g.txt 2>&1 || exit 2
done
for g in 1 0 1 0; do
  VLGBA_ND_GROUPED=$g timeout -k 10 200 python -u tools/prof_cfg5x_solve.py 900 >> $O/solve_g$g.txt 2>&1 || exit 3
done
VLGBA_ND_GROUPED=1 VLGBA_LIB=tools/build/ab/stamps/libvlgba.so timeout -k 10 200 python -u tools/step_stamps.py ladybug > $O/stamps_ladybug.txt 2>&1 || exit 4
